#!/usr/bin/env python3
"""What the SST device forms cost over the plain batch form on the same blocks (round 5): per-call time, 20 calls per
hipGraph replay, of kvsep_crc32c_batch_device, kvsep_sst_trailers_device (the CRC kernel + the trailer-word kernel) and
kvsep_sst_verify_device (the prep kernel + the CRC kernel's verify form, on an intact image and on one whose every
trailer is wrong) over 65,536 blocks of 4 KiB (config 2's SST
blocks, table/table_builder.cc:209-232 / table/format.cc:99-108).  usage: sst_cost_probe.py [count]"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import kvsep  # noqa: E402

dev = torch.device("cuda:0")
count = int(sys.argv[1]) if len(sys.argv) > 1 else 65536
blk = 4096
stride = blk + 5  # a file image: [block][type][trailer word]
span = count * stride
img = torch.empty(span + 64, dtype=torch.uint8, device=dev)
kvsep.fill_splitmix64(img.data_ptr(), span, 9, 0)
off = (np.arange(count, dtype=np.uint64) * np.uint64(stride))
ln = np.full(count, blk, np.uint64)
d_off = torch.from_numpy(off.view(np.int64)).to(dev)
d_len = torch.from_numpy(ln.view(np.int64)).to(dev)
types = torch.zeros(count, dtype=torch.uint8, device=dev)
out = torch.zeros(count, dtype=torch.int32, device=dev)
fb = torch.zeros(1, dtype=torch.int64, device=dev)
nb = torch.zeros(1, dtype=torch.int64, device=dev)
ctx = kvsep.Context(0)
ctx.reserve(count, count * (blk + 1))
total = count * blk
# a well-formed file image: each block followed by its type byte (0) and the trailer word the writer would store
ctx.sst_trailers_device(img.data_ptr(), d_off, d_len, types, out, count=count, total_bytes=total, max_len=blk)
torch.cuda.synchronize()
h = img.cpu().numpy()
words = out.cpu().numpy().view(np.uint32)
for k in range(5):
    h[off.astype(np.int64) + blk + k] = 0 if k == 0 else ((words >> np.uint32(8 * (k - 1))) & np.uint32(255)).astype(np.uint8)
img.copy_(torch.from_numpy(h))
ctx.sst_verify_device(img.data_ptr(), d_off, d_len, out, fb, nb, count=count, total_bytes=total, max_len=blk)
torch.cuda.synchronize()
assert int(fb.item()) == -1 and int(nb.item()) == 0, (int(fb.item()), int(nb.item()))  # every trailer intact
bad = img.clone()  # the same image with every trailer word wrong (a torn or garbage file: every block mismatches)
bh = bad.cpu().numpy()
bh[off.astype(np.int64) + blk + 1] ^= 1
bad.copy_(torch.from_numpy(bh))
cs = lambda: torch.cuda.current_stream()  # noqa: E731
forms = {
    "batch": lambda: ctx.batch_device(img.data_ptr(), d_off, d_len, out, count=count, total_bytes=total, max_len=blk,
                                      stream=cs()),
    "sst_trailers": lambda: ctx.sst_trailers_device(img.data_ptr(), d_off, d_len, types, out, count=count,
                                                    total_bytes=total, max_len=blk, stream=cs()),
    "sst_verify": lambda: ctx.sst_verify_device(img.data_ptr(), d_off, d_len, out, fb, nb, count=count,
                                                total_bytes=total, max_len=blk, stream=cs()),
    "sst_verify_all_bad": lambda: ctx.sst_verify_device(bad.data_ptr(), d_off, d_len, out, fb, nb, count=count,
                                                        total_bytes=total, max_len=blk, stream=cs()),
}


def graph_us(fn, reps=20, rounds=7):
    fn()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(reps):
            fn()
    g.replay()
    torch.cuda.synchronize()
    ts = []
    for _ in range(rounds):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        g.replay()
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1) * 1e3 / reps)
    del g  # the graph is gone: its capture set may serve the next capture
    ctx.release_captures()
    return sorted(ts)[len(ts) // 2]


for r in range(3):
    for name, fn in forms.items():
        print(f"round {r} {name:18s} {graph_us(fn):8.2f} us per call", flush=True)
forms["sst_verify_all_bad"]()
torch.cuda.synchronize()
assert int(fb.item()) == 0 and int(nb.item()) == count, (int(fb.item()), int(nb.item()))  # every block reported
print("all-bad verdict exact: first_bad 0, nbad", count)
