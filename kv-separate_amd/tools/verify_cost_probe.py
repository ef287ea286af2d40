#!/usr/bin/env python3
"""What the verify form costs over the plain batch form, per config (within 1 %).

For each config the same device-resident batch is checksummed K times by kvsep_crc32c_batch_device and K times by
kvsep_crc32c_verify_device (correct stored words, so nbad = 0), each as ONE hipGraph of K back-to-back calls timed with
a HIP event pair on the replay stream, interleaved over several rounds in one process; the median per-call time of each
form is reported (whole call: since round 4 the verify form has no init launch -- the last workgroup publishes the
verdict and resets the context's accumulators), and the CRC kernel
alone (the library's event pair around it, eager launches).  Every verify call's results are checked (out == the batch form's, nbad == 0), and a last verify call
with three planted bad words must report them.  Configs: 2 (65,536 x 4 KiB: the narrow kernel), 3b (65,536 vlog records
of 1,048,609 B: the wide kernel + combine), 4s (config 4's blocks <= 32 KiB: the sorted-window kernel).
usage: verify_cost_probe.py [--configs 2,3b,4s] [--steps 20] [--rounds 5]"""
import argparse
import json
import os
import statistics
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, ".."))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import kvsep  # noqa: E402
from kvsep import workloads as W  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--configs", default="2,3b,4s")
ap.add_argument("--steps", type=int, default=20)
ap.add_argument("--rounds", type=int, default=5)
args = ap.parse_args()
dev = torch.device("cuda:0")
u64 = lambda a: torch.from_numpy(np.ascontiguousarray(a, dtype=np.uint64).view(np.int64)).to(dev)  # noqa: E731


def layout(cfg):
    if cfg == "2":
        off, ln = W.cfg2_layout()
        return off, ln, W.SEED
    if cfg == "3b":
        off, ln = W.cfg3_layout(vlog=True)
        return off, ln, W.SEED + 1
    if cfg == "4s":  # config 4's short blocks, packed: the ragged batch the sorted-window kernel takes
        ln = W.zipf_lengths()
        ln = ln[ln <= 32 * 1024]
        off = np.zeros(ln.size, np.uint64)
        off[1:] = np.cumsum(ln[:-1], dtype=np.uint64)
        return off, ln, W.SEED + 2
    raise SystemExit(cfg)


results = {}
for cfg in args.configs.split(","):
    off, ln, seed = layout(cfg)
    n = ln.size
    span = int(off[-1] + ln[-1])
    data = torch.empty(span + 64, dtype=torch.uint8, device=dev)
    kvsep.fill_splitmix64(data.data_ptr(), span, seed, 0)
    d_off, d_len = u64(off), u64(ln)
    tb, ml = int(ln.sum()), int(ln.max())
    ctx = kvsep.Context(0)
    ctx.reserve(n, tb)
    out_b = torch.zeros(n, dtype=torch.int32, device=dev)
    out_v = torch.zeros(n, dtype=torch.int32, device=dev)
    fb = torch.zeros(1, dtype=torch.int64, device=dev)
    nb = torch.zeros(1, dtype=torch.int64, device=dev)
    ctx.batch_device(data.data_ptr(), d_off, d_len, out_b, total_bytes=tb, max_len=ml)
    torch.cuda.synchronize()
    crc = out_b.cpu().numpy().view(np.uint32)
    stored = np.array([kvsep.mask(int(c)) for c in crc], np.uint32)
    d_exp = torch.from_numpy(stored.view(np.int32)).to(dev)
    kname = ctx.kernel_name(n, ml, tb)

    def batch_call(st):
        ctx.batch_device(data.data_ptr(), d_off, d_len, out_b, total_bytes=tb, max_len=ml, stream=st)

    def verify_call(st):
        ctx.verify_device(data.data_ptr(), d_off, d_len, d_exp, out_v, fb, nb, total_bytes=tb, max_len=ml, stream=st)

    graphs = {}
    for name, fn in (("batch", batch_call), ("verify", verify_call)):
        fn(torch.cuda.current_stream())
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            for _ in range(args.steps):
                fn(torch.cuda.current_stream())
        g.replay()
        torch.cuda.synchronize()
        graphs[name] = g
    times = {"batch": [], "verify": []}
    for r in range(args.rounds):
        for name in (("batch", "verify") if r % 2 == 0 else ("verify", "batch")):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            graphs[name].replay()
            e1.record()
            torch.cuda.synchronize()
            times[name].append(e0.elapsed_time(e1) * 1e3 / args.steps)  # us per call
    # kernel-only: the library's HIP event pair around the main CRC kernel, eager launches (verify vs batch)
    kern = {}
    for name, fn in (("batch", batch_call), ("verify", verify_call)):
        ctx.get_timing()
        ctx.set_timing(True)
        for _ in range(args.steps):
            fn(torch.cuda.current_stream())
        torch.cuda.synchronize()
        ctx.set_timing(False)
        ms, nl = ctx.get_timing()
        kern[name] = ms * 1e3 / max(1, nl)
    ok = np.array_equal(out_v.cpu().numpy(), out_b.cpu().numpy()) and int(nb.item()) == 0 and int(fb.item()) == -1
    bad = stored.copy()
    plant = [n // 3, n // 3 + 1, n - 1]
    for i in plant:
        bad[i] ^= 0x10
    d_bad = torch.from_numpy(bad.view(np.int32)).to(dev)
    ctx.verify_device(data.data_ptr(), d_off, d_len, d_bad, out_v, fb, nb, total_bytes=tb, max_len=ml)
    torch.cuda.synchronize()
    caught = (int(fb.item()), int(nb.item())) == (plant[0], len(plant))
    mb, mv = statistics.median(times["batch"]), statistics.median(times["verify"])
    results[cfg] = {"kernel": kname, "blocks": n, "bytes": tb, "batch_us": round(mb, 2), "verify_us": round(mv, 2),
                    "verify_over_batch": round(mv / mb, 4),
                    "kernel_batch_us": round(kern["batch"], 2), "kernel_verify_us": round(kern["verify"], 2),
                    "kernel_verify_over_batch": round(kern["verify"] / kern["batch"], 4), "batch_runs_us": [round(t, 2) for t in times["batch"]],
                    "verify_runs_us": [round(t, 2) for t in times["verify"]], "verify_exact": ok,
                    "planted_bad_caught": caught}
    print(json.dumps({cfg: results[cfg]}), flush=True)
    ctx.close()
    del data, graphs
    torch.cuda.empty_cache()
