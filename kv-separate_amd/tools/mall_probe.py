#!/usr/bin/env python3
"""Does the 256 MB Infinity Cache (MALL) carry a small batch from one graph-replayed launch to the next (round 5)?
Per-launch time, 20 launches per hipGraph replay (bench.py's config-2 form), of the streaming-read kernel and the CRC
kernel over ONE batch re-read every launch, against the same launches alternating over TWO distinct batches of the
same size (no launch re-reads what the previous one read).  If the one-batch form is faster, part of the small-batch
"ceiling" is cache, not HBM.  usage: mall_probe.py [MiB ...]"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import kvsep  # noqa: E402
from kvsep import workloads as W  # noqa: E402

dev = torch.device("cuda:0")
ctx = kvsep.Context(0)


def graph_us(fns, reps=20, rounds=5):
    for f in fns:
        f()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for i in range(reps):
            fns[i % len(fns)]()
    g.replay()
    torch.cuda.synchronize()
    best = []
    for _ in range(rounds):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        g.replay()
        e1.record()
        torch.cuda.synchronize()
        best.append(e0.elapsed_time(e1) * 1e3 / reps)
    return min(best), sorted(best)[len(best) // 2]


for mib in [int(x) for x in sys.argv[1:]] or [256, 512, 1024]:
    count = mib * 256
    off, ln = W.uniform_layout(count, 4096)
    total = int(ln.sum())
    bufs = []
    for seed in (1, 2):
        d = torch.empty(total + 64, dtype=torch.uint8, device=dev)
        kvsep.fill_splitmix64(d.data_ptr(), total, seed, 0)
        bufs.append(d)
    d_off = torch.from_numpy(off.view(np.int64)).to(dev)
    d_len = torch.from_numpy(ln.view(np.int64)).to(dev)
    outs = [torch.zeros(count, dtype=torch.int32, device=dev) for _ in range(2)]
    sink = torch.zeros(4, dtype=torch.int32, device=dev)
    ctx.reserve(count, total)
    st = lambda b: (lambda: ctx.stream_read(b.data_ptr(), total, sink, stream=torch.cuda.current_stream()))  # noqa
    cr = lambda b, o: (lambda: ctx.batch_device(b.data_ptr(), d_off, d_len, o, count=count, total_bytes=total,  # noqa
                                                max_len=4096, stream=torch.cuda.current_stream()))
    rows = [("stream, one batch", [st(bufs[0])]), ("stream, two batches alternating", [st(bufs[0]), st(bufs[1])]),
            ("crc, one batch", [cr(bufs[0], outs[0])]),
            ("crc, two batches alternating", [cr(bufs[0], outs[0]), cr(bufs[1], outs[1])])]
    for name, fns in rows:
        mn, med = graph_us(fns)
        print(f"{mib:5d} MiB {name:34s} min {mn:8.2f} us  med {med:8.2f} us  {total / med / 1e6:6.3f} TB/s", flush=True)
    del bufs, outs
    torch.cuda.empty_cache()
