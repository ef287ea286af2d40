#!/usr/bin/env python3
"""How fast can ANY kernel read a small batch?  Per-launch time, averaged over 20 back-to-back launches captured in
one hipGraph (bench.py's config-2 timing), of (a) the read-only streaming kernel (stream_read_kernel: no
descriptors, no tables, no compute) and (b) the CRC kernel on packed 4 KiB blocks (narrow kernel, both workgroup
sizes, and the wide kernel), over the same bytes.  The gap between (a) and the spec's time is the launch / ramp /
tail floor of a 1-launch batch of that size; the gap between (b) and (a) is what the CRC kernel adds.
usage: launch_floor_probe.py [MiB ...]"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import kvsep  # noqa: E402
from kvsep import workloads as W  # noqa: E402

dev = torch.device("cuda:0")
sizes = [int(x) for x in sys.argv[1:]] or [64, 256, 1024, 4096]
ctxs = {}
for k in ("auto", "narrow16", "narrow8", "wide"):
    ctxs[k] = kvsep.Context(0)
    ctxs[k].set_kernel(k)


def graph_avg_us(fn, reps=20, rounds=3):
    fn()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        with torch.cuda.graph(g, stream=s):
            for _ in range(reps):
                fn()
    best = []
    for _ in range(rounds):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        g.replay()
        e1.record()
        torch.cuda.synchronize()
        best.append(e0.elapsed_time(e1) * 1e3 / reps)
    del g  # the graph is gone: every context's capture sets may serve the next capture
    for c in ctxs.values():
        c.release_captures()
    return min(best), sorted(best)[len(best) // 2]


for mib in sizes:
    count = mib * 256
    off, ln = W.uniform_layout(count, 4096)
    total = int(ln.sum())
    data = torch.empty(total + 64, dtype=torch.uint8, device=dev)
    kvsep.fill_splitmix64(data.data_ptr(), total, 1, 0)
    d_off = torch.from_numpy(off.view(np.int64)).to(dev)
    d_len = torch.from_numpy(ln.view(np.int64)).to(dev)
    out = torch.zeros(count, dtype=torch.int32, device=dev)
    sink = torch.zeros(4, dtype=torch.int32, device=dev)
    rows = [("stream_read", lambda: ctxs["auto"].stream_read(data.data_ptr(), total, sink,
                                                             stream=torch.cuda.current_stream()))]
    for k, c in ctxs.items():
        c.reserve(count, total)
        rows.append((f"crc {k} ({c.kernel_name(count, 4096) if k == 'auto' else k})",
                     lambda c=c: c.batch_device(data.data_ptr(), d_off, d_len, out, count=count, total_bytes=total,
                                                max_len=4096, stream=torch.cuda.current_stream())))
    ideal = total / 8e12 * 1e6
    for name, fn in rows:
        mn, med = graph_avg_us(fn)
        print(f"{mib:5d} MiB {name:42s} min {mn:8.2f} us  med {med:8.2f} us  {total / med / 1e6:6.2f} TB/s  "
              f"(8 TB/s: {ideal:7.2f} us)", flush=True)
    del data, d_off, d_len, out
    torch.cuda.empty_cache()
