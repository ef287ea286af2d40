#!/usr/bin/env python3
"""Is the first CRC pass over a batch slower because the batch is freshly written, or because it is the
process's first launch (clocks, code object)?  Two 32 GiB batches A and B: A x3, B x3, refill A, A x3.
Prints every launch's kernel time (HIP events)."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import kvsep  # noqa: E402
from kvsep import workloads as W  # noqa: E402

if os.environ.get("KVSEP_LIB"):  # another build of the library (A/B of the data generator)
    kvsep.LIB_PATH, kvsep._lib = os.environ["KVSEP_LIB"], None

count = 32768
off, ln = W.cfg3_layout(count=count)
span = int(off[-1] + ln[-1])
dev = torch.device("cuda:0")
bufs = {k: torch.empty(span + 64, dtype=torch.uint8, device=dev) for k in "AB"}
for i, k in enumerate("AB"):
    kvsep.fill_splitmix64(bufs[k].data_ptr(), span, 10 + i, 0)
d_off = torch.from_numpy(off.view(np.int64)).to(dev)
d_len = torch.from_numpy(ln.view(np.int64)).to(dev)
out = torch.zeros(count, dtype=torch.int32, device=dev)
ctx = kvsep.Context(0)
ctx.reserve(count, int(ln.sum()))
torch.cuda.synchronize()


def run(k, reps=3):
    ctx.set_timing(True)
    ms = []
    for _ in range(reps):
        ctx.batch_device(bufs[k].data_ptr(), d_off, d_len, out, total_bytes=int(ln.sum()), max_len=int(ln.max()))
        torch.cuda.synchronize()
        t, n = ctx.get_timing()
        ms.append(t / n)
    ctx.set_timing(False)
    print(k, " ".join(f"{m:.3f} ms ({int(ln.sum()) / m / 1e6:.0f} GB/s)" for m in ms), flush=True)


run("A")
run("B")
kvsep.fill_splitmix64(bufs["A"].data_ptr(), span, 99, 0)
torch.cuda.synchronize()
run("A")
kvsep.fill_splitmix64(bufs["B"].data_ptr(), span, 98, 0)
torch.cuda.synchronize()
run("B")
