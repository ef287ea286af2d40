#!/usr/bin/env python3
"""Diag (KVSEP_DIAG build): the sorted-window kernel with a vmcnt(0) drain after each group's emit (KVSEP_NARROW=23)
against the shipped form (20), batch form, several groups per window: does draining the staged loads alone change
the CRCs?  usage: sorted_drain_probe.py"""
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, ".."))
sys.path.insert(0, os.path.join(HERE, "..", "..", "tests"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import _diag  # noqa: E402,F401
import kvsep  # noqa: E402
from conftest import load_oracle  # noqa: E402  (the checker)
from kvsep import splitmix64_bytes  # noqa: E402

dev = torch.device("cuda:0")
oracle = load_oracle()
host = splitmix64_bytes(64 << 20, 5, 0)
d = torch.from_numpy(host).to(dev)
u64 = lambda a: torch.from_numpy(np.ascontiguousarray(a, dtype=np.uint64).view(np.int64)).to(dev)  # noqa: E731
rng = np.random.default_rng(1)
for v in ("20", "23"):
    os.environ["KVSEP_NARROW"], os.environ["KVSEP_CRC_VARIANT"] = v, "1"
    ctx = kvsep.Context(0)
    ctx.set_kernel("narrow")  # forces the narrow family; the diag variant picks the form
    for n in (70000, 200000):
        for maxlen in (39, 200):
            ln = rng.integers(0, maxlen + 1, n).astype(np.uint64)
            off = np.zeros(n, np.uint64)
            off[1:] = np.cumsum(ln[:-1], dtype=np.uint64)
            exp = oracle.batch(host, off, ln, None, threads=8)
            out = torch.zeros(n, dtype=torch.int32, device=dev)
            ctx.batch_device(d.data_ptr(), u64(off), u64(ln), out, max_len=int(ln.max()), total_bytes=int(ln.sum()))
            torch.cuda.synchronize()
            bad = int(np.count_nonzero(out.cpu().numpy().view(np.uint32) != exp))
            print(f"variant {v} n={n} maxlen={maxlen}: {bad} mismatches", flush=True)
    ctx.close()
