#!/usr/bin/env python3
"""Diag (KVSEP_DIAG build): the sorted-window kernel with the verify compare INSIDE the kernel as before round 2
(KVSEP_NARROW=24: load expected[b], compare, atomics; 25: only the load of expected[b]) against the shipped form
(20, compare in verify_finish_kernel), verify form, several groups per window, correct expectations: which part of
the in-kernel compare makes the third and later groups wrong?  usage: sorted_vin_probe.py"""
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, ".."))
sys.path.insert(0, os.path.join(HERE, "..", "..", "tests"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import _diag  # noqa: E402,F401
import kvsep  # noqa: E402

if os.environ.get("KVSEP_DIAG_LIB"):  # another diag build, e.g. one without the atomic optimizer
    kvsep.LIB_PATH, kvsep._lib = os.environ["KVSEP_DIAG_LIB"], None
    kvsep.lib()
from conftest import load_oracle  # noqa: E402  (the checker)
from kvsep import splitmix64_bytes  # noqa: E402

dev = torch.device("cuda:0")
oracle = load_oracle()
host = splitmix64_bytes(64 << 20, 5, 0)
d = torch.from_numpy(host).to(dev)
u64 = lambda a: torch.from_numpy(np.ascontiguousarray(a, dtype=np.uint64).view(np.int64)).to(dev)  # noqa: E731
rng = np.random.default_rng(1)
cases = []
for n in (70000, 200000):
    for maxlen in (39, 200):
        ln = rng.integers(0, maxlen + 1, n).astype(np.uint64)
        off = np.zeros(n, np.uint64)
        off[1:] = np.cumsum(ln[:-1], dtype=np.uint64)
        exp = oracle.batch(host, off, ln, None, threads=8)
        cases.append((n, maxlen, off, ln, exp, np.array([kvsep.mask(int(x)) for x in exp], dtype=np.uint32)))
for v in ("20", "24", "25"):
    os.environ["KVSEP_NARROW"], os.environ["KVSEP_CRC_VARIANT"] = v, "1"
    ctx = kvsep.Context(0)
    ctx.set_kernel("narrow")
    for n, maxlen, off, ln, exp, masked in cases:
        for verify in (False, True):
            out = torch.zeros(n, dtype=torch.int32, device=dev)
            fb = torch.zeros(1, dtype=torch.int64, device=dev)
            nb = torch.zeros(1, dtype=torch.int64, device=dev)
            if verify:
                ctx.verify_device(d.data_ptr(), u64(off), u64(ln), torch.from_numpy(masked.view(np.int32)).to(dev),
                                  out, fb, nb, max_len=int(ln.max()), total_bytes=int(ln.sum()))
            else:
                ctx.batch_device(d.data_ptr(), u64(off), u64(ln), out, max_len=int(ln.max()), total_bytes=int(ln.sum()))
            torch.cuda.synchronize()
            bad = int(np.count_nonzero(out.cpu().numpy().view(np.uint32) != exp))
            print(f"variant {v} n={n} maxlen={maxlen} verify={verify}: {bad} mismatches"
                  + (f", nbad={int(nb.item())}" if verify else ""), flush=True)
    ctx.close()
