#!/usr/bin/env python3
"""Diag (KVSEP_DIAG build): bisect the wrong-CRC fault of the sorted-window kernel with the in-kernel verify compare.
Variants (KVSEP_NARROW, crc32c_narrow_sorted_kernel's kVIn): 20 shipped (compare in verify_finish_kernel), 24 the
round-1 compare (load expected, compare, atomics inside the emit branch), 25 only the load, 26 = 24 + s_nops after the
join, 27 = 24 + full s_waitcnt after the join, 28 = 24 with a plain store instead of the atomics, 29 = the compare in
full EXEC (ballot) with the atomics behind a wave-uniform branch.  Correct expectations, so a correct kernel reports
0 wrong CRCs and nbad = 0.  usage: sorted_vin_bisect.py [variant ...]"""
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
cases = []
for n, maxlen in ((70000, 39), (70000, 200), (200000, 39)):
    ln = rng.integers(0, maxlen + 1, n).astype(np.uint64)
    off = np.zeros(n, np.uint64)
    off[1:] = np.cumsum(ln[:-1], dtype=np.uint64)
    exp = oracle.batch(host, off, ln, None, threads=8)
    cases.append((n, maxlen, off, ln, exp, np.array([kvsep.mask(int(x)) for x in exp], dtype=np.uint32)))
for v in sys.argv[1:] or ["20", "24", "25", "26", "27", "28", "29"]:
    os.environ["KVSEP_NARROW"], os.environ["KVSEP_CRC_VARIANT"] = v, "1"
    ctx = kvsep.Context(0)
    ctx.set_kernel("narrow")
    for n, maxlen, off, ln, exp, masked in cases:
        out = torch.zeros(n, dtype=torch.int32, device=dev)
        fb = torch.zeros(1, dtype=torch.int64, device=dev)
        nb = torch.zeros(1, dtype=torch.int64, device=dev)
        ctx.verify_device(d.data_ptr(), u64(off), u64(ln), torch.from_numpy(masked.view(np.int32)).to(dev), out, fb, nb,
                          max_len=int(ln.max()), total_bytes=int(ln.sum()))
        torch.cuda.synchronize()
        bad = int(np.count_nonzero(out.cpu().numpy().view(np.uint32) != exp))
        print(f"variant {v} n={n} maxlen={maxlen}: {bad} wrong CRCs, nbad={int(nb.item())}", flush=True)
    ctx.close()
