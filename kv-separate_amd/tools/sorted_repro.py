#!/usr/bin/env python3
"""Reproducer for a soak.py failure (sorted-window kernel, verify form): which sorted group of a window mismatches
the oracle?  usage: sorted_repro.py"""
import collections
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, ".."))
sys.path.insert(0, os.path.join(HERE, "..", "..", "tests"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import kvsep  # noqa: E402
from conftest import load_oracle  # noqa: E402  (the checker)
from kvsep import splitmix64_bytes  # noqa: E402

dev = torch.device("cuda:0")
oracle = load_oracle()
POOL = 64 << 20
host = splitmix64_bytes(POOL, 5, 0)
d = torch.from_numpy(host).to(dev)
u64 = lambda a: torch.from_numpy(np.ascontiguousarray(a, dtype=np.uint64).view(np.int64)).to(dev)  # noqa: E731
ctx = kvsep.Context(0)
ctx.set_kernel("sorted")
rng = np.random.default_rng(1)
NWAVES = 256 * 16


def group_of(n, ln):
    """(sorted group index within its window, groups in that window) of every block, as the kernel forms them."""
    groups = (n + 7) // 8
    gper = (groups + NWAVES - 1) // NWAVES
    gi = np.zeros(n, np.int64)
    ng = np.zeros(n, np.int64)
    for lo in range(0, n, gper * 8):
        hi = min(n, lo + gper * 8)
        for w in range(lo, hi, 64):
            e = min(hi, w + 64)
            order = np.lexsort((np.arange(e - w), ln[w:e]))  # by (len, lane)
            pos = np.empty(e - w, np.int64)
            pos[order] = np.arange(e - w)
            gi[w:e] = pos // 8
            ng[w:e] = (e - w + 7) // 8
    return gi, ng


for n in (70000, 200000, 40000, 12289):
    for maxlen in (39, 200):
        for verify in (False, True):
            ln = rng.integers(0, maxlen + 1, n).astype(np.uint64)
            off = np.zeros(n, np.uint64)
            off[1:] = np.cumsum(ln[:-1], dtype=np.uint64)
            exp = oracle.batch(host, off, ln, None, threads=8)
            out = torch.zeros(n, dtype=torch.int32, device=dev)
            if verify:
                masked = np.array([kvsep.mask(int(x)) for x in exp], dtype=np.uint32)
                fb = torch.zeros(1, dtype=torch.int64, device=dev)
                nb = torch.zeros(1, dtype=torch.int64, device=dev)
                ctx.verify_device(d.data_ptr(), u64(off), u64(ln), torch.from_numpy(masked.view(np.int32)).to(dev),
                                  out, fb, nb, max_len=int(ln.max()), total_bytes=int(ln.sum()))
            else:
                ctx.batch_device(d.data_ptr(), u64(off), u64(ln), out, max_len=int(ln.max()), total_bytes=int(ln.sum()))
            torch.cuda.synchronize()
            got = out.cpu().numpy().view(np.uint32)
            bad = got != exp
            gi, ng = group_of(n, ln)
            tot = collections.Counter(zip(ng.tolist(), gi.tolist()))
            bd = collections.Counter(zip(ng[bad].tolist(), gi[bad].tolist()))
            print(f"n={n} maxlen={maxlen} verify={verify}: {int(bad.sum())} mismatches; by (groups in window, group): "
                  + " ".join(f"{k}:{bd[k]}/{tot[k]}" for k in sorted(tot)), flush=True)
            if verify:
                print(f"   nbad={int(nb.item())} first_bad={int(fb.item())}", flush=True)
