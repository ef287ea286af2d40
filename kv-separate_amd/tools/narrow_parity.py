#!/usr/bin/env python3
"""Narrow-kernel mismatches against the oracle broken down by the block geometry the slot path branches on:
m = whole 16-B chunks between the 128-B grid and the 16-B end, head bytes (ps mod 16), tail bytes (pe mod 16) and
row count.  usage: narrow_parity.py [kernel ...]   (default: narrow16 narrow8)"""
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
rng = np.random.default_rng(7)
n = 20000
ln = rng.integers(0, 5000, n).astype(np.uint64)
ln[: n // 2] = rng.choice([15, 16, 17, 100, 127, 128, 129, 255, 256, 4096, 4097, 4111], n // 2)
off = np.zeros(n, np.uint64)
off[1:] = np.cumsum(ln[:-1] + rng.integers(0, 40, n - 1).astype(np.uint64), dtype=np.uint64)
host = splitmix64_bytes(int(off[-1] + ln[-1]) + 256, 5, 0)
init = rng.integers(0, 2**32, n, dtype=np.uint64).astype(np.uint32)
exp = oracle.batch(host, off, ln, init, threads=8)
d = torch.from_numpy(host).to(dev)
base = d.data_ptr()
assert base % 256 == 0
u64 = lambda a: torch.from_numpy(np.ascontiguousarray(a, dtype=np.uint64).view(np.int64)).to(dev)  # noqa: E731
pe = off + ln
h0 = np.minimum((off + 15) & ~np.uint64(15), pe)
a1 = np.maximum(pe & ~np.uint64(15), h0)
ar = np.maximum(a1 & ~np.uint64(127), h0)
m = ((a1 - ar) >> np.uint64(4)).astype(int)
K = np.where(ar > h0, (ar - h0 + np.uint64(127)) // np.uint64(128), 0).astype(int)
for k in sys.argv[1:] or ["narrow16", "narrow8"]:
    ctx = kvsep.Context(0)
    ctx.set_kernel(k)
    out = torch.zeros(n, dtype=torch.int32, device=dev)
    ctx.batch_device(base, u64(off), u64(ln), out, init=torch.from_numpy(init.view(np.int32)).to(dev),
                     max_len=int(ln.max()), total_bytes=int(ln.sum()))
    torch.cuda.synchronize()
    bad = out.cpu().numpy().view(np.uint32) != exp
    print(f"{k}: {int(bad.sum())} / {n} mismatches", flush=True)
    for name, key in (("m", m), ("head ps%16", (off % 16).astype(int)), ("tail pe%16", (pe % 16).astype(int)),
                      ("K==0", (K == 0).astype(int)), ("slot", np.arange(n) % 8)):
        tot, bd = collections.Counter(key.tolist()), collections.Counter(key[bad].tolist())
        print(f"  by {name}: " + " ".join(f"{v}:{bd[v]}/{tot[v]}" for v in sorted(tot)), flush=True)
    ctx.close()
