#!/usr/bin/env python3
"""Diag: is the KVSEP_NARROW=24 wrong-CRC fault deterministic, and does it depend on the expected[] words the compare
loads?  Same batch as sorted_vin_probe.py (n=70000, lengths 0..39): three runs with correct expectations (are the wrong
blocks and their values identical?), then expectations all zero (every compare fails, so every atomic runs), then
expectations correct only for the first two groups of each window.  usage: sorted_vin_repeat.py"""
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
n, maxlen = 70000, 39
ln = rng.integers(0, maxlen + 1, n).astype(np.uint64)
off = np.zeros(n, np.uint64)
off[1:] = np.cumsum(ln[:-1], dtype=np.uint64)
exp = oracle.batch(host, off, ln, None, threads=8)
masked = np.array([kvsep.mask(int(x)) for x in exp], dtype=np.uint32)
os.environ["KVSEP_NARROW"], os.environ["KVSEP_CRC_VARIANT"] = "24", "1"
ctx = kvsep.Context(0)
ctx.set_kernel("narrow")


def run(expected, sentinel):
    out = torch.full((n,), sentinel, dtype=torch.int32, device=dev)
    fb = torch.zeros(1, dtype=torch.int64, device=dev)
    nb = torch.zeros(1, dtype=torch.int64, device=dev)
    ctx.verify_device(d.data_ptr(), u64(off), u64(ln), torch.from_numpy(expected.view(np.int32)).to(dev), out, fb, nb,
                      max_len=int(ln.max()), total_bytes=int(ln.sum()))
    torch.cuda.synchronize()
    return out.cpu().numpy().view(np.uint32).copy(), int(nb.item())


ref = None
for rep in range(3):
    got, nb = run(masked, rep)
    bad = got != exp
    print(f"correct expectations, run {rep}: {int(bad.sum())} wrong, nbad={nb}", flush=True)
    if ref is None:
        ref = got
    else:
        print(f"   identical to run 0: {np.array_equal(got, ref)}; differing blocks {int((got != ref).sum())}", flush=True)
zero = np.zeros(n, np.uint32)
got, nb = run(zero, 0)
print(f"all-zero expectations: {int((got != exp).sum())} wrong, nbad={nb}; same wrong values as run 0: "
      f"{np.array_equal(got, ref)}", flush=True)
got, nb = run(~masked, 0)
print(f"all-wrong (complemented) expectations: {int((got != exp).sum())} wrong, nbad={nb}; same as run 0: "
      f"{np.array_equal(got, ref)}", flush=True)
# the wrong values as a function of block: do they depend on which lanes ran the compare branch?
half = masked.copy()
half[::2] ^= 1
got, nb = run(half, 0)
print(f"every other expectation wrong: {int((got != exp).sum())} wrong, nbad={nb}; same as run 0: "
      f"{np.array_equal(got, ref)}", flush=True)
ctx.close()
