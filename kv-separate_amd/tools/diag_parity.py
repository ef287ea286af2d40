#!/usr/bin/env python3
"""Bit-exactness of KVSEP_DIAG kernel variants (tools/libkvsep_diag.so) against the oracle on ragged blocks at every
start offset mod 128, random inits, three piece sizes, both schedules -- the check a variant must pass before it
can be promoted into the shipped library.  usage: diag_parity.py <wide variant> ..."""
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
rng = np.random.default_rng(20261016)
n = 3000
host = splitmix64_bytes(8 << 20, 99, 0)
ln = np.concatenate([rng.integers(0, 40000, n - 40), np.arange(1000, 1040) * 16 + 7, ]).astype(np.uint64)
ln[:200] = rng.integers(0, 300, 200)
off = (rng.integers(0, (host.size - 40000) // 128, n) * 128 + np.arange(n) % 128).astype(np.uint64)
init = rng.integers(0, 2**32, n, dtype=np.uint64).astype(np.uint32)
exp = oracle.batch(host, off, ln, init, threads=8)
d = torch.from_numpy(host).to(dev)
u64 = lambda a: torch.from_numpy(np.ascontiguousarray(a, dtype=np.uint64).view(np.int64)).to(dev)  # noqa: E731
for v in sys.argv[1:]:
    os.environ["KVSEP_CRC_VARIANT"] = v
    ctx = kvsep.Context(0)
    bad = 0
    for piece in (1024, 4096, 128 * 1024):
        ctx.set_piece_bytes(piece)
        for dyn in (None, False, True):
            ctx.set_schedule(dyn)
            for max_len in (0, 64 * 1024 + 1):
                keep = ln <= max_len if max_len else np.ones(n, bool)
                out = torch.zeros(int(keep.sum()), dtype=torch.int32, device=dev)
                ctx.set_kernel("wide")
                ctx.batch_device(d.data_ptr(), u64(off[keep]), u64(ln[keep]), out,
                                 init=torch.from_numpy(init[keep].view(np.int32)).to(dev), max_len=max_len,
                                 total_bytes=int(ln[keep].sum()))
                torch.cuda.synchronize()
                got = out.cpu().numpy().view(np.uint32)
                bad += int(np.count_nonzero(got != exp[keep]))
    print(f"variant {v}: {'BIT-EXACT' if bad == 0 else f'{bad} MISMATCHES'}", flush=True)
    ctx.close()
