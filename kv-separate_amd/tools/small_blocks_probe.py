#!/usr/bin/env python3
"""Kernel time vs block count for uniform small blocks: separates the fixed per-launch cost from the
per-block cost (config 2 diagnosis)."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import kvsep  # noqa: E402
from kvsep import workloads as W  # noqa: E402

dev = torch.device("cuda:0")
ctx = kvsep.Context(0)
for blen in (4096, 16384, 65536):
    for count in (256, 4096, 16384, 65536, 262144):
        if blen * count > (4 << 30):
            continue
        off, ln = W.uniform_layout(count, blen)
        total = int(ln.sum())
        data = torch.empty(total + 64, dtype=torch.uint8, device=dev)
        kvsep.fill_splitmix64(data.data_ptr(), total, 1, 0)
        d_off = torch.from_numpy(off.view(np.int64)).to(dev)
        d_len = torch.from_numpy(ln.view(np.int64)).to(dev)
        out = torch.zeros(count, dtype=torch.int32, device=dev)
        for _ in range(3):
            ctx.batch_device(data.data_ptr(), d_off, d_len, out, total_bytes=total, max_len=blen)
        torch.cuda.synchronize()
        ctx.set_timing(True)
        for _ in range(20):
            ctx.batch_device(data.data_ptr(), d_off, d_len, out, total_bytes=total, max_len=blen)
        torch.cuda.synchronize()
        ctx.set_timing(False)
        ms, n = ctx.get_timing()
        t = ms / n
        print(f"len {blen:6d} count {count:7d} total {total / 2**20:8.1f} MiB: {t * 1e3:9.2f} us  {total / t / 1e6:8.1f} GB/s",
              flush=True)
        del data, d_off, d_len, out
        torch.cuda.empty_cache()
