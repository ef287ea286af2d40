#!/usr/bin/env python3
"""Runs one uniform-block batch `reps` times (no parity check): a fixed target for PMC passes and for the
diagnostic kernel variants (KVSEP_CRC_VARIANT), whose results are deliberately wrong.
Usage: one_batch.py <block_len> <count> [reps]"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import kvsep  # noqa: E402
from kvsep import workloads as W  # noqa: E402

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import _diag  # noqa: E402,F401  -- KVSEP_CRC_VARIANT reaches only the KVSEP_DIAG build

blen = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
count = int(sys.argv[2]) if len(sys.argv) > 2 else 65536
reps = int(sys.argv[3]) if len(sys.argv) > 3 else 5
dev = torch.device("cuda:0")
ctx = kvsep.Context(0)
off, ln = W.uniform_layout(count, blen)
total = int(ln.sum())
data = torch.empty(total + 64, dtype=torch.uint8, device=dev)
kvsep.fill_splitmix64(data.data_ptr(), total, 1, 0)
d_off = torch.from_numpy(off.view(np.int64)).to(dev)
d_len = torch.from_numpy(ln.view(np.int64)).to(dev)
out = torch.zeros(count, dtype=torch.int32, device=dev)
ctx.set_timing(True)
for _ in range(reps):
    ctx.batch_device(data.data_ptr(), d_off, d_len, out, total_bytes=total, max_len=blen)
torch.cuda.synchronize()
ms, n = ctx.get_timing()
print(f"variant {os.environ.get('KVSEP_CRC_VARIANT', '1')} len {blen} count {count}: {ms / n * 1e3:.2f} us/batch "
      f"{total / (ms / n) / 1e6:.1f} GB/s", flush=True)
