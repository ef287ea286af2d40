#!/usr/bin/env python3
"""Config 2's CRC kernel and the streaming-read kernel over the SAME 256 MiB allocation, launched back to back in one
process -- the pair a rocprofv3 --pmc pass compares counter by counter (round 5: where the CRC kernel's extra time goes).
usage: cfg2_pair.py [reps]"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import kvsep  # noqa: E402
from kvsep import workloads as W  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 10
dev = torch.device("cuda:0")
off, ln = W.cfg2_layout()
total = int(ln.sum())
data = torch.empty(total + 64, dtype=torch.uint8, device=dev)
kvsep.fill_splitmix64(data.data_ptr(), total, W.SEED, 0)
d_off = torch.from_numpy(off.view(np.int64)).to(dev)
d_len = torch.from_numpy(ln.view(np.int64)).to(dev)
out = torch.zeros(off.size, dtype=torch.int32, device=dev)
sink = torch.zeros(4, dtype=torch.int32, device=dev)
ctx = kvsep.Context(0)
ctx.reserve(off.size, total)
for _ in range(reps):
    ctx.batch_device(data.data_ptr(), d_off, d_len, out, count=off.size, total_bytes=total, max_len=4096)
    ctx.stream_read(data.data_ptr(), total, sink)
torch.cuda.synchronize()
ref = np.fromfile(os.path.join(os.path.dirname(__file__), "..", "..", "tests", "golden", "full_cfg2.u32"), dtype="<u4")
assert np.array_equal(out.cpu().numpy().view(np.uint32), ref[:off.size]), "config 2 CRCs differ from the reference"
print("ok", ctx.kernel_name(off.size, 4096, total))
