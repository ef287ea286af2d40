#!/usr/bin/env python3
"""Where does config 4's time go?  Times the Zipf batch whole, then its long blocks alone and its short
blocks alone (same data, same offsets), with the wide kernel and -- for the short subset -- the narrow one.
usage: python split_probe.py [threshold_bytes]"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import kvsep  # noqa: E402
from kvsep import workloads as W  # noqa: E402

thr = int(sys.argv[1]) if len(sys.argv) > 1 else 64 * 1024
dev = torch.device("cuda:0")
off, ln = W.cfg4_layout()
span = int(off[-1] + ln[-1])
data = torch.empty(span + 64, dtype=torch.uint8, device=dev)
kvsep.fill_splitmix64(data.data_ptr(), span, 7, 0)
ctx = kvsep.Context(0)
wide_only = kvsep.Context(0)
wide_only.set_kernel("wide")


def timeit(c, o, n, max_len, reps=5):
    d_off = torch.from_numpy(o.view(np.int64)).to(dev)
    d_len = torch.from_numpy(n.view(np.int64)).to(dev)
    out = torch.zeros(o.size, dtype=torch.int32, device=dev)
    c.reserve(o.size, int(n.sum()))
    c.batch_device(data.data_ptr(), d_off, d_len, out, total_bytes=int(n.sum()), max_len=max_len)
    torch.cuda.synchronize()
    c.set_timing(True)
    for _ in range(reps):
        c.batch_device(data.data_ptr(), d_off, d_len, out, total_bytes=int(n.sum()), max_len=max_len)
    torch.cuda.synchronize()
    c.set_timing(False)
    ms, k = c.get_timing()
    return ms / k


short = ln <= thr
t_all = timeit(ctx, off, ln, int(ln.max()))
t_long = timeit(ctx, off[~short], ln[~short], int(ln.max()))
t_short_wide = timeit(wide_only, off[short], ln[short], thr)
t_short_narrow = timeit(ctx, off[short], ln[short], thr)
print(f"threshold {thr}: {short.sum()} short blocks ({ln[short].sum() / 2**30:.2f} GiB), "
      f"{(~short).sum()} long ({ln[~short].sum() / 2**30:.2f} GiB)")
print(f"all {t_all:.3f} ms ({ln.sum() / t_all / 1e6:.1f} GB/s) | long only {t_long:.3f} ms "
      f"({ln[~short].sum() / t_long / 1e6:.1f} GB/s) | short wide {t_short_wide:.3f} ms | short narrow "
      f"{t_short_narrow:.3f} ms", flush=True)
