#!/usr/bin/env python3
"""Rates of the host-memory entry points (PCIe-inclusive), each checked against the device-resident result:
  span/pinned    kvsep_crc32c_batch_host_span on a pinned vlog image (DMA straight from the image)
  span/pageable  the same image in pageable memory (staged through the pinned slots with a host memcpy)
  pointers       kvsep_crc32c_batch_host on one pointer per record (group-commit payloads; gathered)
usage: python host_forms_probe.py [GiB]"""
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import kvsep  # noqa: E402
from kvsep import workloads as W  # noqa: E402

gib = float(sys.argv[1]) if len(sys.argv) > 1 else 2.0
GIB = float(1 << 30)
off, ln = W.cfg3_layout(vlog=True, count=max(1, int(gib * GIB) // (W.VLOG_PAYLOAD + 8)))
span = int(off[-1] + ln[-1])
dev = torch.empty(span, dtype=torch.uint8, device="cuda")
kvsep.fill_splitmix64(dev.data_ptr(), span, 77, 0)
ctx = kvsep.Context(0)
ref = torch.zeros(off.size, dtype=torch.int32, device="cuda")
ctx.batch_device(dev.data_ptr(), torch.from_numpy(off.view(np.int64)).cuda(), torch.from_numpy(ln.view(np.int64)).cuda(),
                 ref, total_bytes=int(ln.sum()), max_len=int(ln.max()))
ref = ref.cpu().numpy().view(np.uint32)
pinned = torch.empty(span, dtype=torch.uint8, pin_memory=True)
pinned.copy_(dev)
pageable = pinned.numpy().copy()
del dev
useful = float(ln.sum())


def rate(fn, reps=3):
    res = fn()
    t0 = time.perf_counter()
    for _ in range(reps):
        res = fn()
    dt = (time.perf_counter() - t0) / reps
    return useful / GIB / dt, bool(np.array_equal(res, ref))


views = [pageable[int(o):int(o + n)] for o, n in zip(off, ln)]
for name, fn in (("span/pinned", lambda: ctx.batch_host_span(pinned.numpy(), off, ln)),
                 ("span/pageable", lambda: ctx.batch_host_span(pageable, off, ln)),
                 ("pointers", lambda: ctx.batch_host(views))):
    r, ok = rate(fn)
    print(f"{name:14s} {r:8.2f} GiB/s  parity={ok}  ({useful / GIB:.2f} GiB, {off.size} records)", flush=True)
