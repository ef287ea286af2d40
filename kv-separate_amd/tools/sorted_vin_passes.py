#!/usr/bin/env python3
"""Diag: which compiler pass does the sorted-window in-kernel-compare fault (KVSEP_NARROW=24, and 28: the same with a
plain store instead of the atomics) depend on?  The KVSEP_DIAG library rebuilt with one LLVM option each:
  libkvsep_diag_novgprlr.so  -mllvm --amdgpu-opt-vgpr-liverange=false   (SIOptimizeVGPRLiveRange off)
  libkvsep_diag_noexecpre.so -mllvm --amdgpu-opt-exec-mask-pre-ra=false (SIOptimizeExecMaskingPreRA off)
  libkvsep_diag_snop.so      -mllvm --amdgpu-snop-padding=2             (s_nop 2 before every instruction)
  libkvsep_diag_wz.so        -mllvm --amdgpu-waitcnt-forcezero          (every wait is vmcnt(0) lgkmcnt(0))
  libkvsep_diag_nopeep.so    -mllvm --amdgpu-sdwa-peephole=false --amdgpu-dpp-combine=false
  libkvsep_diag_nosdwa.so    -mllvm --amdgpu-sdwa-peephole=false                (profiles/round3/sorted_vin_passes2.log)
  libkvsep_diag_nodpp.so     -mllvm --amdgpu-dpp-combine=false
plus the plain diag build.  Same batch as tools/sorted_vin_probe.py (n = 70,000, lengths 0..39, correct stored
words): a library whose variant 24 / 28 gets 0 wrong CRCs points at the pass or mechanism it switched off.
Build one: the diag Makefile line with the option added, e.g.
  hipcc <CXXFLAGS> -DKVSEP_DIAG -mllvm --amdgpu-sdwa-peephole=false -shared -o tools/libkvsep_diag_nosdwa.so <SRCS>
Result and cause: DESIGN.md §3.5.
usage: sorted_vin_passes.py [lib ...]"""
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
libs = sys.argv[1:] or ["libkvsep_diag.so", "libkvsep_diag_novgprlr.so", "libkvsep_diag_noexecpre.so",
                        "libkvsep_diag_snop.so", "libkvsep_diag_wz.so", "libkvsep_diag_nopeep.so"]
for name in libs:
    path = os.path.join(HERE, name)
    if not os.path.exists(path):
        print(f"{name}: missing", flush=True)
        continue
    kvsep.LIB_PATH, kvsep._lib = path, None
    kvsep.lib()
    for v in ("20", "24", "28"):
        os.environ["KVSEP_NARROW"], os.environ["KVSEP_CRC_VARIANT"] = v, "1"
        ctx = kvsep.Context(0)
        ctx.set_kernel("narrow")
        out = torch.zeros(n, dtype=torch.int32, device=dev)
        fb = torch.zeros(1, dtype=torch.int64, device=dev)
        nb = torch.zeros(1, dtype=torch.int64, device=dev)
        ctx.verify_device(d.data_ptr(), u64(off), u64(ln), torch.from_numpy(masked.view(np.int32)).to(dev), out, fb,
                          nb, max_len=int(ln.max()), total_bytes=int(ln.sum()))
        torch.cuda.synchronize()
        bad = int(np.count_nonzero(out.cpu().numpy().view(np.uint32) != exp))
        print(f"{name} variant {v}: {bad} wrong CRCs", flush=True)
        ctx.close()
