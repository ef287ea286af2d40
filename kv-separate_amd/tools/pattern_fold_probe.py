#!/usr/bin/env python3
"""Do the read patterns keep their rate with the CRC fold chain on every row?  KVSEP_DIAG stream_fold_kernel
(wrong results by design) against the plain streaming-read ceiling and the real CRC kernel on config 3a, over ONE
64 GiB allocation, interleaved in one process: variant 0 = stream_read_kernel (no compute); 31 / 32 = the ceiling's
pattern (a workgroup's waves interleave the 1 KiB rows of a 1 MiB chunk) with 8 / 4 rows per round and the
Z_1024 fold; 33 / 34 = per-wave 128 KiB chunks with the fold; crc = the shipped CRC kernel on 65,536 x 1 MiB.
usage: pattern_fold_probe.py [--rounds 5]"""
import argparse
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, ".."))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import _diag  # noqa: E402,F401
import kvsep  # noqa: E402
from kvsep import workloads as W  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--reps", type=int, default=3)
    args = ap.parse_args()
    dev = torch.device("cuda:0")
    off, ln = W.cfg3_layout()
    span = int(off[-1] + ln[-1])
    data = torch.empty(span + 64, dtype=torch.uint8, device=dev)
    kvsep.fill_splitmix64(data.data_ptr(), span, 1, 0)
    sink = torch.zeros(4, dtype=torch.int32, device=dev)
    ctxs = {}
    for v in ("0", "31", "32", "33", "34"):
        os.environ["KVSEP_CRC_VARIANT"], os.environ["KVSEP_NARROW"] = v, "1"
        ctxs[v] = kvsep.Context(0)
    os.environ["KVSEP_CRC_VARIANT"] = "1"
    crc = kvsep.Context(0)
    d_off = torch.from_numpy(off.view(np.int64)).to(dev)
    d_len = torch.from_numpy(ln.view(np.int64)).to(dev)
    out = torch.zeros(off.size, dtype=torch.int32, device=dev)
    useful = int(ln.sum())
    crc.reserve(off.size, useful)
    res = {k: [] for k in list(ctxs) + ["crc"]}
    for r in range(args.rounds + 1):
        for k, c in ctxs.items():
            c.set_timing(True)
            for _ in range(args.reps):
                c.stream_read(data.data_ptr(), span, sink)
            torch.cuda.synchronize()
            c.set_timing(False)
            ms, n = c.get_timing()
            if r:
                res[k].append(span / (ms / n * 1e-3) / 1e9)
        crc.set_timing(True)
        for _ in range(args.reps):
            crc.batch_device(data.data_ptr(), d_off, d_len, out, total_bytes=useful, max_len=int(ln.max()))
        torch.cuda.synchronize()
        crc.set_timing(False)
        ms, n = crc.get_timing()
        if r:
            res["crc"].append(useful / (ms / n * 1e-3) / 1e9)
    for k, v in res.items():
        v = sorted(v)
        print(f"variant {k:>4s}: median {v[len(v) // 2]:8.1f} GB/s  min {v[0]:8.1f}  max {v[-1]:8.1f}", flush=True)


if __name__ == "__main__":
    main()
