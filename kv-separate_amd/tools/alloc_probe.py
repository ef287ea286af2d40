#!/usr/bin/env python3
"""How much of the run-to-run spread of config 3a comes from the allocation?  In ONE process: allocate a 64 GiB
batch, fill it, time the CRC kernel and the streaming-read ceiling over it (HIP events, several passes), free
it, and repeat with a fresh allocation `--allocs` times.  Usage: alloc_probe.py [--allocs 4] [--passes 6]"""
import argparse
import os
import statistics
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import kvsep  # noqa: E402
from kvsep import workloads as W  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--allocs", type=int, default=4)
    ap.add_argument("--passes", type=int, default=6)
    ap.add_argument("--schedules", action="store_true", help="also time the static and round-robin schedules")
    args = ap.parse_args()
    dev = torch.device("cuda:0")
    off, ln = W.cfg3_layout()
    total = int(ln.sum())
    d_off = torch.from_numpy(off.view(np.int64)).to(dev)
    d_len = torch.from_numpy(ln.view(np.int64)).to(dev)
    out = torch.zeros(off.size, dtype=torch.int32, device=dev)
    sink = torch.zeros(64, dtype=torch.int32, device=dev)
    ctx = kvsep.Context(0)
    ctx.reserve(off.size, total)
    # the same kernel under the other two schedules: static contiguous runs, static round-robin pieces (all waves
    # inside one sweeping window of the batch at any time: far fewer distinct pages in flight)
    scheds = {"guided": ctx}
    if args.schedules:
        c = kvsep.Context(0)
        c.set_schedule(False)
        c.reserve(off.size, total)
        scheds["static"] = c
        c = kvsep.Context(0)
        c.set_schedule("rr")
        c.reserve(off.size, total)
        scheds["static-rr"] = c
    for k in range(args.allocs):
        data = torch.empty(total + 64, dtype=torch.uint8, device=dev)
        kvsep.fill_splitmix64(data.data_ptr(), total, 1 + k, 0)
        torch.cuda.synchronize()
        crc, rd = [], []
        other = {k: [] for k in scheds if k != "guided"}
        for p in range(args.passes + 1):
            for name, c in scheds.items():
                c.set_timing(True)
                c.batch_device(data.data_ptr(), d_off, d_len, out, total_bytes=total, max_len=int(ln.max()))
                torch.cuda.synchronize()
                c.set_timing(False)
                ms, n = c.get_timing()
                if p and name != "guided":
                    other[name].append(total / (ms / n) / 1e6)
                if name == "guided":
                    gms, gn = ms, n
            ms, n = gms, gn
            ctx.set_timing(True)
            ctx.stream_read(data.data_ptr(), total, sink)
            torch.cuda.synchronize()
            ctx.set_timing(False)
            ms2, n2 = ctx.get_timing()
            if p:  # pass 0 is the first pass over freshly written data
                crc.append(total / (ms / n) / 1e6)
                rd.append(total / (ms2 / n2) / 1e6)
        print(f"alloc {k} @ {data.data_ptr():#x}: crc {statistics.median(crc):.0f} GB/s "
              f"(min {min(crc):.0f} max {max(crc):.0f})  read ceiling {statistics.median(rd):.0f} GB/s  "
              f"ratio {statistics.median(crc) / statistics.median(rd):.3f}"
              + "".join(f"  {k} {statistics.median(v):.0f}" for k, v in other.items()), flush=True)
        del data
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
