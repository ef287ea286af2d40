#!/usr/bin/env python3
"""Per-kernel durations from a rocprofv3 --kernel-trace CSV, split into the warm-up and the timed launches.

usage: python trace_summary.py gpurun_out/prof/stats_kernel_trace.csv --warmup 1 --bench gpurun_out/b.json
       [--out profiles/round1/kernel_trace_cfg3a.json]

rocprofv3's --stats table averages every dispatch, including bench.py's warm-up launches (the first pass over
a freshly written 64 GiB batch runs ~10 % slower).  bench.py's own kernel time (HIP events on the launch
stream) covers only the timed launches, so this script reports both averages for the CRC kernel, and the
ratio of the timed-launch average to bench.py's `roofline.kernel_avg_ms` when --bench is given.
"""
import argparse
import csv
import json
import statistics

CRC_KERNELS = ("crc32c_pieces_kernel", "crc32c_narrow_kernel", "crc32c_narrow_claim_kernel", "crc32c_narrow_sorted_kernel")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--warmup", type=int, default=1, help="warm-up launches of the CRC kernel to set apart")
    ap.add_argument("--last", type=int, default=0,
                    help="take only the last N launches as the timed ones (graph-replay runs: warm-up steps and "
                         "the warm replay come first)")
    ap.add_argument("--bench", default=None, help="bench.py JSON line of the same run")
    ap.add_argument("--out", default=None)
    args = ap.parse_args()
    by = {}
    with open(args.trace) as f:
        for row in csv.DictReader(f):
            dur = (int(row["End_Timestamp"]) - int(row["Start_Timestamp"])) / 1e6
            by.setdefault(row["Kernel_Name"], []).append((int(row["Dispatch_Id"]), dur))
    out = {"source": args.trace, "kernels": {}}
    for name, v in by.items():
        v.sort()
        ms = [d for _, d in v]
        e = {"calls": len(ms), "avg_ms_all": statistics.mean(ms), "min_ms": min(ms), "max_ms": max(ms)}
        if any(k in name for k in CRC_KERNELS) and len(ms) > args.warmup:
            cut = len(ms) - args.last if args.last and len(ms) > args.last else args.warmup
            timed = ms[cut:]
            e.update({"warmup_ms": ms[:cut][:8], "timed_calls": len(timed),
                      "avg_ms_timed": statistics.mean(timed), "median_ms_timed": statistics.median(timed)})
            out["crc_kernel"] = name
            out["crc_avg_ms_timed"] = e["avg_ms_timed"]
        out["kernels"][name] = e
    if args.bench and "crc_avg_ms_timed" in out:
        b = json.loads(open(args.bench).read().strip().splitlines()[-1])
        out["bench_kernel_avg_ms"] = b["roofline"]["kernel_avg_ms"]
        out["rocprof_over_bench"] = out["crc_avg_ms_timed"] / b["roofline"]["kernel_avg_ms"]
    s = json.dumps(out, indent=1)
    if args.out:
        open(args.out, "w").write(s + "\n")
    print(s)


if __name__ == "__main__":
    main()
