#!/usr/bin/env python3
"""The reference's own CRC measurement convention, three ways on one box.

db_bench --benchmarks=crc32c (benchmarks/db_bench.cc:693-710) checksums 4 KiB of 'x' with crc32c::Value, repeated until
500 MiB are done (128,000 calls), and reports MB/s with MB = 2^20 (db_bench.cc:320-321).  Here:
  reference   oracle/_ref/dbbench_crc32c_ref: that loop (tools/dbbench_crc32c.cc) linked with the reference's
              util/crc32c.cc (portable path, -O3) -- what db_bench prints for this fork on this host
  drop-in     tools/dbbench_crc32c_kvsep: the same loop linked with libkvsep_leveldb_abi.so, i.e. the link-level
              drop-in; a 4 KiB Extend runs on the library's host leg (a single call cannot win on the GPU): the
              VPCLMULQDQ fold where the CPU has it ("dropin"), and the SSE4.2 crc32q loop (KVSEP_HOST_CRC=sse42,
              "dropin_sse42")
  device      the same 128,000 blocks as ONE batched call (kvsep_crc32c_batch_device): 500 MiB of 'x' resident in
              HBM, 128,000 descriptors, the north star's block batch; K calls captured into one hipGraph, HIP events
  host batch  the same 128,000 blocks from a pinned host buffer (kvsep_crc32c_batch_host_span: H2D + kernel + D2H)
Every path's CRCs are checked: all 128,000 results equal the reference binary's printed value.
usage: dbbench_crc32c.py [--reps 5] [--steps 20]"""
import argparse
import json
import os
import statistics
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.abspath(os.path.join(HERE, "..", ".."))
sys.path.insert(0, os.path.join(HERE, ".."))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import kvsep  # noqa: E402

SIZE, TOTAL = 4096, 500 * 1048576
OPS = TOTAL // SIZE
MB = 1048576.0


def run_binary(path, reps, env=None):
    if not os.path.exists(path):
        return None
    lines = subprocess.run([path, str(reps)], capture_output=True, text=True, check=True, timeout=600,
                           env=dict(os.environ, **(env or {}))).stdout
    runs = [json.loads(l) for l in lines.splitlines() if l.startswith("{")]
    return {"MBps_median": round(statistics.median(r["MBps"] for r in runs), 1),
            "MBps_runs": [r["MBps"] for r in runs], "crc": runs[0]["crc"], "ops": runs[0]["ops"],
            "threads": 1}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--steps", type=int, default=20)
    args = ap.parse_args()
    out = {"convention": "db_bench --benchmarks=crc32c: 4 KiB of 'x', Value repeated to 500 MiB (128,000 calls), "
                         "MB/s with MB = 2^20 (benchmarks/db_bench.cc:693-710, :320-321)"}
    out["reference"] = run_binary(os.path.join(ROOT, "oracle", "_ref", "dbbench_crc32c_ref"), args.reps)
    out["dropin"] = run_binary(os.path.join(HERE, "dbbench_crc32c_kvsep"), args.reps)
    out["dropin_sse42"] = run_binary(os.path.join(HERE, "dbbench_crc32c_kvsep"), args.reps, {"KVSEP_HOST_CRC": "sse42"})
    want = int((out["reference"] or out["dropin"])["crc"], 16)
    for k in ("dropin", "dropin_sse42"):
        if out[k]:
            out[k]["crc_equals_reference"] = int(out[k]["crc"], 16) == want

    dev = torch.device("cuda:0")
    ctx = kvsep.Context(0)
    data = torch.full((TOTAL + 64,), ord("x"), dtype=torch.uint8, device=dev)
    off = torch.arange(OPS, dtype=torch.int64, device=dev) * SIZE
    ln = torch.full((OPS,), SIZE, dtype=torch.int64, device=dev)
    res = torch.zeros(OPS, dtype=torch.int32, device=dev)
    ctx.reserve(OPS, TOTAL)

    def call(st):
        ctx.batch_device(data.data_ptr(), off, ln, res, count=OPS, total_bytes=TOTAL, max_len=SIZE, stream=st)

    call(torch.cuda.current_stream())
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(args.steps):
            call(torch.cuda.current_stream())
    g.replay()
    torch.cuda.synchronize()
    per = []
    for _ in range(args.reps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        g.replay()
        e1.record()
        torch.cuda.synchronize()
        per.append(e0.elapsed_time(e1) * 1e-3 / args.steps)
    crcs = res.cpu().numpy().view(np.uint32)
    out["device_batch"] = {"MBps_median": round(TOTAL / MB / statistics.median(per), 1),
                           "us_per_call_median": round(statistics.median(per) * 1e6, 2),
                           "kernel": ctx.kernel_name(OPS, SIZE, TOTAL), "calls_per_graph": args.steps,
                           "all_crcs_equal_reference": bool((crcs == want).all()), "blocks": OPS}

    host = torch.full((TOTAL,), ord("x"), dtype=torch.uint8).pin_memory().numpy()
    hoff = np.arange(OPS, dtype=np.uint64) * np.uint64(SIZE)
    hln = np.full(OPS, SIZE, np.uint64)
    ctx.batch_host_span(host, hoff, hln)  # warm the staging
    import time
    ts = []
    for _ in range(args.reps):
        t0 = time.perf_counter()
        h = ctx.batch_host_span(host, hoff, hln)
        ts.append(time.perf_counter() - t0)
    out["host_batch"] = {"MBps_median": round(TOTAL / MB / statistics.median(ts), 1),
                         "form": "kvsep_crc32c_batch_host_span from pinned host memory (H2D + kernel + D2H)",
                         "all_crcs_equal_reference": bool((h == want).all())}
    out["crc"] = hex(want)
    ctx.close()
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
