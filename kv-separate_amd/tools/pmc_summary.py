#!/usr/bin/env python3
"""Summarise rocprofv3 --pmc passes of bench.py into profiles/pmc_<cfg>.json (and pmc_latest.json for 3a).

usage: python pmc_summary.py --config 3a --fetch gpurun_out/pmc1 --rdreq gpurun_out/pmc2 [--lds gpurun_out/pmc3]
       [--algorithmic BYTES] [--out profiles/round1/pmc_cfg3a.json]

Per-launch HBM bytes of the CRC kernel from two separate counter passes (MI355X_MICROARCH.md, HBM section):
  * FETCH_SIZE (KB) x 1024 x 2   -- gfx950 FETCH_SIZE counts half the bytes of a wide coalesced stream;
  * TCC_EA0_RDREQ_sum x 128 B    -- the same bytes from the L2's fabric read requests (128-B requests).
The last launch of the CRC kernel in each pass is skipped only if there is a single one (warm-up included).
"""
import argparse
import csv
import json
import os
import statistics

CRC_KERNELS = ("crc32c_pieces_kernel", "crc32c_narrow_kernel", "crc32c_narrow_claim_kernel", "crc32c_narrow_sorted_kernel")


def per_launch(path, counter):
    """Mean per-dispatch value of `counter` over the CRC kernel's dispatches in one pass."""
    f = os.path.join(path, "pmc_counter_collection.csv")
    vals, name = {}, None
    with open(f) as fh:
        for row in csv.DictReader(fh):
            if row["Counter_Name"] != counter or not any(k in row["Kernel_Name"] for k in CRC_KERNELS):
                continue
            d = row["Dispatch_Id"]
            vals[d] = vals.get(d, 0.0) + float(row["Counter_Value"])  # sum over XCD/agent instances
            name = row["Kernel_Name"]
    if not vals:
        raise SystemExit(f"{counter}: no CRC kernel dispatch in {f}")
    v = [vals[k] for k in sorted(vals, key=int)]
    return statistics.mean(v), len(v), name


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="3a")
    ap.add_argument("--fetch", required=True)
    ap.add_argument("--rdreq", required=True)
    ap.add_argument("--lds", default=None)
    ap.add_argument("--algorithmic", type=int, default=None, help="sum of block lengths per launch")
    ap.add_argument("--out", required=True)
    ap.add_argument("--source", default="")
    args = ap.parse_args()
    if args.algorithmic is None:
        import sys
        sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
        from kvsep import workloads as W
        lay = {"3a": W.cfg3_layout, "3b": lambda: W.cfg3_layout(vlog=True), "2": W.cfg2_layout,
               "4": W.cfg4_layout}[args.config]
        args.algorithmic = int(lay()[1].sum())
    fetch_kb, n1, kname = per_launch(args.fetch, "FETCH_SIZE")
    rdreq, n2, _ = per_launch(args.rdreq, "TCC_EA0_RDREQ_sum")
    hbm = fetch_kb * 1024 * 2
    out = {
        "config": args.config,
        "kernel": kname,
        "launches": [n1, n2],
        "FETCH_SIZE_KB_per_launch": fetch_kb,
        "correction": "gfx950 FETCH_SIZE counts half the bytes of a wide coalesced stream "
                      "(MI355X_MICROARCH.md HBM): bytes = FETCH_SIZE*1024*2",
        "hbm_bytes_per_launch": int(hbm),
        "TCC_EA0_RDREQ_sum_per_launch": rdreq,
        "rdreq_bytes_at_128B": rdreq * 128,
        "algorithmic_bytes_per_launch": args.algorithmic,
        "traffic_over_algorithmic": hbm / args.algorithmic,
        "source": args.source,
    }
    if args.lds:
        conf, _, _ = per_launch(args.lds, "SQ_LDS_BANK_CONFLICT")
        act, _, _ = per_launch(args.lds, "SQ_LDS_IDX_ACTIVE")
        out["SQ_LDS_BANK_CONFLICT_per_launch"] = conf
        out["SQ_LDS_IDX_ACTIVE_per_launch"] = act
        out["lds_conflict_fraction"] = conf / act if act else None
    os.makedirs(os.path.dirname(os.path.abspath(args.out)), exist_ok=True)
    with open(args.out, "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
