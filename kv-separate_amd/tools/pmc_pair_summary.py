#!/usr/bin/env python3
"""Per-kernel means of rocprofv3 --pmc counter passes (pmc_counter_collection.csv of each pass directory) for the
kernels a pair script alternates (cfg2_pair.py: config 2's CRC kernel and the streaming-read kernel over the same
allocation), over dispatches `skip`.. of each kernel, plus the per-wave instruction counts and the share of wave-cycles
with an instruction in issue.  usage: pmc_pair_summary.py <out.json> <pass dir>... [--skip N] [--note TEXT]"""
import argparse
import collections
import csv
import json
import os

KERNELS = ("crc32c_narrow_claim_kernel", "stream_read_kernel")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("out")
    ap.add_argument("dirs", nargs="+")
    ap.add_argument("--skip", type=int, default=2)
    ap.add_argument("--note", default="")
    a = ap.parse_args()
    vals = {k: collections.defaultdict(list) for k in KERNELS}
    for d in a.dirs:
        path = None
        for root, _, files in os.walk(d):
            for f in files:
                if f.endswith("counter_collection.csv"):
                    path = os.path.join(root, f)
        if path is None:
            raise SystemExit(f"no counter_collection.csv under {d}")
        per = collections.defaultdict(lambda: collections.defaultdict(float))
        order = collections.defaultdict(list)
        for r in csv.DictReader(open(path)):
            k = next((k for k in KERNELS if k in r["Kernel_Name"]), None)
            if k is None:
                continue
            did = int(r["Dispatch_Id"])
            if did not in order[k]:
                order[k].append(did)
            per[(k, did)][r["Counter_Name"]] += float(r["Counter_Value"])
        for k in KERNELS:
            for did in order[k][a.skip:]:
                for c, v in per[(k, did)].items():
                    vals[k][c].append(v)
    res = {"source": a.note, "kernels": {}, "per_wave": {}}
    for k in KERNELS:
        m = {c: sum(v) / len(v) for c, v in vals[k].items() if v}
        res["kernels"][k] = m
        w = m.get("SQ_WAVES") or 0
        if w:
            res["per_wave"][k] = {"VALU": m.get("SQ_INSTS_VALU", 0) / w, "LDS": m.get("SQ_INSTS_LDS", 0) / w,
                                  "VMEM_RD": m.get("SQ_INSTS_VMEM_RD", 0) / w, "SALU": m.get("SQ_INSTS_SALU", 0) / w,
                                  "active_inst_over_wave_cycles":
                                      m.get("SQ_ACTIVE_INST_ANY", 0) / max(1.0, m.get("SQ_WAVE_CYCLES", 0))}
    json.dump(res, open(a.out, "w"), indent=1)
    print(json.dumps(res["per_wave"], indent=1))


if __name__ == "__main__":
    main()
