#!/usr/bin/env python3
"""One line per bench JSON file (last line of each): value, kernel GB/s, roofline fraction."""
import json
import sys

for f in sorted(sys.argv[1:]):
    try:
        d = json.loads(open(f).read().strip().splitlines()[-1])
    except Exception as e:  # noqa: BLE001
        print(f, "ERR", e)
        continue
    r = d["roofline"]
    print(f"{f:40s} {d['value']:9.1f} GiB/s {d['ms_per_step']:8.3f} ms  kern {r['achieved']:7.1f} GB/s "
          f"frac {r['frac']:.4f} ceil {d['read_ceiling_GBps']} ({d['frac_of_read_ceiling']}) "
          f"par {d.get('parity') or d['parity_spot_check']} rt {d['host_roundtrip_GiBps']} cpu {(d['cpu_baseline'] or {}).get('value')}")
