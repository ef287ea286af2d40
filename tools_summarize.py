import json,sys,glob
for f in sorted(sys.argv[1:]):
    try:
        d=json.loads(open(f).read().strip().splitlines()[-1])
    except Exception as e:
        print(f, "ERR", e); continue
    r=d['roofline']
    print(f"{f:32s} {d['value']:9.1f} GiB/s {d['ms_per_step']:8.3f} ms  kern {r['achieved']:7.1f} GB/s frac {r['frac']:.4f} ceil {d['read_ceiling_GBps']:7.1f} ({d['frac_of_read_ceiling']:.3f}) par {d['parity_spot_check']} rt {d['host_roundtrip_GiBps']} cpu {(d['cpu_baseline'] or {}).get('value')}")
