#!/bin/bash
# Instruction-mix PMC of narrow-kernel variants (KVSEP_DIAG build) on one uniform batch: per variant one --pmc pass
# (kernel trace only) over tools/one_batch.py, summarised per CRC kernel launch.
# usage: bash pmc_ab.sh <block_len> <count> <narrow variant> ...
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out
mkdir -p $O
export TMPDIR=/tmp
cd /tmp
L=$1; N=$2; shift 2
for v in "$@"; do
  KVSEP_NARROW=$v timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM SQ_INSTS_BRANCH SQ_WAVES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY --kernel-trace -d $O/pmcab_$v -o pmc --output-format csv -- python3 $R/kv-separate_amd/tools/one_batch.py $L $N 5 > $O/pmcab_$v.log 2>&1 || exit 1
  python3 - $O/pmcab_$v $v <<'PY' || exit 1
import csv, glob, sys, collections
f = glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True)[0]
acc = collections.defaultdict(list)
for r in csv.DictReader(open(f)):
    if "crc32c_narrow" in r["Kernel_Name"]:
        acc[r["Counter_Name"]].append(float(r["Counter_Value"]))
print(f"variant {sys.argv[2]}: " + "  ".join(f"{k} {sum(v) / len(v):.4g}" for k, v in sorted(acc.items())), flush=True)
PY
done
