#!/bin/bash
# HBM traffic of the CRC kernel for the given bench configs: separate FETCH_SIZE and TCC_EA0_RDREQ_sum passes (each
# with --kernel-trace only), summarised into gpurun_out/pmc_cfg<c>.json.  usage: bash pmc_configs.sh 3b 4
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out
mkdir -p $O
export TMPDIR=/tmp
cd /tmp
B="$R/bench.py --pmc-live off --steps 3 --warmup 1 --no-cpu --roundtrip-gib 0"
for c in "$@"; do
  timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d $O/pmc_fetch_$c -o pmc --output-format csv -- python3 $B --config $c > $O/pmc_fetch_$c.log 2>&1 || exit 1
  timeout -k 10 300 rocprofv3 --pmc TCC_EA0_RDREQ_sum --kernel-trace -d $O/pmc_rdreq_$c -o pmc --output-format csv -- python3 $B --config $c > $O/pmc_rdreq_$c.log 2>&1 || exit 1
  cd $R
  python kv-separate_amd/tools/pmc_summary.py --config $c --fetch $O/pmc_fetch_$c --rdreq $O/pmc_rdreq_$c --out $O/pmc_cfg$c.json --source "rocprofv3 --pmc FETCH_SIZE / --pmc TCC_EA0_RDREQ_sum, each with --kernel-trace only, python3 bench.py --config $c --steps 3 --warmup 1 --no-cpu --roundtrip-gib 0" || exit 1
  cd /tmp
done
echo done
