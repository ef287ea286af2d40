#!/bin/bash
# Round 6: config 2's CRC kernel next to the streaming-read kernel over the same allocation (cfg2_pair.py), counters in
# three separate rocprofv3 --pmc passes (no trace domains; each pass within the per-block counter limits: 8 SQ / 8 SQ /
# 4 TCC-TCP-TA), summarised per kernel and per wave by pmc_pair_summary.py into gpurun_out/pmc_pair/pmc_cfg2_pair.json.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
O=gpurun_out/pmc_pair
mkdir -p $O
A="SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAVES SQ_WAVE_CYCLES"
B="SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_WAVES"
C="TA_BUSY_avr TCC_HIT_sum TCC_MISS_sum TCP_TCC_READ_REQ_sum"
i=0
for P in "$A" "$B" "$C"; do
  i=$((i + 1))
  timeout -s KILL 120 rocprofv3 --pmc $P --kernel-trace --output-format csv -d $O/p$i -o pmc -- python3 kv-separate_amd/tools/cfg2_pair.py 10 \
    > $O/p$i.log 2>&1 || { tail -20 $O/p$i.log; exit 1; }
done
python3 kv-separate_amd/tools/pmc_pair_summary.py $O/pmc_cfg2_pair.json $O/p1 $O/p2 $O/p3 \
  --note "rocprofv3 --pmc <group> --kernel-trace, three separate passes, python3 kv-separate_amd/tools/cfg2_pair.py 10 (config 2's CRC kernel and the streaming-read kernel alternating over the same 256 MiB); mean per dispatch of dispatches 3-10"
