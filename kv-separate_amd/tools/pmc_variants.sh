# PMC instruction/wait counters of one uniform-block batch, one pass per KVSEP_CRC_VARIANT given.
# usage: bash pmc_variants.sh <block_len> <count> <variant>...
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
export TMPDIR=/tmp
cd /tmp
BL=$1; CNT=$2; shift 2
for v in "$@"; do
  export KVSEP_CRC_VARIANT=$v
  timeout -k 10 200 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY --kernel-trace -d $R/gpurun_out/pmcv$v -o pmc --output-format csv -- python3 $R/kv-separate_amd/tools/one_batch.py $BL $CNT 5 > $R/gpurun_out/pmcv$v.log 2>&1 || exit 1
done
echo ok
