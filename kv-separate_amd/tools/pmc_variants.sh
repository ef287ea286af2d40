set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
export TMPDIR=/tmp
cd /tmp
for v in 1 8 9; do
  export KVSEP_CRC_VARIANT=$v
  timeout -k 10 200 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY --kernel-trace -d $R/gpurun_out/pmcv$v -o pmc --output-format csv -- python3 $R/kv-separate_amd/tools/one_batch.py 4096 65536 5 > $R/gpurun_out/pmcv$v.log 2>&1 || exit 1
done
echo ok
