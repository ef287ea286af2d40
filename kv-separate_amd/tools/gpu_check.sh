#!/bin/bash
# One GPU call: the -m gpu suite, then short bench lines of the given configs (default 3a and 2).
# usage: bash kv-separate_amd/tools/gpu_check.sh [configs...]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
  > gpurun_out/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -3 gpurun_out/pytest_gpu.log
for c in "${@:-3a 2}"; do
  timeout -k 10 300 python -u bench.py --config $c --no-cpu --roundtrip-gib 0 > gpurun_out/bench_$c.json 2> gpurun_out/bench_$c.err || { tail -20 gpurun_out/bench_$c.err; exit 1; }
  cat gpurun_out/bench_$c.json
done
