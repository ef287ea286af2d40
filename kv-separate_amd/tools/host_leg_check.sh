#!/bin/bash
# One GPU-box call for the host leg: its per-size rates with the fold and with the SSE4.2 loop (host_leg_bench),
# db_bench's crc32c convention four ways (dbbench_crc32c.py), the drop-in's GPU crossover (dropin_probe.py), and the GPU tests that drive the scalar drop-in.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out/host_leg
grep -m1 "model name" /proc/cpuinfo > gpurun_out/host_leg/cpu.txt
grep -m1 "^flags" /proc/cpuinfo | tr ' ' '\n' | grep -E "^(avx512f|vpclmulqdq|pclmulqdq|sse4_2)$" >> gpurun_out/host_leg/cpu.txt
for m in default sse42; do
  KVSEP_HOST_CRC=$m timeout -k 10 120 ./kv-separate_amd/tools/host_leg_bench 1024 > gpurun_out/host_leg/host_leg_$m.jsonl || exit 1
done
timeout -k 10 300 python -u kv-separate_amd/tools/dbbench_crc32c.py > gpurun_out/host_leg/dbbench_crc32c.json || exit 1
timeout -k 10 300 python -u kv-separate_amd/tools/dropin_probe.py gpurun_out/host_leg/dropin_crossover.json \
  > gpurun_out/host_leg/dropin_crossover.jsonl || exit 1
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_parity.py \
  tests/test_gpu_concurrency.py tests/test_refcallsites.py tests/test_abi_cpu.py > gpurun_out/host_leg/pytest.log 2>&1 \
  || { tail -30 gpurun_out/host_leg/pytest.log; exit 1; }
tail -2 gpurun_out/host_leg/pytest.log
cat gpurun_out/host_leg/cpu.txt gpurun_out/host_leg/host_leg_*.jsonl gpurun_out/host_leg/dbbench_crc32c.json
