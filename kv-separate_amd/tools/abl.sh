mkdir -p gpurun_out
timeout -k 10 500 python -m pytest tests -m gpu -q --maxfail=3 > gpurun_out/gpu_tests.log 2>&1 || exit 1
timeout -k 10 200 python kv-separate_amd/tools/small_blocks_probe.py > gpurun_out/sb.txt 2>&1 || exit 1
timeout -k 10 500 python kv-separate_amd/tools/ab_variants.py --variants 1,2 --configs 2,3a,4,3b --rounds 3 --steps 4 > gpurun_out/ab.txt 2>&1 || exit 1
