set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out; mkdir -p $O; cd $R
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests -m gpu > $O/ab_tests.log 2>&1 || exit 1
timeout -k 10 600 python -u kv-separate_amd/tools/ab_variants.py --variants 1,b1 --configs 2,u8192x4096,u16384x16384,u32768x32768,u32768x16384,4,3a --rounds 3 --steps 5 > $O/ab_thr.txt 2>&1 || exit 1
echo done
