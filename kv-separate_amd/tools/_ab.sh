set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out; mkdir -p $O; cd $R
timeout -k 10 400 python -u kv-separate_amd/tools/ab_variants.py --variants 1,b1 --configs 2,u16384x4096,u32768x4096,u4096x65536,u1000x100000,u256x1048576,u20000x1000,u3000x4096 --rounds 5 --steps 10 > $O/ab_wm.txt 2>&1 || exit 1
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests -m gpu > $O/ab_tests.log 2>&1 || exit 1
echo done
