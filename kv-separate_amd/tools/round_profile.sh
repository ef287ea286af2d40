# One GPU call: default bench + per-config benches + rocprofv3 kernel stats + separate PMC passes.
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
timeout -k 10 400 python bench.py > gpurun_out/bench_default.json 2> gpurun_out/bench_default.err || exit 1
for c in 3b 4 2; do
  timeout -k 10 400 python bench.py --config $c --steps 10 --warmup 2 --no-cpu --roundtrip-gib 0 > gpurun_out/bench_cfg$c.json 2>/dev/null || exit 1
done
export TMPDIR=/tmp
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof -o stats --output-format csv -- python3 $R/bench.py --steps 5 --warmup 1 --no-cpu --roundtrip-gib 0 > $R/gpurun_out/prof.log 2>&1 || exit 1
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d $R/gpurun_out/pmc1 -o pmc --output-format csv -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu --roundtrip-gib 0 > $R/gpurun_out/pmc1.log 2>&1 || exit 1
timeout -k 10 400 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum --kernel-trace -d $R/gpurun_out/pmc2 -o pmc --output-format csv -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu --roundtrip-gib 0 > $R/gpurun_out/pmc2.log 2>&1 || exit 1
timeout -k 10 400 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAVES --kernel-trace -d $R/gpurun_out/pmc3 -o pmc --output-format csv -- python3 $R/bench.py --config 2 --steps 3 --warmup 1 --no-cpu --roundtrip-gib 0 > $R/gpurun_out/pmc3.log 2>&1 || exit 1
echo done
