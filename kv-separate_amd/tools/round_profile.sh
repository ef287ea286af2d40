# One GPU call: parity tests, default bench + per-config benches, rocprofv3 kernel stats, and separate PMC
# passes per config (one counter group per run, --kernel-trace only), summarised into gpurun_out/pmc_cfg*.json.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out
mkdir -p $O
cd $R
timeout -k 10 400 python bench.py > $O/bench_default.json 2> $O/bench_default.err || exit 1
timeout -k 10 400 python -u kv-separate_amd/tools/framing_bench.py --out $O/framing_bench.json > $O/framing_bench.log 2>&1 || exit 1
for c in 3b 4 2 5; do
  timeout -k 10 400 python bench.py --config $c --steps 10 --warmup 2 --no-cpu --roundtrip-gib 0 > $O/bench_cfg$c.json 2>$O/bench_cfg$c.err || exit 1
done
timeout -k 10 300 python -u kv-separate_amd/tools/launch_floor_probe.py 64 256 1024 4096 > $O/launch_floor.txt 2>&1 || exit 1
export TMPDIR=/tmp
cd /tmp
B="$R/bench.py --steps 3 --warmup 1 --no-cpu --roundtrip-gib 0 --pmc-live off"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof -o stats --output-format csv -- python3 $R/bench.py --steps 20 --warmup 1 --no-cpu --roundtrip-gib 0 --launch eager --pmc-live off > $O/prof.json 2> $O/prof.err || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof2 -o stats --output-format csv -- python3 $R/bench.py --config 2 --steps 20 --warmup 1 --no-cpu --roundtrip-gib 0 --pmc-live off > $O/prof2.json 2> $O/prof2.err || exit 1
for c in 3a 3b 4 2; do
  timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d $O/pmc_fetch_$c -o pmc --output-format csv -- python3 $B --config $c > $O/pmc_fetch_$c.log 2>&1 || exit 1
  timeout -k 10 300 rocprofv3 --pmc TCC_EA0_RDREQ_sum --kernel-trace -d $O/pmc_rdreq_$c -o pmc --output-format csv -- python3 $B --config $c > $O/pmc_rdreq_$c.log 2>&1 || exit 1
done
timeout -k 10 300 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE --kernel-trace -d $O/pmc_lds_2 -o pmc --output-format csv -- python3 $B --config 2 > $O/pmc_lds_2.log 2>&1 || exit 1
cd $R
for c in 3a 3b 4 2; do
  L=""; [ $c = 2 ] && L="--lds $O/pmc_lds_2"
  python kv-separate_amd/tools/pmc_summary.py --config $c --fetch $O/pmc_fetch_$c --rdreq $O/pmc_rdreq_$c $L --out $O/pmc_cfg$c.json --source "rocprofv3 --pmc FETCH_SIZE / --pmc TCC_EA0_RDREQ_sum, each with --kernel-trace only, python3 bench.py --config $c --steps 3 --warmup 1 --no-cpu --roundtrip-gib 0" > /dev/null || exit 1
done
python kv-separate_amd/tools/trace_summary.py $O/prof/stats_kernel_trace.csv --warmup 1 --bench $O/prof.json --out $O/kernel_trace_cfg3a.json > /dev/null || exit 1
python kv-separate_amd/tools/trace_summary.py $O/prof2/stats_kernel_trace.csv --last 20 --bench $O/prof2.json --out $O/kernel_trace_cfg2.json > /dev/null || exit 1
echo done
