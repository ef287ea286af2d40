# One GPU call: rocprofv3 --kernel-trace --stats of configs 3b, 4 and 5 (eager launches, so every CRC launch is its
# own dispatch), each next to bench.py's own HIP-event kernel time of the same run (trace_summary.py).
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out
mkdir -p $O
export TMPDIR=/tmp
cd /tmp
for c in 3b 4; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_$c -o stats --output-format csv -- python3 $R/bench.py --config $c --steps 20 --warmup 1 --no-cpu --roundtrip-gib 0 --launch eager --pmc-live off > $O/prof_$c.json 2> $O/prof_$c.err || exit 1
done
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof_5 -o stats --output-format csv -- python3 $R/bench.py --config 5 --steps 2 --warmup 1 --no-cpu --roundtrip-gib 0 --pmc-live off > $O/prof_5.json 2> $O/prof_5.err || exit 1
cd $R
python kv-separate_amd/tools/trace_summary.py $O/prof_3b/stats_kernel_trace.csv --warmup 1 --bench $O/prof_3b.json --out $O/kernel_trace_cfg3b.json > /dev/null || exit 1
python kv-separate_amd/tools/trace_summary.py $O/prof_4/stats_kernel_trace.csv --warmup 1 --bench $O/prof_4.json --out $O/kernel_trace_cfg4.json > /dev/null || exit 1
python kv-separate_amd/tools/trace_summary.py $O/prof_5/stats_kernel_trace.csv --warmup 8 --bench $O/prof_5.json --out $O/kernel_trace_cfg5.json > /dev/null || exit 1
echo done
