# Copy the judged artefacts of one round_profile.sh call from gpurun_out/ into profiles/<round>/ (tracked),
# and the per-config PMC summaries that bench.py reads for roofline.traffic into profiles/.
# usage: bash kv-separate_amd/tools/collect_profiles.sh round1
set -e
R=$(cd "$(dirname "$0")/../.." && pwd)
O=$R/gpurun_out
D=$R/profiles/${1:?round name}
mkdir -p $D
cp $O/bench_default.json $D/bench_default.json
for c in 3b 4 2 5; do cp $O/bench_cfg$c.json $D/bench_cfg$c.json; done
cp $O/launch_floor.txt $D/launch_floor.txt
cp $O/framing_bench.json $D/framing_bench.json
cp $O/prof/stats_kernel_stats.csv $D/kernel_stats_cfg3a.csv
cp $O/prof/stats_kernel_trace.csv $D/kernel_trace_cfg3a.csv
cp $O/kernel_trace_cfg3a.json $D/kernel_trace_cfg3a.json
cp $O/prof.json $D/bench_under_rocprof_cfg3a.json
cp $O/prof2/stats_kernel_stats.csv $D/kernel_stats_cfg2.csv
cp $O/kernel_trace_cfg2.json $D/kernel_trace_cfg2.json
for c in 3a 3b 4 2; do
  cp $O/pmc_cfg$c.json $D/pmc_cfg$c.json
  cp $O/pmc_cfg$c.json $R/profiles/pmc_cfg$c.json
  cp $O/pmc_fetch_$c/pmc_counter_collection.csv $D/pmc_fetch_size_cfg$c.csv
  cp $O/pmc_rdreq_$c/pmc_counter_collection.csv $D/pmc_rdreq_cfg$c.csv
done
cp $O/pmc_lds_2/pmc_counter_collection.csv $D/pmc_lds_cfg2.csv
echo "collected into $D"
