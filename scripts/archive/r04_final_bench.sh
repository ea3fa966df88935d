# round-4 final measurements (after the tests): bench.py with CPU baselines, its rocprof kernel trace + stats, the
# per-launch overlap of the decode-side elimination, PMC traffic passes, every config, ragged rates
set -o pipefail
mkdir -p gpurun_out/final
R=$PWD
timeout -k 10 400 python bench.py > gpurun_out/final/bench.json 2> gpurun_out/final/bench.err || { tail -20 gpurun_out/final/bench.err; exit 1; }
echo "bench done"
( cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/final/prof_bench -o run -- python $R/bench.py --no-cpu-baseline > $R/gpurun_out/final/prof_bench.log 2>&1 ) || exit 1
python3 scripts/rocpd_stats.py gpurun_out/final/prof_bench/run_results.db > gpurun_out/final/bench_kernel_stats.csv
python3 scripts/launch_overlap.py gpurun_out/final/prof_bench/run_results.db --match gf_rref_block_kernel > gpurun_out/final/rref_overlap.csv
echo "rocprof done"
timeout -k 10 400 bash scripts/pmc_bench.sh > gpurun_out/final/pmc.log 2>&1 || { tail gpurun_out/final/pmc.log; exit 1; }
cp -r gpurun_out/pmc_bench/summary.jsonl gpurun_out/final/pmc_summary.jsonl
echo "pmc done"
timeout -k 10 400 python scripts/bench_configs.py > gpurun_out/final/configs.jsonl 2> gpurun_out/final/configs.err || { tail gpurun_out/final/configs.err; exit 1; }
echo "configs done"
timeout -k 10 120 python scripts/ragged_rate.py > gpurun_out/final/ragged_rate.jsonl 2>/dev/null || exit 1
echo "all done"
