# round-5 GPU step 7: whole -m gpu suite, then configs[0] decode (3 runs) and its kernel breakdown
set -o pipefail
O=${1:-gpurun_out/r05i}
mkdir -p $O
R=$PWD
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests > $O/gpu_tests.log 2>&1 || { tail -40 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
for i in 1 2 3; do CONFIGS=0 timeout -k 10 120 python scripts/bench_configs.py >> $O/configs0.jsonl 2>/dev/null || exit 1; done
cat $O/configs0.jsonl | cut -c1-330
( cd /tmp && export TMPDIR=/tmp && CONFIGS=0 timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $R/$O/prof -o run -- python $R/scripts/bench_configs.py > $R/$O/prof.log 2>&1 ) || { tail $O/prof.log; exit 1; }
python3 scripts/rocpd_stats.py $O/prof/run_results.db > $O/cfg0_kernel_stats.csv
head -6 $O/cfg0_kernel_stats.csv
echo "all done"
