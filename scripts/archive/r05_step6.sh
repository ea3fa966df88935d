# round-5 GPU step 6: small-object elimination parity + timing, configs[0] decode and its rocprofv3 kernel breakdown
set -o pipefail
O=${1:-gpurun_out/r05g}
mkdir -p $O
R=$PWD
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_parity.py -k "small or decode" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 120 python scripts/elim_small_probe.py > $O/elim.jsonl 2>/dev/null || exit 1
cat $O/elim.jsonl
for i in 1 2 3; do CONFIGS=0 timeout -k 10 120 python scripts/bench_configs.py >> $O/configs0.jsonl 2>/dev/null || exit 1; done
cat $O/configs0.jsonl
( cd /tmp && export TMPDIR=/tmp && CONFIGS=0 timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $R/$O/prof -o run -- python $R/scripts/bench_configs.py > $R/$O/prof.log 2>&1 ) || { tail $O/prof.log; exit 1; }
python3 scripts/rocpd_stats.py $O/prof/run_results.db > $O/cfg0_kernel_stats.csv
cat $O/cfg0_kernel_stats.csv
echo "all done"
