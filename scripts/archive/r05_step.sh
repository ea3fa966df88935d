# round-5 GPU step: the whole -m gpu suite, the default bench line, and a rocprofv3 kernel trace of the same bench
# command with the breakdown launches (the ones roofline.kernel_ms times) selected from it
set -o pipefail
O=${1:-gpurun_out/r05}
mkdir -p $O
R=$PWD
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests > $O/gpu_tests.log 2>&1 || { tail -40 $O/gpu_tests.log; exit 1; }
tail -2 $O/gpu_tests.log
timeout -k 10 400 python bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
echo "bench done"; cat $O/bench.json | cut -c1-400
( cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/$O/prof_bench -o run -- python $R/bench.py --no-cpu-baseline > $R/$O/prof_bench.json 2> $R/$O/prof_bench.log ) || { tail $O/prof_bench.log; exit 1; }
python3 scripts/rocpd_stats.py $O/prof_bench/run_results.db > $O/bench_kernel_stats.csv
python3 scripts/breakdown_launches.py $O/prof_bench/run_results.db $O/prof_bench.json > $O/breakdown_launches.json
cat $O/breakdown_launches.json
echo "all done"
