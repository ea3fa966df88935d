# round 6 checkpoint / closing measurements at head: both GPU suites (shipped + A/B build), smoke, the default bench
# line, a rocprofv3 kernel trace of the same command with the encode and decode breakdown launches selected, the PMC
# traffic passes, every config, configs[4] at N = 1 and N = 2 (both ranks on the lease's GPU), the object-API grid
set -o pipefail
O=${1:-gpurun_out/r06_ck}
mkdir -p $O
R=$PWD
timeout -k 10 900 python -u -m pytest -q --timeout 120 --timeout-method thread -m gpu tests > $O/gpu_tests.log 2>&1
rc=$?; tail -1 $O/gpu_tests.log
[ $rc -le 1 ] || { tail -60 $O/gpu_tests.log; exit $rc; }
grep -E "FAILED|ERROR" $O/gpu_tests.log | head -20
RLNC_LIB_PATH=$R/rlnc_amd/librlnc_hip_ab.so timeout -k 10 600 python -u -m pytest -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_fullrange.py tests/test_gpu_graph.py > $O/ab_tests.log 2>&1
rc=$?; tail -1 $O/ab_tests.log
[ $rc -le 1 ] || { tail -40 $O/ab_tests.log; exit $rc; }
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { tail $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 400 python bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
grep '^{' $O/bench.json | cut -c1-300
( cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/$O/prof_bench -o run -- python $R/bench.py --no-cpu-baseline > $R/$O/prof_bench.json 2> $R/$O/prof_bench.log ) || { tail $O/prof_bench.log; exit 1; }
python3 scripts/rocpd_stats.py $O/prof_bench/run_results.db > $O/bench_kernel_stats.csv
python3 scripts/breakdown_launches.py $O/prof_bench/run_results.db $O/prof_bench.json > $O/breakdown_launches.json
python3 scripts/breakdown_launches.py $O/prof_bench/run_results.db $O/prof_bench.json --decode > $O/breakdown_launches_decode.json
cat $O/breakdown_launches.json $O/breakdown_launches_decode.json | cut -c1-400
rm -rf $O/prof_bench
bash scripts/pmc_bench.sh || exit $?
cp -r gpurun_out/pmc_bench $O/pmc_bench
timeout -k 10 400 python scripts/bench_configs.py > $O/configs.jsonl 2> $O/configs.err || { tail $O/configs.err; exit 1; }
cut -c1-200 $O/configs.jsonl
timeout -k 10 400 python bench.py --workload config5 --no-cpu-baseline > $O/config5_n1.json 2> $O/config5_n1.err || { tail -20 $O/config5_n1.err; exit 1; }
grep '^{' $O/config5_n1.json | cut -c1-200
timeout -k 10 500 python bench.py --gpus 2 --workload config5 --no-cpu-baseline --no-ceiling > $O/config5_n2_onegpu.json 2> $O/config5_n2_onegpu.err || { tail -20 $O/config5_n2_onegpu.err; exit 1; }
grep '^{' $O/config5_n2_onegpu.json | cut -c1-200
timeout -k 10 600 build/object_api_bench > $O/object_api_grid.jsonl 2> $O/object_api_grid.err || { tail $O/object_api_grid.err; exit 1; }
echo "all done"
