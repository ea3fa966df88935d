# round 6, at the last commit: the GPU suite, smoke and the default bench line (run on more than one box for the spread)
set -o pipefail
O=${1:-gpurun_out/r06_head_a}
mkdir -p $O
timeout -k 10 900 python -u -m pytest -q --timeout 120 --timeout-method thread -m gpu tests > $O/gpu_tests.log 2>&1
rc=$?; tail -1 $O/gpu_tests.log
[ $rc -le 1 ] || { tail -60 $O/gpu_tests.log; exit $rc; }
grep -E "FAILED|ERROR" $O/gpu_tests.log | head -20
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { tail $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 400 python bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
grep '^{' $O/bench.json | cut -c1-300
echo "all done"
