set -o pipefail
for g in 0 50 100; do
  RLNC_BSJ_GUIDED=$g timeout -k 10 120 python -m pytest tests/test_gpu_parity.py -m gpu -q -x -k column_runs -p no:cacheprovider > gpurun_out/guided_test_$g.log 2>&1 || { echo "test g=$g failed"; tail -20 gpurun_out/guided_test_$g.log; exit 1; }
  tail -1 gpurun_out/guided_test_$g.log
done
AB="v8::--no-ceiling v9::--variant,9,--no-ceiling g50:RLNC_BSJ_GUIDED=50:--variant,9,--no-ceiling g75:RLNC_BSJ_GUIDED=75:--variant,9,--no-ceiling g90:RLNC_BSJ_GUIDED=90:--variant,9,--no-ceiling g75p1:RLNC_BSJ_GUIDED=75:--variant,9,--pipeline,1,--no-ceiling" bash scripts/bench_ab.sh > gpurun_out/ab_guided.txt 2>&1
