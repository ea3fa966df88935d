# round-5 GPU step 4: the small-object elimination's work queue -- parity tests, waves-per-SIMD A/B, timeline, the
# configs[0] decode
set -o pipefail
O=${1:-gpurun_out/r05d}
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_parity.py -k "small or queue" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for q in 0 1 2 3 4 5; do
  RLNC_SMALL_QUEUE=$q timeout -k 10 120 python scripts/elim_small_probe.py 2>/dev/null | sed "s/^{/{\"queue_waves_per_simd\": $q, /" >> $O/queue_ab.jsonl || exit 1
  RLNC_SMALL_QUEUE=$q CONFIGS=0 timeout -k 10 120 python scripts/bench_configs.py 2>/dev/null | sed "s/^{/{\"queue_waves_per_simd\": $q, /" >> $O/queue_ab.jsonl || exit 1
done
cat $O/queue_ab.jsonl
RLNC_LIB_PATH=$PWD/rlnc_amd/librlnc_hip_ab.so timeout -k 10 120 python scripts/elim_small_prof.py > $O/elim_prof.jsonl 2> $O/elim_prof.err || { tail $O/elim_prof.err; exit 1; }
cat $O/elim_prof.jsonl
echo "all done"
