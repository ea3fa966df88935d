# round-5 GPU step 5: the small-object elimination's prefix-decomposed dirty step -- parity, timing, timeline
set -o pipefail
O=${1:-gpurun_out/r05e}
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_parity.py -k "small or decode" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 120 python scripts/elim_small_probe.py > $O/elim.jsonl 2>/dev/null || exit 1
cat $O/elim.jsonl
CONFIGS=0 timeout -k 10 120 python scripts/bench_configs.py > $O/configs0.jsonl 2>/dev/null || exit 1
cat $O/configs0.jsonl
RLNC_LIB_PATH=$PWD/rlnc_amd/librlnc_hip_ab.so timeout -k 10 120 python scripts/elim_small_prof.py > $O/elim_prof.jsonl 2> $O/elim_prof.err || { tail $O/elim_prof.err; exit 1; }
cat $O/elim_prof.jsonl
echo "all done"
