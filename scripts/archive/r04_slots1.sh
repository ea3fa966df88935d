# round-4 GPU step: ragged 1-/2-wave classes ordered by source count; ring depth of the 1-wave program (slots1 = 5
# shipped candidate, 3 = round 3)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_ragged.py > gpurun_out/t_s1.log 2>&1 || { tail -30 gpurun_out/t_s1.log; exit 1; }
tail -2 gpurun_out/t_s1.log
for v in main s1_3 main s1_3; do
  if [ $v = main ]; then lib=$PWD/rlnc_amd/librlnc_hip.so; else lib=$PWD/build/$v/librlnc_hip.so; fi
  RLNC_LIB_PATH=$lib timeout -k 10 120 python scripts/ragged_rate.py > gpurun_out/rr_$v.jsonl 2>/dev/null || exit 1
  echo "$v $(grep -o '"abi_decode_ms.*' gpurun_out/rr_$v.jsonl)"
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_rag -o run -- python $GRAFT_REPO_ROOT/scripts/ragged_rate.py > $GRAFT_REPO_ROOT/gpurun_out/prof_rag.log 2>&1 || exit 1
