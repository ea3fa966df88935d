# round-4 GPU step: ragged/wire parity after the table-copy kernel, ragged rate, profile
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_ragged.py tests/test_gpu_wire.py tests/test_gpu_graph.py > gpurun_out/t_rag.log 2>&1 || { tail -30 gpurun_out/t_rag.log; exit 1; }
tail -2 gpurun_out/t_rag.log
for i in 1 2; do
  timeout -k 10 120 python scripts/ragged_rate.py > gpurun_out/ragged_rate.jsonl 2>/dev/null || exit 1
  cat gpurun_out/ragged_rate.jsonl
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --memory-copy-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_rag -o run -- python $GRAFT_REPO_ROOT/scripts/ragged_rate.py > $GRAFT_REPO_ROOT/gpurun_out/prof_rag.log 2>&1 || exit 1
