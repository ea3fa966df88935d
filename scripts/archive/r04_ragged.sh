# round-4 GPU step: ragged parity (1-/2-wave bit-sliced classes), ragged rate, configs[0]-shape enc/dec, profiled
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_ragged.py tests/test_gpu_wire.py tests/test_gpu_graph.py > gpurun_out/t_rag.log 2>&1 || { tail -30 gpurun_out/t_rag.log; exit 1; }
tail -3 gpurun_out/t_rag.log
timeout -k 10 200 python scripts/ragged_rate.py > gpurun_out/ragged_rate.jsonl 2> gpurun_out/ragged_rate.err || { tail gpurun_out/ragged_rate.err; exit 1; }
cat gpurun_out/ragged_rate.jsonl
CONFIGS=0 timeout -k 10 200 python scripts/bench_configs.py > gpurun_out/cfg0.jsonl 2> gpurun_out/cfg0.err || { tail gpurun_out/cfg0.err; exit 1; }
cat gpurun_out/cfg0.jsonl
cd /tmp && export TMPDIR=/tmp
CONFIGS=0 timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_cfg0 -o run -- python $GRAFT_REPO_ROOT/scripts/bench_configs.py > $GRAFT_REPO_ROOT/gpurun_out/prof_cfg0.log 2>&1 || exit 1
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_rag -o run -- python $GRAFT_REPO_ROOT/scripts/ragged_rate.py > $GRAFT_REPO_ROOT/gpurun_out/prof_rag.log 2>&1 || exit 1
echo done
