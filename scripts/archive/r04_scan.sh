# round-4 GPU step: fused marker scan -- decode parity suites, configs[0] shape
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_configs.py tests/test_gpu_api.py tests/test_gpu_ragged.py tests/test_gpu_wire.py tests/test_gpu_boundary.py tests/test_gpu_piece.py > gpurun_out/t_scan.log 2>&1 || { tail -30 gpurun_out/t_scan.log; exit 1; }
tail -1 gpurun_out/t_scan.log
for i in 1 2; do
  CONFIGS=0 timeout -k 10 120 python scripts/bench_configs.py 2>/dev/null | grep -o '"encode_ms.*'
done
