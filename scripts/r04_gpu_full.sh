# the whole -m gpu suite (fail-fast), then the HSA dispatch probe and the piece A/B
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_lifetime.py tests/test_gpu_piece.py tests > gpurun_out/gpu_tests.log 2>&1 || { tail -40 gpurun_out/gpu_tests.log; exit 1; }
tail -3 gpurun_out/gpu_tests.log
timeout -k 10 60 build/ubench_hsa_dispatch > gpurun_out/hsa.jsonl 2>&1
bash scripts/r04_piece_ab.sh
