set -o pipefail
mkdir -p gpurun_out
timeout -k 10 200 python -u -m pytest -x -v -rs --timeout 120 --timeout-method thread -m gpu tests/test_gpu_lifetime.py > gpurun_out/t_life.log 2>&1 || { tail -30 gpurun_out/t_life.log; exit 1; }
grep -E "PASS|SKIP|FAIL" gpurun_out/t_life.log
