# round-4 GPU step: non-temporal tile stores in the 1- and 2-wave programs -- parity suites, configs[0] shape, ragged
set -o pipefail
mkdir -p gpurun_out/ntsmall
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_ragged.py tests/test_gpu_configs.py tests/test_gpu_wire.py > gpurun_out/ntsmall/tests.log 2>&1 || { tail -30 gpurun_out/ntsmall/tests.log; exit 1; }
tail -1 gpurun_out/ntsmall/tests.log
for rep in 1 2; do
  CONFIGS=0 timeout -k 10 120 python scripts/bench_configs.py 2>/dev/null | grep -o '"encode_ms[^,]*,\|"decode_ms[^,]*,' | tr '\n' ' '; echo
done
timeout -k 10 120 python scripts/ragged_rate.py 2>/dev/null | grep -o '"abi_decode_ms.*'
