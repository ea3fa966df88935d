# round-4 GPU step: the small-object elimination writes the product's block-offset stream -- parity (the new block-
# product test first), configs, then configs[0]-shape timing twice
set -o pipefail
mkdir -p gpurun_out/fusedoff
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_parity.py -k "many_small_objects" > gpurun_out/fusedoff/t_small.log 2>&1 || { tail -30 gpurun_out/fusedoff/t_small.log; exit 1; }
tail -1 gpurun_out/fusedoff/t_small.log
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_configs.py tests/test_gpu_graph.py tests/test_gpu_ragged.py > gpurun_out/fusedoff/t_all.log 2>&1 || { tail -30 gpurun_out/fusedoff/t_all.log; exit 1; }
tail -1 gpurun_out/fusedoff/t_all.log
for rep in 1 2; do
  CONFIGS=0 timeout -k 10 120 python scripts/bench_configs.py 2>/dev/null | grep -o '"encode_ms[^,]*,\|"decode_ms[^,]*,\|"decode_T[^,]*,' | tr '\n' ' '; echo
done
