# round-4 GPU step: ring depth of the 2-wave bit-sliced program (slots2 = 3 shipped, 4, 5) on configs[0]'s shape
set -o pipefail
mkdir -p gpurun_out
for v in s2_4 s2_5; do
  RLNC_LIB_PATH=$PWD/build/$v/librlnc_hip.so timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_ragged.py > gpurun_out/t_$v.log 2>&1 || { tail -30 gpurun_out/t_$v.log; exit 1; }
  echo "$v $(tail -1 gpurun_out/t_$v.log)"
done
for v in main s2_4 s2_5 main s2_4 s2_5; do
  if [ $v = main ]; then lib=$PWD/rlnc_amd/librlnc_hip.so; else lib=$PWD/build/$v/librlnc_hip.so; fi
  RLNC_LIB_PATH=$lib CONFIGS=0 timeout -k 10 120 python scripts/bench_configs.py > gpurun_out/c0_$v.jsonl 2>/dev/null || exit 1
  echo "$v $(grep -o '"encode_ms[^,]*,' gpurun_out/c0_$v.jsonl) $(grep -o '"decode_ms[^,]*,' gpurun_out/c0_$v.jsonl)"
done
