# round-4 GPU step: cache-policy hints of the bit-sliced programs on the HBM-bound small products (configs[0] shape:
# 4,096 objects of 16 x 4 KiB, encode and decode), libraries from scripts/build_hint_vars.sh, interleaved twice
set -o pipefail
mkdir -p gpurun_out/hint
for v in stnt bothnt; do
  RLNC_LIB_PATH=$PWD/build/var/$v/librlnc_hip.so timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py > gpurun_out/hint/t_$v.log 2>&1 || { tail -20 gpurun_out/hint/t_$v.log; exit 1; }
  echo "$v $(tail -1 gpurun_out/hint/t_$v.log)"
done
for rep in 1 2; do
  for v in base stnt ldnt bothnt; do
    if [ $v = base ]; then lib=$PWD/rlnc_amd/librlnc_hip.so; else lib=$PWD/build/var/$v/librlnc_hip.so; fi
    echo "$v $(RLNC_LIB_PATH=$lib CONFIGS=0 timeout -k 10 120 python scripts/bench_configs.py 2>/dev/null | grep -o '"encode_ms[^,]*,\|"decode_ms[^,]*,' | tr '\n' ' ')"
  done
done
