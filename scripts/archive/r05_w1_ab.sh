# round-5: configs[0] encode/decode with 16-row products as two 1-wave tiles (scripts/build_w1_vars.sh), interleaved
set -o pipefail
O=gpurun_out/r05_w1
mkdir -p $O
for v in w1 w1s5; do
  RLNC_LIB_PATH=$PWD/build/w2var/$v/librlnc_hip.so timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py -k "small or decode or bitsliced" > $O/t_$v.log 2>&1 || { tail -20 $O/t_$v.log; exit 1; }
  echo "$v $(tail -1 $O/t_$v.log)"
done
for rep in 1 2 3; do
  for v in base w1 w1s5; do
    if [ $v = base ]; then lib=$PWD/rlnc_amd/librlnc_hip.so; else lib=$PWD/build/w2var/$v/librlnc_hip.so; fi
    r=$(RLNC_LIB_PATH=$lib CONFIGS=0 timeout -k 10 120 python scripts/bench_configs.py 2>/dev/null) || exit 1
    echo "{\"variant\": \"$v\", \"r\": $r}" >> $O/ab.jsonl
    echo "$v $(echo $r | grep -o '"encode_ms[^,]*,\|"decode_ms[^,]*,\|"verified[^,}]*' | tr '\n' ' ')"
  done
done
