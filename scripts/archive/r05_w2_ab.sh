# round-5: configs[0] encode/decode times of the 2-wave program variants (scripts/build_w2_vars.sh), interleaved
set -o pipefail
O=gpurun_out/r05_w2
mkdir -p $O
RLNC_LIB_PATH=$PWD/build/w2var/slots5/librlnc_hip.so timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py -k "small or decode or bitsliced" > $O/t_slots5.log 2>&1 || { tail -20 $O/t_slots5.log; exit 1; }
echo "slots5 $(tail -1 $O/t_slots5.log)"
for rep in 1 2; do
  for v in base slots5 nosmem novm slots5nosmem; do
    if [ $v = base ]; then lib=$PWD/rlnc_amd/librlnc_hip.so; else lib=$PWD/build/w2var/$v/librlnc_hip.so; fi
    r=$(RLNC_LIB_PATH=$lib CONFIGS=0 timeout -k 10 120 python scripts/bench_configs.py 2>/dev/null) || exit 1
    echo "{\"variant\": \"$v\", \"r\": $r}" >> $O/ab.jsonl
    echo "$v $(echo $r | grep -o '"encode_ms[^,]*,\|"decode_ms[^,]*,\|"verified[^,}]*' | tr '\n' ' ')"
  done
done
