# round-5: the split 2-wave program (scripts/build_split_var.sh): parity suite on it, then configs[0] A/B interleaved
set -o pipefail
O=gpurun_out/r05_split
mkdir -p $O
lib=$PWD/build/w2var/split/librlnc_hip.so
RLNC_LIB_PATH=$lib timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py -k "small or decode or bitsliced or matmul" > $O/t_split.log 2>&1 || { tail -30 $O/t_split.log; exit 1; }
echo "split $(tail -1 $O/t_split.log)"
for rep in 1 2 3; do
  for v in base split; do
    if [ $v = base ]; then l=$PWD/rlnc_amd/librlnc_hip.so; else l=$lib; fi
    r=$(RLNC_LIB_PATH=$l CONFIGS=0 timeout -k 10 120 python scripts/bench_configs.py 2>/dev/null) || exit 1
    echo "{\"variant\": \"$v\", \"r\": $r}" >> $O/ab.jsonl
    echo "$v $(echo $r | grep -o '"encode_ms[^,]*,\|"decode_ms[^,]*,\|"verified[^,}]*' | tr '\n' ' ')"
  done
done
