# round-5: configs[0] encode/decode with the 2-wave program at set-building diagnostics (scripts/build_sets_vars.sh)
set -o pipefail
O=gpurun_out/r05_sets
mkdir -p $O
for rep in 1 2 3; do
  for v in base nocombo nosets; do
    if [ $v = base ]; then lib=$PWD/rlnc_amd/librlnc_hip.so; else lib=$PWD/build/w2var/$v/librlnc_hip.so; fi
    r=$(RLNC_LIB_PATH=$lib CONFIGS=0 timeout -k 10 120 python scripts/bench_configs.py 2>/dev/null) || exit 1
    echo "{\"variant\": \"$v\", \"r\": $r}" >> $O/ab.jsonl
    echo "$v $(echo $r | grep -o '"encode_ms[^,]*,\|"decode_ms[^,]*,\|"verified[^,}]*' | tr '\n' ' ')"
  done
done
