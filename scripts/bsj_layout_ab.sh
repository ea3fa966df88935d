#!/usr/bin/env bash
# A/B of the bit-sliced jump program's code-block layout (gen_bsjump.py --stride/--align): prebuilt libraries in
# build/var/<name>/librlnc_hip.so are swapped in for the product library; each is checked by the matmul parity tests,
# then bench.py runs, interleaved over two passes.  Output: gpurun_out/bsj_layout_ab.jsonl.  The product library is
# restored at the end.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT
cp rlnc_amd/librlnc_hip.so /tmp/librlnc_hip.base.so
: > $OUT/bsj_layout_ab.jsonl
rc=0
for pass in $(seq 1 ${PASSES:-2}); do
  for v in base ${VARIANTS:-s256a8 s192a6 s136a3}; do
    if [ $v = base ]; then cp /tmp/librlnc_hip.base.so rlnc_amd/librlnc_hip.so; else cp build/var/$v/librlnc_hip.so rlnc_amd/librlnc_hip.so; fi
    if [ $pass = 1 ]; then
      timeout -k 10 200 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread \
          -k "matmul or golden_encode or config" > $OUT/bsj_t_$v.log 2>&1
      rc=$?; echo "$v parity rc=$rc $(tail -1 $OUT/bsj_t_$v.log)"
      if [ $rc -ne 0 ]; then break 2; fi
    fi
    timeout -k 10 300 python bench.py --steps 30 --no-cpu-baseline --no-ceiling > $OUT/bsj_b.json 2>/dev/null
    rc=$?; if [ $rc -ne 0 ]; then echo "$v bench rc=$rc"; break 2; fi
    python -c "
import json; d=json.load(open('$OUT/bsj_b.json')); b=d['breakdown']
print(json.dumps({'layout': '$v', 'pass': $pass, 'value': d['value'], 'encode_kernel_ms': b['encode_kernel_ms'], 'decode_ms': b['decode_ms']}))" >> $OUT/bsj_layout_ab.jsonl
  done
done
cp /tmp/librlnc_hip.base.so rlnc_amd/librlnc_hip.so
cat $OUT/bsj_layout_ab.jsonl
exit $rc
