# round-5: payload-tail marker answer -- decode / small-object parity tests, a configs[0] kernel trace, then the
# configs[0] decode A/B against RLNC_FUSED_SCAN=0 (interleaved)
set -o pipefail
O=${1:-gpurun_out/r05_tail3}
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_configs.py -k "small or decode or marker or config" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
bash scripts/archive/r05_cfg0_prof.sh $O/prof || exit 1
for i in 1 2 3; do
  r=$(CONFIGS=0 timeout -k 10 120 python scripts/bench_configs.py 2>/dev/null) || exit 1
  echo "{\"fused\": 1, \"r\": $r}" >> $O/ab.jsonl
  r=$(RLNC_FUSED_SCAN=0 CONFIGS=0 timeout -k 10 120 python scripts/bench_configs.py 2>/dev/null) || exit 1
  echo "{\"fused\": 0, \"r\": $r}" >> $O/ab.jsonl
done
python3 -c "
import json
for l in open('$O/ab.jsonl'):
    j=json.loads(l); r=j['r']; print('fused', j['fused'], 'decode', r['decode_ms'], 'encode', r['encode_ms'], r['verified'])
"
