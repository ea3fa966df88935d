# fused marker scan: full GPU suite, then configs[0] decode A/B (fused vs RLNC_FUSED_SCAN=0), alternating
set -o pipefail
O=${1:-gpurun_out/r05_fused}
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests > $O/gpu_tests.log 2>&1 || { tail -40 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
for i in 1 2 3; do
  CONFIGS=0 timeout -k 10 120 python scripts/bench_configs.py | sed 's/^/{"fused":1,"r":/; s/$/}/' >> $O/ab.jsonl || exit 1
  RLNC_FUSED_SCAN=0 CONFIGS=0 timeout -k 10 120 python scripts/bench_configs.py | sed 's/^/{"fused":0,"r":/; s/$/}/' >> $O/ab.jsonl || exit 1
done
python3 -c "
import json
for l in open('$O/ab.jsonl'):
    j=json.loads(l); r=j['r']; print('fused', j['fused'], 'decode', r['decode_ms'], 'encode', r['encode_ms'], r['verified'])
"
