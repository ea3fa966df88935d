# configs[0] decode check: small / decode parity tests, the elimination alone, configs[0] three times
set -o pipefail
O=${1:-gpurun_out/r05_cfg0}
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_parity.py -k "small or decode" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 120 python scripts/elim_small_probe.py > $O/elim.jsonl 2>/dev/null || exit 1
cat $O/elim.jsonl
for i in 1 2 3; do CONFIGS=0 timeout -k 10 120 python scripts/bench_configs.py >> $O/configs0.jsonl 2>/dev/null || exit 1; done
python3 -c "
import json
for l in open('$O/configs0.jsonl'):
    r=json.loads(l); print('decode', r['decode_ms'], r['decode_T_muladd_per_s'], 'encode', r['encode_ms'], r['verified'])
"
