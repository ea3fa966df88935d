set -u
cd "${GRAFT_REPO_ROOT}"
for pass in 1 2; do
  for v in ${VARIANTS:-8 7 9}; do
    VARIANT=$v timeout -k 10 300 python scripts/bench_configs.py > gpurun_out/v_$v.jsonl 2>/dev/null || { echo "v=$v failed"; exit 1; }
    python -c "
import json
for l in open('gpurun_out/v_$v.jsonl'):
    d = json.loads(l)
    print('v=$v pass=$pass', d['config'][:28], {k: v for k, v in d.items() if k.endswith('_ms')})"
  done
done
