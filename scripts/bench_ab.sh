#!/usr/bin/env bash
# Bench A/B (no CPU baselines): "label:env:args" specs in AB, run twice interleaved; prints value / ms_per_step /
# the encode launch's kernel_ms per run.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for rep in 1 2; do
  for spec in $AB; do
    label=${spec%%:*}; rest=${spec#*:}; envs=${rest%%:*}; args=${rest#*:}
    # exit 3 = verification failed: expected of the timing-only diagnostic builds (their JSON line is still printed)
    out=$(env ${envs//,/ } timeout -k 10 200 python bench.py --no-cpu-baseline ${args//,/ } 2>/dev/null)
    rc=$?; if [ $rc -ne 0 ] && [ $rc -ne 3 ]; then echo "$label failed ($rc)"; exit 1; fi
    echo "$out" | python -c "import json,sys; d=json.loads([l for l in sys.stdin.read().splitlines() if l.startswith('{')][-1]); print('$label', d['value'], d['ms_per_step'], d['roofline']['kernel_ms'], 'decode_ms', d.get('breakdown', {}).get('decode_ms'), 'verified' if d.get('verified', d.get('breakdown', {}).get('verified')) else 'NOT-verified')"
  done
done
