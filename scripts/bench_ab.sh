#!/usr/bin/env bash
# Bench A/B (no CPU baselines): "label:env:args" specs in AB, run twice interleaved; prints value / ms_per_step /
# the encode launch's kernel_ms per run.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for rep in 1 2; do
  for spec in $AB; do
    label=${spec%%:*}; rest=${spec#*:}; envs=${rest%%:*}; args=${rest#*:}
    out=$(env ${envs//,/ } timeout -k 10 200 python bench.py --no-cpu-baseline ${args//,/ } 2>/dev/null) || { echo "$label failed"; exit 1; }
    echo "$out" | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$label', d['value'], d['ms_per_step'], d['roofline']['kernel_ms'])"
  done
done
