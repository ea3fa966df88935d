#!/usr/bin/env bash
# Narrow-operand kernel A/B: the GPU tests (new kernel, default), then scripts/bench_configs.py with RLNC_NARROW=0
# (round-1 perm path) / 1 (gf_matmul_narrow_kernel), interleaved; configs[3]'s recode carries a 64-byte tail.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
    > $OUT/narrow_tests.log 2>&1
rc=$?; echo "tests rc=$rc $(tail -1 $OUT/narrow_tests.log)"; [ $rc -eq 0 ] || { tail -30 $OUT/narrow_tests.log; exit $rc; }
for pass in 1 2; do
  for f in 0 1; do
    RLNC_NARROW=$f timeout -k 10 300 python scripts/bench_configs.py > $OUT/nw_cfg_$f.jsonl 2> $OUT/nw_cfg_$f.err
    rc=$?; [ $rc -eq 0 ] || { echo "configs narrow=$f rc=$rc"; tail -3 $OUT/nw_cfg_$f.err; exit $rc; }
    python -c "
import json
for l in open('$OUT/nw_cfg_$f.jsonl'):
    d = json.loads(l)
    print('narrow=$f pass=$pass', d['config'][:28], {k: v for k, v in d.items() if k.endswith('_ms') or k == 'verified'})"
  done
done
