#!/usr/bin/env bash
# A/B of the blocked elimination's forms (RLNC_BLK: 8/16 pieces per block, +100 = Gauss-Jordan block step): the decode
# parity tests under each form, then scripts/elim_timing.py (path 5).  Stops at the first failure.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT
: > $OUT/elim_ab.jsonl
for f in ${FORMS:-16 8 116 108}; do
  RLNC_BLK=$f timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread \
      -k "decode" > $OUT/elim_ab_t$f.log 2>&1
  rc=$?; echo "form $f pytest rc=$rc $(tail -1 $OUT/elim_ab_t$f.log)"
  if [ $rc -ne 0 ]; then tail -30 $OUT/elim_ab_t$f.log; exit $rc; fi
  RLNC_BLK=$f ELIM_PATHS=5 timeout -k 10 300 python scripts/elim_timing.py 2>/dev/null | sed "s/^{/{\"blk\": $f, /" >> $OUT/elim_ab.jsonl
  rc=$?; if [ $rc -ne 0 ]; then echo "timing rc=$rc"; exit $rc; fi
done
