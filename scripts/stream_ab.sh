#!/usr/bin/env bash
# A/B of the single-pass stream kernel forms (RLNC_STREAM_FORM, kernels.hip launch_stream): n = 1, 2, 3 coded
# pieces per source pass, 32 objects x k = 32 x 1 MiB, two interleaved passes.  Output: gpurun_out/stream_ab.jsonl
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT
: > $OUT/stream_ab.jsonl
for pass in 1 2; do
  for f in ${FORMS:-0 1 2 3 4 5 6 7}; do
    RLNC_STREAM_FORM=$f HBM_OBJECTS=32 HBM_NS=1,2,3 HBM_VARIANTS=8 timeout -k 10 120 python scripts/hbm_encode.py 2>/dev/null \
      | sed "s/^{/{\"form\": $f, \"pass\": $pass, /" >> $OUT/stream_ab.jsonl
    rc=$?; if [ $rc -ne 0 ]; then echo "form $f rc=$rc"; exit $rc; fi
  done
done
cat $OUT/stream_ab.jsonl
