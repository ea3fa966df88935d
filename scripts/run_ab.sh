#!/usr/bin/env bash
# Column-run A/B (variant 9): run lengths, variant 8 as the control, and the no-store diagnostic build
# (scripts/bsj_diag.sh DIAGS="rnostore:--diag=rnostore"); scripts/tile_overhead.py shapes, k = 16 and 32.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
echo "== variant 8"; VARIANT=8 timeout -k 10 120 python scripts/tile_overhead.py 2>/dev/null | head -2 || exit 1
for r in ${RUNS:-1 4 8 16}; do
  echo "== run $r"; RLNC_BSJ_RUN=$r VARIANT=9 timeout -k 10 120 python scripts/tile_overhead.py 2>/dev/null | head -2 || exit 1
done
if [ -f build/diag_rnostore/librlnc_hip.so ]; then
  echo "== nostore run 8"; RLNC_LIB_PATH=build/diag_rnostore/librlnc_hip.so RLNC_BSJ_RUN=8 VARIANT=9 timeout -k 10 120 python scripts/tile_overhead.py 2>/dev/null | head -2
fi
