#!/usr/bin/env bash
# Interleaved A/B of the single-pass encode HBM rate (scripts/hbm_encode.py) across library builds:
# product + build/diag_<name>/librlnc_hip.so for each name in DIAGS, two passes.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for rep in 1 2; do
  for d in product ${DIAGS:-}; do
    if [ $d = product ]; then unset RLNC_LIB_PATH; else export RLNC_LIB_PATH=build/diag_$d/librlnc_hip.so; fi
    echo "== $d"
    HBM_VARIANTS=6 timeout -k 10 120 python scripts/hbm_encode.py 2>&1 | grep n_coded || exit 1
  done
done
