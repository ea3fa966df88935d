#!/usr/bin/env bash
# A/B timing of diagnostic library builds (scripts/bs_diag.sh) against the product library, interleaved
# twice: the encode and decode launch shapes of the bench via scripts/sweep.py.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for rep in 1 2; do
  for d in product ${DIAGS:-novm nosmem novm_nosmem}; do
    if [ $d = product ]; then unset RLNC_LIB_PATH; else export RLNC_LIB_PATH=build/diag_$d/librlnc_hip.so; fi
    echo "== $d"
    RLNC_DIAG=1 timeout -k 10 120 python scripts/sweep.py --configs ${CONFIGS:-6:0} --rounds ${ROUNDS:-10} 2>&1 | grep -v amdgpu.ids || exit $?
  done
done
