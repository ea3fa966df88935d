#!/usr/bin/env bash
# Phase cycle counts of gf_rref_block_kernel (decode path 5): a diagnostic build (-DRLNC_RREF_PROFILE, statuses 0..7
# become s_memtime phase sums of wave 0) swapped in for scripts/elim_timing.py, then the normal library restored.
set -eu
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
# the instrumented round-3 copy of rref.hip (scripts/diag/rref_profile.hip) in place of the shipped one
scripts/diag_build.sh build/diag rref.hip=scripts/diag/rref_profile.hip -- -DRLNC_RREF_PROFILE > /dev/null
cp rlnc_amd/librlnc_hip.so /tmp/librlnc_hip.normal.so
cp build/diag/librlnc_hip.so rlnc_amd/librlnc_hip.so
ELIM_PROFILE=1 ELIM_PATHS=5 timeout -k 10 200 python scripts/elim_timing.py || true
cp /tmp/librlnc_hip.normal.so rlnc_amd/librlnc_hip.so
