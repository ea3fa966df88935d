#!/usr/bin/env bash
# Per-piece cycle counts of gf_rref_batch_kernel: a diagnostic build (-DRLNC_RREF_PROFILE, statuses become
# s_memtime deltas) swapped in for scripts/rref_timing.py, then the normal library restored.
set -eu
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
python -c "import __graft_entry__ as g; g.build()" > /dev/null
# the instrumented round-3 copy of rref.hip (scripts/diag/rref_profile.hip) in place of the shipped one
scripts/diag_build.sh build/diag rref.hip=scripts/diag/rref_profile.hip -- -DRLNC_RREF_PROFILE > /dev/null
cp rlnc_amd/librlnc_hip.so /tmp/librlnc_hip.normal.so
cp build/diag/librlnc_hip.so rlnc_amd/librlnc_hip.so
RLNC_RREF_PROFILE=1 timeout -k 10 200 python scripts/rref_timing.py || true
cp /tmp/librlnc_hip.normal.so rlnc_amd/librlnc_hip.so
