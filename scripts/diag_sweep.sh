#!/usr/bin/env bash
# A/B a diagnostic build of librlnc_hip (build/diag) against the normal one with scripts/sweep.py.
set -eu
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
python -c "import __graft_entry__ as g; g.build()" > /dev/null
echo "normal:"; timeout -k 10 200 python scripts/sweep.py --rounds 6 --configs ${CONFIGS:-0:0}
cp rlnc_amd/librlnc_hip.so /tmp/librlnc_hip.normal.so
cp build/diag/librlnc_hip.so rlnc_amd/librlnc_hip.so
echo "diag:"; RLNC_DIAG=1 timeout -k 10 200 python scripts/sweep.py --rounds 6 --configs ${CONFIGS:-0:0}
cp /tmp/librlnc_hip.normal.so rlnc_amd/librlnc_hip.so
