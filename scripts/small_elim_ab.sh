#!/usr/bin/env bash
# Small-object elimination A/B (diagnostic library): the multi-object kernel at 1/2/4/8 objects per workgroup
# (RLNC_SMALL_NW), from 512 objects on (RLNC_SMALL_MIN=1), against the round-2 one-wave register kernel (path 4)
# and the blocked run (path 5); scripts/elim_timing.py checks every path's outputs equal to the first's.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export RLNC_LIB_PATH=$PWD/rlnc_amd/librlnc_hip_ab.so ELIM_SHAPES=small
for nw in 4 1 2 8; do
  echo "== RLNC_SMALL_NW=$nw RLNC_SMALL_MIN=1 (paths 0, 4, 5)"
  RLNC_SMALL_NW=$nw RLNC_SMALL_MIN=1 ELIM_PATHS=0,4,5 timeout -k 10 120 python3 scripts/elim_timing.py || exit $?
done
