#!/usr/bin/env bash
# One PMC pass (clock, wave occupancy, issue/wait split) over the bench-shaped encode/decode launches of the
# product library and of diagnostic builds (scripts/bs_diag.sh), then the per-kernel summary of each.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd)
export TMPDIR=/tmp
CNT=${PMC_COUNTERS:-"GRBM_GUI_ACTIVE SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU"}
for d in product ${DIAGS:-}; do
  OUT=$ROOT/gpurun_out/pmc_diag/$d
  rm -rf "$OUT"; mkdir -p "$OUT"
  if [ $d = product ]; then unset RLNC_LIB_PATH; else export RLNC_LIB_PATH=$ROOT/build/diag_$d/librlnc_hip.so; fi
  (cd /tmp && RLNC_DIAG=1 timeout -k 10 -s KILL 120 rocprofv3 --kernel-trace --pmc $CNT -d "$OUT" -o run --output-format csv -- \
      python3 "$ROOT/scripts/sweep.py" --configs ${CONFIGS:-6:0} --rounds 2 > "$OUT/log" 2>&1)
  rc=$?; echo "== $d rc=$rc"
  [ $rc -ne 0 ] && { tail -5 "$OUT/log"; exit $rc; }
  python3 "$ROOT/scripts/pmc_summary.py" "$OUT" | grep -E "bs_kernel|bsj_kernel"
done
