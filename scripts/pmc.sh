#!/usr/bin/env bash
# PMC passes (one counter group per rocprofv3 run, --kernel-trace only; never combined with sys/runtime
# traces) over the bench-shaped kernels driven by scripts/sweep.py.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd)
OUT=$ROOT/gpurun_out/pmc
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp
rocprofv3 -L > "$OUT/counters_available.txt" 2>&1 || true
i=0
# counter groups: one per line in $PMC_GROUPS_FILE (default: the set below); at most 8 SQ counters per line
# (more aborts rocprofv3 with "Request exceeds the capabilities of the hardware")
GROUPS_FILE=${PMC_GROUPS_FILE:-}
if [ -z "$GROUPS_FILE" ]; then
  GROUPS_FILE=/tmp/pmc_groups.txt
  cat > "$GROUPS_FILE" <<'GROUPS'
SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VALU GRBM_GUI_ACTIVE GRBM_COUNT
SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_SALU
FETCH_SIZE
WRITE_SIZE
GROUPS
fi
while read -r group; do
  [ -z "$group" ] && continue
  i=$((i+1))
  timeout -k 10 ${PMC_TIMEOUT:-150} rocprofv3 --kernel-trace --pmc $group -d "$OUT/p$i" -o run --output-format csv -- \
      python3 "$ROOT/scripts/sweep.py" --rounds 2 --configs ${SWEEP_CONFIGS:-0:0} > "$OUT/p$i.log" 2>&1
  rc=$?; echo "pmc pass $i ($group) rc=$rc"
  case $rc in 124|134|137|139) exit $rc;; esac
done < "$GROUPS_FILE"
python3 "$ROOT/scripts/pmc_summary.py" "$OUT" > "$OUT/summary.txt" 2>&1; cat "$OUT/summary.txt"
