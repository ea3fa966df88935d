#!/usr/bin/env bash
# HBM traffic of the bench's own kernels: two PMC passes (FETCH_SIZE, WRITE_SIZE — they cannot share a pass:
# 3 + 2 TCC counters > 4), each `rocprofv3 --kernel-trace --pmc` only, over a short bench run; then the
# per-(kernel, grid) summary with the gfx950 FETCH_SIZE x2 correction (scripts/pmc_summary.py).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd)
OUT=$ROOT/gpurun_out/pmc_bench
rm -rf "$OUT"; mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp
i=0
for group in FETCH_SIZE WRITE_SIZE ${EXTRA_GROUPS:-}; do
  i=$((i+1))
  timeout -k 10 -s KILL 120 rocprofv3 --kernel-trace --pmc ${group//,/ } -d "$OUT/p$i" -o run --output-format csv -- \
      python3 "$ROOT/bench.py" --steps 3 --warmup 1 --no-cpu-baseline ${BENCH_ARGS:-} > "$OUT/p$i.log" 2>&1
  rc=$?; echo "pmc pass $i ($group) rc=$rc"
  [ $rc -ne 0 ] && exit $rc
done
python3 "$ROOT/scripts/pmc_summary.py" "$OUT" > "$OUT/summary.jsonl" 2>&1; cat "$OUT/summary.jsonl"
