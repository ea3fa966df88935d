#!/usr/bin/env bash
# One GPU-box session: gpu tests → smoke → bench → rocprofv3 kernel stats.  Stops at the first GPU fault,
# abort, segfault or timeout (exit codes 124/134/137/139), never retries.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd)
OUT=$ROOT/gpurun_out
mkdir -p "$OUT"
export TMPDIR=/tmp
fatal() { case "$1" in 124|134|137|139) return 0;; *) return 1;; esac; }

python -c "import __graft_entry__ as g; g.build()" > "$OUT/build.log" 2>&1 || { echo "build failed"; exit 1; }
rocminfo 2>/dev/null | grep -m2 -E "gfx950|Marketing" > "$OUT/device.txt" || true

if [ "${SKIP_TESTS:-0}" != "1" ]; then
  timeout -k 10 ${TEST_TIMEOUT:-900} python -m pytest tests -m gpu -q -p no:cacheprovider ${PYTEST_ARGS:-} > "$OUT/pytest_gpu.log" 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -5 "$OUT/pytest_gpu.log"
  if fatal $rc; then echo "fatal rc from pytest; stopping"; exit $rc; fi
fi

if [ -n "${SWEEP:-}" ]; then
  timeout -k 10 300 python scripts/sweep.py ${SWEEP} > "$OUT/sweep.jsonl" 2> "$OUT/sweep.err"
  rc=$?; echo "sweep rc=$rc"; cat "$OUT/sweep.jsonl"; tail -3 "$OUT/sweep.err"
  if fatal $rc; then exit $rc; fi
fi

timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1
rc=$?; echo "smoke rc=$rc"; tail -3 "$OUT/smoke.log"
if fatal $rc; then exit $rc; fi

timeout -k 10 600 python bench.py ${BENCH_ARGS:-} > "$OUT/bench.json" 2> "$OUT/bench.err"
rc=$?; echo "bench rc=$rc"; cat "$OUT/bench.json"; tail -3 "$OUT/bench.err"
if fatal $rc; then exit $rc; fi

if [ "${SKIP_PROF:-0}" != "1" ]; then
  cd /tmp
  # per-kernel durations of isolated launches (pipeline-1 steps: no overlap between steps), the roofline's source
  timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run --output-format csv -- \
      python3 "$ROOT/bench.py" --steps 10 --warmup 3 --no-cpu-baseline --pipeline 1 ${BENCH_ARGS:-} > "$OUT/prof.log" 2>&1
  rc=$?; echo "rocprof rc=$rc"; tail -3 "$OUT/prof.log"
  find "$OUT/prof" -name "*stats*" | head
  if fatal $rc; then exit $rc; fi
  # the default (cross-step pipelined) bench's timeline
  timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$OUT/prof_p2" -o run --output-format csv -- \
      python3 "$ROOT/bench.py" --steps 10 --warmup 3 --no-cpu-baseline ${BENCH_ARGS:-} > "$OUT/prof_p2.log" 2>&1
  rc=$?; echo "rocprof (pipelined) rc=$rc"
fi
