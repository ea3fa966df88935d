#!/bin/bash
# Round-3 state measurements on one MI355X (gpurun from the repo root): every BASELINE config's device rates, the
# misaligned-row rates, the bench line, and rocprofv3 kernel stats of the bench (pipeline-1 groups: isolated launch
# durations for the roofline's kernel_ms).  Stops at the first failure.
set -o pipefail
O=gpurun_out/r03f
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python scripts/bench_configs.py > $O/configs.jsonl 2> $O/configs.err &&
timeout -k 10 200 python scripts/unaligned_rates.py > $O/unaligned.jsonl 2> $O/unaligned.err &&
timeout -k 10 300 python bench.py > $O/bench.json 2> $O/bench.err &&
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/prof -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 10 --warmup 3 --no-cpu-baseline --pipeline 1 > $GRAFT_REPO_ROOT/$O/prof.log 2>&1)
rc=$?
echo "rc=$rc"
cat $O/configs.jsonl; cat $O/unaligned.jsonl; tail -c 700 $O/bench.json
exit $rc
