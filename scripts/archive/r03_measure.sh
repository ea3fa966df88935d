#!/bin/bash
# Round-3 measurements on one MI355X (run through gpurun from the repo root): the bench line (config2, N=1), the
# configs[4] strong-scaling workload at N=1, rocprofv3 kernel stats of both, and the ragged-batch rates + launches.
set -o pipefail
mkdir -p gpurun_out/r03
export TMPDIR=/tmp
O=gpurun_out/r03
timeout -k 10 300 python bench.py > $O/bench.json 2> $O/bench.err &&
timeout -k 10 300 python bench.py --workload config5 > $O/config5.json 2> $O/config5.err &&
timeout -k 10 200 python scripts/ragged_rate.py > $O/ragged.json 2> $O/ragged.err &&
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/prof_bench -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 10 --warmup 3 --no-cpu-baseline > $GRAFT_REPO_ROOT/$O/prof_bench.json 2> $GRAFT_REPO_ROOT/$O/prof_bench.err) &&
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/prof_config5 -o run -- python3 $GRAFT_REPO_ROOT/bench.py --workload config5 --steps 3 --warmup 1 --no-cpu-baseline > $GRAFT_REPO_ROOT/$O/prof_config5.json 2> $GRAFT_REPO_ROOT/$O/prof_config5.err) &&
(cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/prof_ragged -o run -- python3 $GRAFT_REPO_ROOT/scripts/ragged_rate.py > $GRAFT_REPO_ROOT/$O/prof_ragged.json 2> $GRAFT_REPO_ROOT/$O/prof_ragged.err)
rc=$?
echo "rc=$rc"
tail -c 600 $O/bench.json; echo; tail -c 400 $O/config5.json; echo; cat $O/ragged.json
exit $rc
