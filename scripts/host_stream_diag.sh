#!/bin/bash
# Bimodal host-stream rate: five consecutive processes of the pinned host-stream pipeline, each under
# rocprofv3 --memory-copy-trace --kernel-trace (no counters), then three without the profiler.  The per-copy records
# (which queue / engine each copy ran on, its duration, how the two directions overlapped) are summarised by
# scripts/host_stream_copies.py.  Run from the repo root through gpurun.
set -o pipefail
O=gpurun_out/hs
mkdir -p $O
export TMPDIR=/tmp
for i in 1 2 3 4 5; do
  (cd /tmp && timeout -k 10 200 rocprofv3 --memory-copy-trace --kernel-trace -d $GRAFT_REPO_ROOT/$O/p$i -o run -- \
     python3 $GRAFT_REPO_ROOT/scripts/host_stream_rate.py --modes pinned --steps 5 > $GRAFT_REPO_ROOT/$O/p$i.json \
     2> $GRAFT_REPO_ROOT/$O/p$i.err) || exit 1
done
for i in 1 2 3; do
  timeout -k 10 200 python3 scripts/host_stream_rate.py --modes pinned,raw --steps 5 > $O/plain$i.json 2> $O/plain$i.err || exit 1
done
for i in 1 2 3 4 5; do python3 scripts/host_stream_copies.py $O/p$i/run_results.db $O/p$i.json; done > $O/summary.txt
cat $O/summary.txt
for i in 1 2 3; do python3 -c "import json,sys; d=json.load(open('$O/plain$i.json')); print('plain', d['pinned']['value'], d['pinned']['step_ms'], d.get('pinned_h2d_GBps'), d.get('pinned_d2h_GBps'), d.get('pinned_bidirectional_GBps'))"; done
