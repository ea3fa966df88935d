# kernel durations of the piece path at the 1 MB rows (rocprofv3 kernel trace), encode then recode
set -o pipefail
mkdir -p gpurun_out/piece_prof
cd /tmp && export TMPDIR=/tmp
for only in encode recode; do
  OBJ_BENCH_SMALL=1 OBJ_BENCH_ONLY=$only timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/piece_prof/$only -o run -- $GRAFT_REPO_ROOT/build/object_api_bench --quick > $GRAFT_REPO_ROOT/gpurun_out/piece_prof/$only.log 2>&1
done
