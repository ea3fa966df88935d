# the 1 MB decode rows: piece-call phases (RLNC_PIECE_TRACE) and kernel durations (rocprofv3)
set -o pipefail
mkdir -p gpurun_out/dec_prof
OBJ_BENCH_SMALL=1 OBJ_BENCH_ONLY=decode RLNC_PIECE_TRACE=1 timeout -k 10 120 build/object_api_bench --quick > gpurun_out/dec_prof/trace.txt 2>&1
cd /tmp && export TMPDIR=/tmp
OBJ_BENCH_SMALL=1 OBJ_BENCH_ONLY=decode timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/dec_prof/prof -o run -- $GRAFT_REPO_ROOT/build/object_api_bench --quick > $GRAFT_REPO_ROOT/gpurun_out/dec_prof/prof.log 2>&1
