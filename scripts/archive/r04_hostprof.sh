# round-4 GPU step: HIP API trace of the ragged calls (host cost per call)
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --hip-runtime-trace --kernel-trace -d $GRAFT_REPO_ROOT/gpurun_out/prof_host -o run -- python $GRAFT_REPO_ROOT/scripts/ragged_rate.py > $GRAFT_REPO_ROOT/gpurun_out/prof_host.log 2>&1 || exit 1
