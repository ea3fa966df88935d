# round-4 GPU step: upper bound of fewer barriers in the 4-wave shared program (the decode's 32-row T x data):
# --diag=snobar removes its per-row barrier (timing only) -- what an NT = 4 8-wave form (a barrier every 3 rows) could
# at most gain
set -o pipefail
mkdir -p gpurun_out
AB="product:X=1: snobar:RLNC_LIB_PATH=$PWD/build/diag_snobar/librlnc_hip.so:" bash scripts/bench_ab.sh 2>&1 | tee gpurun_out/snobar_ab.txt
