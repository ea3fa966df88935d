# round-4 GPU step: upper bound of a barrier-free 8-wave encode loop (--diag=s8nobar, timing only) against the product
set -o pipefail
mkdir -p gpurun_out
AB="product:X=1: s8nobar:RLNC_LIB_PATH=$PWD/build/diag_s8nobar/librlnc_hip.so:" bash scripts/bench_ab.sh 2>&1 | tee gpurun_out/s8nobar_ab.txt
