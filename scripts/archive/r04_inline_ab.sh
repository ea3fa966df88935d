# piece-path A/B at the 1 MB rows: coefficients in the kernel arguments (default) vs read from pinned host memory
# (RLNC_PIECE_INLINE=0): call medians, then the kernel's own duration under rocprofv3
set -o pipefail
mkdir -p gpurun_out/inline_ab
R=$PWD
export OBJ_BENCH_SMALL=1 OBJ_BENCH_ONLY=encode
for rep in 1 2; do
  for v in 1 0; do
    echo "== RLNC_PIECE_INLINE=$v" >> gpurun_out/inline_ab/calls.txt
    RLNC_PIECE_INLINE=$v timeout -k 10 60 build/object_api_bench --quick >> gpurun_out/inline_ab/calls.txt 2>&1 || exit 1
  done
done
cd /tmp && export TMPDIR=/tmp
for v in 1 0; do
  RLNC_PIECE_INLINE=$v timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/inline_ab/p$v -o run -- $R/build/object_api_bench --quick > $R/gpurun_out/inline_ab/p$v.log 2>&1 || exit 1
  python3 $R/scripts/rocpd_stats.py $R/gpurun_out/inline_ab/p$v/run_results.db --match gf_piece > $R/gpurun_out/inline_ab/kernels_inline$v.csv
done
cat $R/gpurun_out/inline_ab/kernels_inline1.csv $R/gpurun_out/inline_ab/kernels_inline0.csv
