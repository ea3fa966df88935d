# round-4 GPU step: the call-latency kernel's cross-workgroup source split -- piece tests with the automatic split and
# forced to 3 workgroups per block (every product above 64 sources, multi-row decodes included), then the 1 MB rows
# with the split (default) against RLNC_PIECE_SPLIT=1, twice, and the kernel durations under rocprofv3
set -o pipefail
mkdir -p gpurun_out/split_ab
R=$PWD
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_piece.py tests/test_gpu_api.py > gpurun_out/split_ab/t_auto.log 2>&1 || { tail -30 gpurun_out/split_ab/t_auto.log; exit 1; }
tail -1 gpurun_out/split_ab/t_auto.log
RLNC_PIECE_SPLIT=3 timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_piece.py > gpurun_out/split_ab/t_3.log 2>&1 || { tail -30 gpurun_out/split_ab/t_3.log; exit 1; }
tail -1 gpurun_out/split_ab/t_3.log
export OBJ_BENCH_SMALL=1
for rep in 1 2; do
  for v in 0 1; do
    for only in encode recode; do
      echo "== RLNC_PIECE_SPLIT=$v $only" >> gpurun_out/split_ab/calls.txt
      RLNC_PIECE_SPLIT=$v OBJ_BENCH_ONLY=$only timeout -k 10 60 build/object_api_bench --quick >> gpurun_out/split_ab/calls.txt 2>&1 || exit 1
    done
  done
  echo "rep $rep done"
done
cd /tmp && export TMPDIR=/tmp
for v in 0 1; do
  RLNC_PIECE_SPLIT=$v timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/split_ab/p$v -o run -- $R/build/object_api_bench --quick > $R/gpurun_out/split_ab/p$v.log 2>&1 || exit 1
  python3 $R/scripts/rocpd_stats.py $R/gpurun_out/split_ab/p$v/run_results.db --match gf_piece > $R/gpurun_out/split_ab/kernels_split$v.csv
done
cat $R/gpurun_out/split_ab/kernels_split0.csv $R/gpurun_out/split_ab/kernels_split1.csv
