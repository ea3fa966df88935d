# round-4 GPU step: lifetime / piece / API tests, then the call-latency path's completion granularity
# (RLNC_PIECE_CHUNK = workgroups per host flag; 1 = a flag per workgroup, no counter) at the 1 MB rows
set -o pipefail
mkdir -p gpurun_out/chunk_ab
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_lifetime.py tests/test_gpu_piece.py tests/test_gpu_api.py tests/test_gpu_boundary.py > gpurun_out/chunk_ab/tests.log 2>&1 || { tail -30 gpurun_out/chunk_ab/tests.log; exit 1; }
tail -1 gpurun_out/chunk_ab/tests.log
export OBJ_BENCH_SMALL=1
for rep in 1 2; do
  for c in 64 1 4 16; do
    for only in encode recode; do
      echo "== RLNC_PIECE_CHUNK=$c $only" >> gpurun_out/chunk_ab/calls.txt
      RLNC_PIECE_CHUNK=$c OBJ_BENCH_ONLY=$only timeout -k 10 60 build/object_api_bench --quick >> gpurun_out/chunk_ab/calls.txt 2>&1 || exit 1
    done
  done
  echo "rep $rep done"
done
