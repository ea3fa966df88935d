# round-4 GPU step: object-API parity tests, then the reference's bench grid on the object API (piece path and the
# round-3 path by RLNC_PIECE=0), host elimination push cost
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_piece.py tests/test_gpu_api.py tests/test_gpu_boundary.py tests/test_gpu_cpp.py > gpurun_out/t1.log 2>&1 || { tail -30 gpurun_out/t1.log; exit 1; }
tail -3 gpurun_out/t1.log
timeout -k 10 60 build/elim_push_bench > gpurun_out/elim_push.jsonl 2>&1
timeout -k 10 200 build/object_api_bench --quick > gpurun_out/obj_piece.jsonl 2>&1
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/bench.json 2> gpurun_out/bench.err
