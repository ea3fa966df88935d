# round-4 GPU step: staged device-to-host copy of large decoded objects -- piece / API tests, the 16 and 32 MB rows
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_piece.py tests/test_gpu_api.py tests/test_gpu_lifetime.py tests/test_gpu_cpp.py > gpurun_out/t_d2h.log 2>&1 || { tail -30 gpurun_out/t_d2h.log; exit 1; }
tail -1 gpurun_out/t_d2h.log
OBJ_BENCH_ONLY=decode timeout -k 10 300 build/object_api_bench > gpurun_out/obj_d2h.jsonl 2> gpurun_out/obj_d2h.err || { tail gpurun_out/obj_d2h.err; exit 1; }
grep -c . gpurun_out/obj_d2h.jsonl
