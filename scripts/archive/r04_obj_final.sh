# round-4 final object-API step: piece / API / lifetime / C++ tests (automatic split and forced split 3), then the
# reference's whole bench grid on the object API
set -o pipefail
mkdir -p gpurun_out/objfinal
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_piece.py tests/test_gpu_api.py tests/test_gpu_lifetime.py tests/test_gpu_cpp.py tests/test_gpu_boundary.py > gpurun_out/objfinal/tests.log 2>&1 || { tail -30 gpurun_out/objfinal/tests.log; exit 1; }
tail -1 gpurun_out/objfinal/tests.log
RLNC_PIECE_SPLIT=3 timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_piece.py > gpurun_out/objfinal/tests_split3.log 2>&1 || { tail -30 gpurun_out/objfinal/tests_split3.log; exit 1; }
tail -1 gpurun_out/objfinal/tests_split3.log
timeout -k 10 700 build/object_api_bench > gpurun_out/objfinal/obj_full.jsonl 2> gpurun_out/objfinal/obj_full.err || { tail gpurun_out/objfinal/obj_full.err; exit 1; }
grep -c . gpurun_out/objfinal/obj_full.jsonl
