# the reference's whole bench grid on the object API (build/object_api_bench, full sample counts), after the piece
# path's parity tests
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_piece.py tests/test_gpu_lifetime.py > gpurun_out/piece_tests.log 2>&1 || { tail -30 gpurun_out/piece_tests.log; exit 1; }
tail -2 gpurun_out/piece_tests.log
timeout -k 10 600 build/object_api_bench > gpurun_out/obj_full.jsonl 2> gpurun_out/obj_full.err
