# the object-API grid (the reference's five benches x 15 shapes) on this box; the run tag names the output file
set -o pipefail
T=${1:-a}
mkdir -p gpurun_out/r05_objgrid
timeout -k 10 200 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_piece.py tests/test_gpu_cpp.py > gpurun_out/r05_objgrid/tests_$T.log 2>&1 || { tail -30 gpurun_out/r05_objgrid/tests_$T.log; exit 1; }
tail -1 gpurun_out/r05_objgrid/tests_$T.log
timeout -k 10 600 build/object_api_bench > gpurun_out/r05_objgrid/grid_$T.jsonl 2> gpurun_out/r05_objgrid/grid_$T.err || { tail gpurun_out/r05_objgrid/grid_$T.err; exit 1; }
wc -l gpurun_out/r05_objgrid/grid_$T.jsonl
