# round-4 closing step: the whole -m gpu suite (shipped library, then the A/B build's variants), smoke(), bench.py
set -o pipefail
mkdir -p gpurun_out/final2
timeout -k 10 900 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests > gpurun_out/final2/gpu_tests.log 2>&1 || { tail -40 gpurun_out/final2/gpu_tests.log; exit 1; }
tail -1 gpurun_out/final2/gpu_tests.log
RLNC_LIB_PATH=$PWD/rlnc_amd/librlnc_hip_ab.so timeout -k 10 900 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_fullrange.py tests/test_gpu_graph.py > gpurun_out/final2/ab_tests.log 2>&1 || { tail -40 gpurun_out/final2/ab_tests.log; exit 1; }
tail -1 gpurun_out/final2/ab_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/final2/smoke.log 2>&1 || { tail -20 gpurun_out/final2/smoke.log; exit 1; }
tail -1 gpurun_out/final2/smoke.log
timeout -k 10 400 python bench.py > gpurun_out/final2/bench.json 2> gpurun_out/final2/bench.err || { tail -20 gpurun_out/final2/bench.err; exit 1; }
python3 -c "import json; d=json.loads([l for l in open('gpurun_out/final2/bench.json') if l.startswith('{')][-1]); print(d['value'], d['ms_per_step'], d['roofline']['kernel_ms'], d['breakdown']['decode_ms'], d['hbm_single_pass_encode']['read_frac'])"
