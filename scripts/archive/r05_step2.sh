# round-5 GPU step 2: whole -m gpu suite + the A/B build's parity tests, the configs[0] overlap exploration, the
# object-API grid (five benches x 15 shapes), configs[0] through bench_configs
set -o pipefail
O=${1:-gpurun_out/r05b}
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests > $O/gpu_tests.log 2>&1 || { tail -40 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
RLNC_LIB_PATH=$PWD/rlnc_amd/librlnc_hip_ab.so timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_fullrange.py tests/test_gpu_graph.py > $O/ab_tests.log 2>&1 || { tail -40 $O/ab_tests.log; exit 1; }
tail -1 $O/ab_tests.log
timeout -k 10 300 python scripts/cfg0_overlap.py > $O/cfg0_overlap.jsonl 2> $O/cfg0_overlap.err || { tail -20 $O/cfg0_overlap.err; exit 1; }
echo "overlap done"
CONFIGS=0 timeout -k 10 200 python scripts/bench_configs.py > $O/configs0.jsonl 2> $O/configs0.err || { tail $O/configs0.err; exit 1; }
cat $O/configs0.jsonl
timeout -k 10 400 build/object_api_bench > $O/object_api_bench.jsonl 2> $O/object_api_bench.err || { tail $O/object_api_bench.err; exit 1; }
echo "all done"
