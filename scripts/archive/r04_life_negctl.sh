# negative control of tests/test_gpu_lifetime.py::test_block_reused_only_after_uses_on_two_streams: the library built
# without ObjUse's cross-stream wait (build/negctl) must fail it; the shipped library passes it.  Build the control
# first (on the CPU):
#   mkdir -p build/negctl && sed 's/        if (used \&\& s != last) HIP_TRY(hipStreamWaitEvent(s, ev, 0));/        \/\/ negative control/' \
#       rlnc_amd/csrc/context.hpp > build/negctl/context.hpp && scripts/diag_build.sh build/negctl context.hpp=build/negctl/context.hpp
set -o pipefail
mkdir -p gpurun_out
T="tests/test_gpu_lifetime.py::test_block_reused_only_after_uses_on_two_streams"
RLNC_LIB_PATH=$PWD/build/negctl/librlnc_hip.so timeout -k 10 200 python -u -m pytest -q --timeout 120 --timeout-method thread -m gpu "$T" > gpurun_out/t_negctl.log 2>&1
echo "negative control rc=$? (1 = the test caught the missing wait)"
grep -E "passed|failed|Error" gpurun_out/t_negctl.log | head -3
timeout -k 10 200 python -u -m pytest -q --timeout 120 --timeout-method thread -m gpu "$T" > gpurun_out/t_ctl.log 2>&1
echo "shipped library rc=$?"
tail -1 gpurun_out/t_ctl.log
