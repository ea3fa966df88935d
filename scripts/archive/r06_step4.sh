# round 6, fourth GPU call: compact set slots (the shipped library) + barrier-spacing variants of the shared programs:
# w4b3 / w4b2 = the 4-wave program in the 8-wave form with a barrier every 3rd / 2nd row (gen_bsjump.py --w4bar), b84 =
# the 8-wave program with a barrier every 4th row (--bar8 4), w4b3b84 = both.  Parity on each, then interleaved A/B.
set -o pipefail
O=gpurun_out/r06_s4
mkdir -p $O
R=$PWD
timeout -k 10 900 python -u -m pytest -q --timeout 120 --timeout-method thread -m gpu tests > $O/gpu_tests.log 2>&1
rc=$?; tail -1 $O/gpu_tests.log
[ $rc -le 1 ] || { tail -60 $O/gpu_tests.log; exit $rc; }
grep -E "FAILED|ERROR" $O/gpu_tests.log | head -20
VARS="w4b3 w4b2 b84 w4b3b84"
for v in $VARS; do
  RLNC_LIB_PATH=$R/build/var_$v/librlnc_hip.so timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_ragged.py tests/test_gpu_configs.py > $O/tests_$v.log 2>&1
  rc=$?; echo "$v: $(tail -1 $O/tests_$v.log)"
  [ $rc -le 1 ] || { tail -30 $O/tests_$v.log; exit $rc; }
done
for rep in 1 2; do
  for lib in product $VARS; do
    if [ $lib = product ]; then unset RLNC_LIB_PATH; else export RLNC_LIB_PATH=$R/build/var_$lib/librlnc_hip.so; fi
    echo "== $lib rep $rep" >> $O/sweep.txt
    timeout -k 10 120 python scripts/sweep.py --objects 32 --configs 8:0 --rounds 12 >> $O/sweep.txt 2>&1 || { tail $O/sweep.txt; exit 1; }
  done
done
unset RLNC_LIB_PATH
grep -E "^==|enc_ms" $O/sweep.txt | paste - - | sed 's/"variant": "bitsliced-jump-shared-8w", "tile_rows": 0, //' | cut -c1-200
for lib in product $VARS; do
  if [ $lib = product ]; then unset RLNC_LIB_PATH; else export RLNC_LIB_PATH=$R/build/var_$lib/librlnc_hip.so; fi
  timeout -k 10 300 python bench.py --no-cpu-baseline --no-ceiling > $O/bench_$lib.json 2> $O/bench_$lib.err || { tail $O/bench_$lib.err; exit 1; }
  python3 -c "import json,sys; l=json.loads([x for x in open('$O/bench_$lib.json') if x.startswith('{')][-1]); print('$lib', l['value'], l['ms_per_step'], l['roofline']['kernel_ms'], l['roofline_decode']['kernel_ms'], l['breakdown']['verified'])"
done
echo "all done"
