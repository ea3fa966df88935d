# round 6, eighth GPU call: wave priority re-tuned on the set-planes programs: p8a / p8b = the 8-wave program's calls 2.. at s_setprio 2 / calls 4.. at 1 (--prio8), p4off / p4b = the 4-wave program without priority / calls 4.. at 2 (--prio)
# (interleaved with the shipped library: parity on each variant, then sweep and bench passes)
#
set -o pipefail
O=gpurun_out/r06_s8
mkdir -p $O
R=$PWD
VARS="p8a p8b p4off p4b"
for v in $VARS; do
  RLNC_LIB_PATH=$R/build/var_$v/librlnc_hip.so timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_ragged.py tests/test_gpu_configs.py > $O/tests_$v.log 2>&1
  rc=$?; echo "$v: $(tail -1 $O/tests_$v.log)"
  [ $rc -le 1 ] || { tail -30 $O/tests_$v.log; exit $rc; }
done
for rep in 1 2 3; do
  for lib in product $VARS; do
    if [ $lib = product ]; then unset RLNC_LIB_PATH; else export RLNC_LIB_PATH=$R/build/var_$lib/librlnc_hip.so; fi
    echo "== $lib rep $rep" >> $O/sweep.txt
    timeout -k 10 120 python scripts/sweep.py --objects 32 --configs 8:0 --rounds 12 >> $O/sweep.txt 2>&1 || { tail $O/sweep.txt; exit 1; }
  done
done
unset RLNC_LIB_PATH
grep -E "^==|enc_ms" $O/sweep.txt | paste - - | sed 's/"variant": "bitsliced-jump-shared-8w", "tile_rows": 0, //' | cut -c1-200
for rep in 1 2; do
for lib in product $VARS; do
  if [ $lib = product ]; then unset RLNC_LIB_PATH; else export RLNC_LIB_PATH=$R/build/var_$lib/librlnc_hip.so; fi
  timeout -k 10 300 python bench.py --no-cpu-baseline --no-ceiling > $O/bench_${lib}_$rep.json 2> $O/bench_${lib}_$rep.err || { tail $O/bench_${lib}_$rep.err; exit 1; }
  python3 -c "import json,sys; l=json.loads([x for x in open('$O/bench_${lib}_$rep.json') if x.startswith('{')][-1]); print('$lib', $rep, l['value'], l['ms_per_step'], l['roofline']['kernel_ms'], l['roofline_decode']['kernel_ms'], l['breakdown']['verified'])"
done
done
echo "all done"
