# round 6: composites as VOP3 v_bitop3 in the 8-wave programs only (gen_bsjump.py --combo3-8) against the shipped form
# (parity on the variant, then interleaved A/B: sweep three passes, bench two)
#
set -o pipefail
O=gpurun_out/r06_s14
mkdir -p $O
R=$PWD
VARS="c38"
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
