# round 6, third GPU call: (1) the set-planes variant of the shared programs (gen_bsjump.py --setplanes, built into
# build/var_sp): parity suites on it, then interleaved A/B against the product library (sweep: the encode launch and
# the 32-row decode product; bench.py lines); (2) the object uploads of Encoder::new / Recoder::new on their own stream
# vs on the leased call stream (RLNC_OBJ_UPLOAD=lease) at the reference's 1 MB recode rows, interleaved
set -o pipefail
O=gpurun_out/r06_s3
mkdir -p $O
R=$PWD
SP=$R/build/var_sp/librlnc_hip.so
RLNC_LIB_PATH=$SP timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_configs.py tests/test_gpu_fullrange.py tests/test_gpu_ragged.py > $O/sp_tests.log 2>&1 || { tail -40 $O/sp_tests.log; exit 1; }
tail -1 $O/sp_tests.log
for rep in 1 2 3; do
  for lib in product sp; do
    if [ $lib = product ]; then unset RLNC_LIB_PATH; else export RLNC_LIB_PATH=$SP; fi
    echo "== $lib rep $rep" >> $O/sweep.txt
    timeout -k 10 120 python scripts/sweep.py --objects 32 --configs 8:0 --rounds 12 >> $O/sweep.txt 2>&1 || { tail $O/sweep.txt; exit 1; }
  done
done
unset RLNC_LIB_PATH
grep -E "^==|enc_ms" $O/sweep.txt | paste - - | cut -c1-220
for rep in 1 2; do
  for lib in product sp; do
    if [ $lib = product ]; then unset RLNC_LIB_PATH; else export RLNC_LIB_PATH=$SP; fi
    timeout -k 10 300 python bench.py --no-cpu-baseline --no-ceiling > $O/bench_${lib}_$rep.json 2> $O/bench_${lib}_$rep.err || { tail $O/bench_${lib}_$rep.err; exit 1; }
    python3 -c "import json,sys; l=json.loads([x for x in open('$O/bench_${lib}_$rep.json') if x.startswith('{')][-1]); print('$lib', $rep, l['value'], l['ms_per_step'], l['roofline']['kernel_ms'], l['roofline_decode']['kernel_ms'], l['breakdown']['verified'])"
  done
done
unset RLNC_LIB_PATH
export OBJ_BENCH_SMALL=1 OBJ_BENCH_ONLY=recode
for rep in 1 2 3; do
  for up in own lease; do
    if [ $up = lease ]; then export RLNC_OBJ_UPLOAD=lease; else unset RLNC_OBJ_UPLOAD; fi
    echo "== upload $up rep $rep" >> $O/recode_ab.txt
    timeout -k 10 120 build/object_api_bench >> $O/recode_ab.txt 2>&1 || { tail $O/recode_ab.txt; exit 1; }
  done
done
for up in own lease; do
  if [ $up = lease ]; then export RLNC_OBJ_UPLOAD=lease; else unset RLNC_OBJ_UPLOAD; fi
  echo "== trace upload $up k=16" >> $O/recode_trace.txt
  RLNC_PIECE_TRACE=1 OBJ_BENCH_K=16 timeout -k 10 120 build/object_api_bench >> $O/recode_trace.txt 2>&1 || { tail $O/recode_trace.txt; exit 1; }
done
cat $O/recode_trace.txt
python3 - <<'PY'
import json, collections
rows = collections.defaultdict(list)
cur = None
for ln in open("gpurun_out/r06_s3/recode_ab.txt"):
    if ln.startswith("=="):
        cur = ln.split()[2]
    elif ln.startswith("{"):
        d = json.loads(ln)
        rows[(cur, d["bench"], d["k"])].append(d["median_us"])
for key in sorted(rows):
    print(key, rows[key])
PY
echo "all done"
