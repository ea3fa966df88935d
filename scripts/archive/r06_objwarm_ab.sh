# round 6: Recoder::new followed by one throwaway call-kernel pass over the fresh pieces (RLNC_OBJ_WARM=1: zero
# coefficients, the recode call's grid, so the lines sit in the L2 of the XCD that reads them) vs the shipped create,
# at the 1 MB recode rows (build/object_api_bench times only the recode call, the create is outside, as in divan),
# ABBA order; piece parity under the knob first
set -o pipefail
O=gpurun_out/r06_ow
mkdir -p $O
RLNC_OBJ_WARM=1 timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_piece.py tests/test_gpu_api.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
export OBJ_BENCH_SMALL=1 OBJ_BENCH_ONLY=recode
for F in def warm warm def def warm warm def; do
  unset RLNC_OBJ_WARM
  [ $F = warm ] && export RLNC_OBJ_WARM=1
  echo "== $F" >> $O/grid.txt
  timeout -k 10 120 build/object_api_bench >> $O/grid.txt 2>&1 || { tail $O/grid.txt; exit 1; }
done
python3 - <<'PY'
import json, collections
rows = collections.defaultdict(list)
cur = None
for ln in open("gpurun_out/r06_ow/grid.txt"):
    if ln.startswith("=="):
        cur = ln.split()[1]
    elif ln.startswith("{") and '"bench"' in ln:
        d = json.loads(ln)
        rows[(d["bench"], d["k"], cur)].append(d["median_us"])
for key in sorted(rows):
    v = rows[key]
    print(key, v, "mean %.2f" % (sum(v) / len(v)))
PY
echo "all done"
