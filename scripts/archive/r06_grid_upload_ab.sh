# round 6: Recoder::new uploading small objects with a copy kernel on the recode call's grid (default after this
# change) vs the DMA upload (RLNC_GRID_UPLOAD=0): parity suites on the new default, then the 1 MB recode rows in ABBA
# order with Recoder::new's own time beside the call's (new_median_us)
set -o pipefail
O=gpurun_out/r06_gu
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_piece.py tests/test_gpu_api.py tests/test_gpu_boundary.py tests/test_gpu_configs.py tests/test_gpu_parity.py tests/test_gpu_lifetime.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
export OBJ_BENCH_SMALL=1 OBJ_BENCH_ONLY=recode
for F in grid dma dma grid grid dma dma grid; do
  unset RLNC_GRID_UPLOAD
  [ $F = dma ] && export RLNC_GRID_UPLOAD=0
  echo "== $F" >> $O/grid.txt
  timeout -k 10 120 build/object_api_bench >> $O/grid.txt 2>&1 || { tail $O/grid.txt; exit 1; }
done
python3 - <<'PY'
import json, collections
rows = collections.defaultdict(list); new = collections.defaultdict(list)
cur = None
for ln in open("gpurun_out/r06_gu/grid.txt"):
    if ln.startswith("=="):
        cur = ln.split()[1]
    elif ln.startswith("{") and '"bench"' in ln:
        d = json.loads(ln)
        rows[(d["bench"], d["k"], cur)].append(d["median_us"])
        if "new_median_us" in d:
            new[(d["k"], cur)].append(d["new_median_us"])
for key in sorted(rows):
    v = rows[key]; print(key, v, "mean %.2f" % (sum(v) / len(v)))
for key in sorted(new):
    v = new[key]; print("Recoder::new", key, v, "mean %.2f" % (sum(v) / len(v)))
PY
echo "all done"
