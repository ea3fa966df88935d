# round 6: balanced completion chunks (shipped after this run if it holds) -- the GPU suite on them, then ABBA against
# the previous rule (RLNC_PIECE_CHUNK=64 reproduces it: 64 workgroups per flag, tail chunk kept) at the 1 MB rows
set -o pipefail
O=gpurun_out/r06_bal
mkdir -p $O
timeout -k 10 900 python -u -m pytest -q --timeout 120 --timeout-method thread -m gpu tests > $O/gpu_tests.log 2>&1
rc=$?; tail -1 $O/gpu_tests.log
[ $rc -eq 0 ] || { grep -E "FAILED|ERROR" $O/gpu_tests.log | head -20; exit 1; }
export OBJ_BENCH_SMALL=1
for F in bal c64 c64 bal bal c64 c64 bal; do
  unset RLNC_PIECE_CHUNK
  [ $F = c64 ] && export RLNC_PIECE_CHUNK=64
  for only in encode recode; do
    echo "== $F $only" >> $O/grid.txt
    OBJ_BENCH_ONLY=$only timeout -k 10 120 build/object_api_bench >> $O/grid.txt 2>&1 || { tail $O/grid.txt; exit 1; }
  done
done
python3 - <<'PY'
import json, collections
rows = collections.defaultdict(list)
cur = None
for ln in open("gpurun_out/r06_bal/grid.txt"):
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
