# round 6: the reference's 1 MB rows (encode and recode benches) on the round-5 library + its bench build (build/r05)
# against head's, interleaved on one box: is the recode's spread across round 6's boxes the code or the boxes?
set -o pipefail
O=gpurun_out/r06_s12
mkdir -p $O
export OBJ_BENCH_SMALL=1
for rep in 1 2 3; do
  for lib in head r05; do
    b=build/object_api_bench; [ $lib = r05 ] && b=build/r05/object_api_bench
    echo "== $lib rep $rep" >> $O/grid_ab.txt
    timeout -k 10 120 $b >> $O/grid_ab.txt 2>&1 || { tail $O/grid_ab.txt; exit 1; }
  done
done
python3 - <<'PY'
import json, collections
rows = collections.defaultdict(list)
cur = None
for ln in open("gpurun_out/r06_s12/grid_ab.txt"):
    if ln.startswith("=="):
        cur = ln.split()[1]
    elif ln.startswith("{"):
        d = json.loads(ln)
        if "median_us" in d and d["bench"] != "decode":
            rows[(d["bench"], d["k"], cur)].append(d["median_us"])
for key in sorted(rows):
    print(key, rows[key])
PY
echo "all done"
