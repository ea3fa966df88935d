# round 6: one flag per row (RLNC_PIECE_CHUNK=128) vs the shipped 64 workgroups per flag at k = 16 (65 workgroups: two
# chunks under the default, one under c128), ABBA order over four passes so the pass position cancels; encode + recode
set -o pipefail
O=gpurun_out/r06_abba
mkdir -p $O
export OBJ_BENCH_SMALL=1 OBJ_BENCH_K=16
for F in def c128 c128 def def c128 c128 def; do
  unset RLNC_PIECE_CHUNK
  [ $F = c128 ] && export RLNC_PIECE_CHUNK=128
  for only in encode recode; do
    echo "== $F $only" >> $O/grid.txt
    OBJ_BENCH_ONLY=$only timeout -k 10 120 build/object_api_bench >> $O/grid.txt 2>&1 || { tail $O/grid.txt; exit 1; }
  done
done
python3 - <<'PY'
import json, collections
rows = collections.defaultdict(list)
cur = None
for ln in open("gpurun_out/r06_abba/grid.txt"):
    if ln.startswith("=="):
        cur = ln.split()[1]
    elif ln.startswith("{") and '"bench"' in ln:
        d = json.loads(ln)
        rows[(d["bench"], d["k"], cur)].append(d["median_us"])
for key in sorted(rows):
    v = rows[key]
    print(key, v, "median", sorted(v)[len(v) // 2])
PY
echo "all done"
