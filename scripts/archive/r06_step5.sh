# round 6, fifth GPU call: the per-term breakdown of the 8-wave unit again, on the set-planes form (s8nocombo: the
# 44 composite XORs per source row skipped), then the call-latency path's completion granularity (RLNC_PIECE_CHUNK
# = workgroups per host flag: 64 default, 16, 32) at the reference's 1 MB rows, three interleaved passes
set -o pipefail
O=gpurun_out/r06_s5
mkdir -p $O
DIAGS="s8inline s8noread s8noown s8nobar s8nocombo" bash scripts/archive/r06_unit_breakdown.sh $O/unit > /dev/null || exit $?
grep -E "^==|enc_ms" $O/unit/sweep.txt | paste - - | sed 's/"variant": "bitsliced-jump-shared-8w", "tile_rows": 0, //' | cut -c1-200
export OBJ_BENCH_SMALL=1
for rep in 1 2 3; do
  for c in 64 16 32; do
    echo "== chunk $c rep $rep" >> $O/chunk_ab.txt
    RLNC_PIECE_CHUNK=$c timeout -k 10 120 build/object_api_bench >> $O/chunk_ab.txt 2>&1 || { tail $O/chunk_ab.txt; exit 1; }
  done
done
python3 - <<'PY'
import json, collections
rows = collections.defaultdict(list)
cur = None
for ln in open("gpurun_out/r06_s5/chunk_ab.txt"):
    if ln.startswith("=="):
        cur = int(ln.split()[2])
    elif ln.startswith("{"):
        d = json.loads(ln)
        if "median_us" in d:
            rows[(d["bench"], d["k"], cur)].append(d["median_us"])
for key in sorted(rows):
    print(key, rows[key])
PY
echo "all done"
