# round 6: the 1 MB recode rows (build/object_api_bench, OBJ_BENCH_SMALL=1, OBJ_BENCH_ONLY=recode) under the call
# kernel's remaining knobs, interleaved: default (4 waves at <= 32 sources, 64 workgroups per flag), one flag for the
# whole row (RLNC_PIECE_CHUNK=128: one wait, one copy), and 2 / 8 waves per workgroup (RLNC_PIECE_WAVES)
set -o pipefail
O=gpurun_out/r06_rk
mkdir -p $O
export OBJ_BENCH_SMALL=1 OBJ_BENCH_ONLY=recode
for rep in 1 2 3; do
  for F in def c128 w2 w8; do
    unset RLNC_PIECE_CHUNK RLNC_PIECE_WAVES
    case $F in c128) export RLNC_PIECE_CHUNK=128;; w2) export RLNC_PIECE_WAVES=2;; w8) export RLNC_PIECE_WAVES=8;; esac
    echo "== $F rep $rep" >> $O/grid.txt
    timeout -k 10 120 build/object_api_bench >> $O/grid.txt 2>&1 || { tail $O/grid.txt; exit 1; }
  done
done
python3 - <<'PY'
import json, collections
rows = collections.defaultdict(list)
cur = None
for ln in open("gpurun_out/r06_rk/grid.txt"):
    if ln.startswith("=="):
        cur = ln.split()[1]
    elif ln.startswith("{") and '"bench"' in ln:
        d = json.loads(ln)
        rows[(d["bench"], d["k"], cur)].append(d["median_us"])
for key in sorted(rows):
    print(key, rows[key])
PY
echo "all done"
