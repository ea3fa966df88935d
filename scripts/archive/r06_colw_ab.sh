# round 6: column-split call-latency kernel (RLNC_PIECE_COLW=W: each wave owns 1 KiB of columns and walks every
# source, W times fewer workgroups) vs the source-split form, at the reference's 1 MB encode / recode rows
# (build/object_api_bench, OBJ_BENCH_SMALL=1), interleaved; parity of the piece tests under each W first
set -o pipefail
O=gpurun_out/r06_colw
mkdir -p $O
for W in 4 16; do
  RLNC_PIECE_COLW=$W timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_piece.py > $O/tests_w$W.log 2>&1 || { tail -30 $O/tests_w$W.log; exit 1; }
  tail -1 $O/tests_w$W.log
done
RLNC_PIECE_COLW=16 RLNC_PIECE_CHUNK=1 timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_piece.py > $O/tests_w16c1.log 2>&1 || { tail -30 $O/tests_w16c1.log; exit 1; }
tail -1 $O/tests_w16c1.log
export OBJ_BENCH_SMALL=1
for rep in 1 2 3; do
  for W in 0 4 8 16 16c1; do
    unset RLNC_PIECE_CHUNK
    case $W in 16c1) export RLNC_PIECE_COLW=16 RLNC_PIECE_CHUNK=1;; *) export RLNC_PIECE_COLW=$W;; esac
    for only in encode recode; do
      echo "== $W $only rep $rep" >> $O/grid.txt
      OBJ_BENCH_ONLY=$only timeout -k 10 120 build/object_api_bench >> $O/grid.txt 2>&1 || { tail $O/grid.txt; exit 1; }
    done
  done
done
unset RLNC_PIECE_CHUNK
for W in 0 4 8 16; do
  echo "== trace $W k=16" >> $O/trace.txt
  RLNC_PIECE_COLW=$W RLNC_PIECE_TRACE=1 OBJ_BENCH_K=16 OBJ_BENCH_ONLY=recode timeout -k 10 120 build/object_api_bench >> $O/trace.txt 2>&1 || { tail $O/trace.txt; exit 1; }
done
grep -v "^{\"bench\"" $O/trace.txt | head -40
python3 - <<'PY'
import json, collections
rows = collections.defaultdict(list)
cur = None
for ln in open("gpurun_out/r06_colw/grid.txt"):
    if ln.startswith("=="):
        cur = ln.split()[1]
    elif ln.startswith("{") and '"bench"' in ln:
        d = json.loads(ln)
        rows[(d["bench"], d["k"], cur)].append(d["median_us"])
for key in sorted(rows):
    print(key, rows[key], "epyc")
PY
echo "all done"
