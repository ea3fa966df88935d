# round 6: HIP runtime launch settings at the reference's 1 MB encode / recode rows (build/object_api_bench,
# OBJ_BENCH_SMALL=1), interleaved: default, kernel arguments forced into device memory (HIP_FORCE_DEV_KERNARG=1) and
# forced into host memory (=0); then the k = 16 recode call traced under each
set -o pipefail
O=gpurun_out/r06_env
mkdir -p $O
export OBJ_BENCH_SMALL=1
for rep in 1 2 3; do
  for E in def dk1 dk0; do
    unset HIP_FORCE_DEV_KERNARG
    case $E in dk1) export HIP_FORCE_DEV_KERNARG=1;; dk0) export HIP_FORCE_DEV_KERNARG=0;; esac
    for only in encode recode; do
      echo "== $E $only rep $rep" >> $O/grid.txt
      OBJ_BENCH_ONLY=$only timeout -k 10 120 build/object_api_bench >> $O/grid.txt 2>&1 || { tail $O/grid.txt; exit 1; }
    done
  done
done
for E in def dk1 dk0; do
  unset HIP_FORCE_DEV_KERNARG
  case $E in dk1) export HIP_FORCE_DEV_KERNARG=1;; dk0) export HIP_FORCE_DEV_KERNARG=0;; esac
  echo "== trace $E k=16" >> $O/trace.txt
  RLNC_PIECE_TRACE=1 OBJ_BENCH_K=16 OBJ_BENCH_ONLY=recode timeout -k 10 120 build/object_api_bench >> $O/trace.txt 2>&1 || { tail $O/trace.txt; exit 1; }
done
unset HIP_FORCE_DEV_KERNARG
grep -v '^{"bench"' $O/trace.txt
python3 - <<'PY'
import json, collections
rows = collections.defaultdict(list)
cur = None
for ln in open("gpurun_out/r06_env/grid.txt"):
    if ln.startswith("=="):
        cur = ln.split()[1]
    elif ln.startswith("{") and '"bench"' in ln:
        d = json.loads(ln)
        rows[(d["bench"], d["k"], cur)].append(d["median_us"])
for key in sorted(rows):
    print(key, rows[key])
PY
echo "all done"
