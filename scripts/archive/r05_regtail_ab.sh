# round-5 A/B: payload tails prefetched into registers (build/w2var/regtail, G = 8 kernel) against the LDS-DMA staging
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05_regtail
mkdir -p $O
for v in base regtail base regtail; do
  if [ $v = base ]; then l=$PWD/rlnc_amd/librlnc_hip.so; else l=$PWD/build/w2var/regtail/librlnc_hip.so; fi
  rm -rf $O/$v
  RLNC_LIB_PATH=$l ROUNDS=2 CONFIGS=0 timeout -k 10 200 rocprofv3 --kernel-trace -d $O/$v -o run -- python3 scripts/bench_configs.py >> $O/run_$v.log 2>&1 || exit 1
  python3 - $O/$v <<'PY'
import sqlite3,glob,statistics as st,sys
db=glob.glob(sys.argv[1]+'/**/*.db',recursive=True)[0]
c=sqlite3.connect(db); rows=list(c.execute("select name, start, end, duration from kernels order by start"))
el=[r[3]/1e3 for r in rows if 'rref_small' in r[0]]
dec=[]
for i,(n,s,e,d) in enumerate(rows):
    if 'rref_small' in n:
        j=i+1
        while j<len(rows) and 'gf_matmul_bsj' not in rows[j][0]: j+=1
        dec.append((rows[j][2]-s)/1e3)
print(sys.argv[1], "elim", round(st.median(el),2), "decode span", round(st.median(dec),2))
PY
done
for v in base regtail; do
  if [ $v = base ]; then l=$PWD/rlnc_amd/librlnc_hip.so; else l=$PWD/build/w2var/regtail/librlnc_hip.so; fi
  r=$(RLNC_LIB_PATH=$l CONFIGS=0 timeout -k 10 120 python scripts/bench_configs.py 2>/dev/null) || exit 1
  echo "$v $(echo $r | grep -o '"decode_ms[^,]*,\|"verified[^,}]*' | tr '\n' ' ')"
done
