# round-4 GPU step: Recoder::new's upload through pinned staging (default) vs the pageable 2D copy
# (RLNC_RECODER_STAGE=0), then the recode call that follows (1 MB rows, a fresh Recoder per sample), interleaved 3x
set -o pipefail
mkdir -p gpurun_out/stage_ab
export OBJ_BENCH_SMALL=1 OBJ_BENCH_ONLY=recode
for rep in 1 2 3; do
  for v in 1 0; do
    echo "== RLNC_RECODER_STAGE=$v" >> gpurun_out/stage_ab/calls.txt
    RLNC_RECODER_STAGE=$v timeout -k 10 60 build/object_api_bench --quick >> gpurun_out/stage_ab/calls.txt 2>&1 || exit 1
  done
done
grep -v amdgpu gpurun_out/stage_ab/calls.txt | python3 -c "
import sys,json
from collections import defaultdict
cur=None; r=defaultdict(list)
for l in sys.stdin:
    if l.startswith('=='): cur=l.strip()[3:]; continue
    if l.startswith('{'):
        d=json.loads(l); r[(cur,d['k'])].append(d['median_us'])
for (c,k),v in sorted(r.items()): print(c,k,v)
"
