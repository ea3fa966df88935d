# A/B: the encode's code-block address stream written ahead on the side stream (default) vs in front of the product on
# the launch stream (--no-plan); 3 interleaved repetitions of the default bench step (no CPU baseline, no ceilings)
set -o pipefail
O=gpurun_out/r05_plan
mkdir -p $O
for rep in 1 2 3; do
  for mode in plan noplan; do
    extra=""; [ $mode = noplan ] && extra="--no-plan"
    timeout -k 10 300 python bench.py --no-cpu-baseline --no-ceiling $extra 2> $O/err_$mode.log | grep '^{' > $O/line.json || { tail $O/err_$mode.log; exit 1; }
    python3 -c "
import json
d=json.load(open('$O/line.json'))
print(json.dumps({'mode': '$mode', 'rep': $rep, 'value': d['value'], 'ms_per_step': d['ms_per_step'], 'kernel_ms': d['roofline']['kernel_ms'], 'decode_ms': d['breakdown']['decode_ms'], 'verified': d['breakdown']['verified']}))
" >> $O/ab.jsonl
  done
done
cat $O/ab.jsonl
