# round 6: the bench's other modes still run and verify after this round's changes (pipeline 0 / 1, --no-plan, --graph 1,
# --encode-only, --variant 7), short runs
set -o pipefail
O=gpurun_out/r06_modes
mkdir -p $O
for m in "--pipeline 0" "--pipeline 1" "--no-plan" "--graph 1" "--encode-only" "--variant 7"; do
  n=$(echo $m | tr -d ' -')
  timeout -k 10 300 python bench.py --steps 5 --warmup 2 --breakdown-steps 4 --no-cpu-baseline --no-ceiling $m > $O/$n.json 2> $O/$n.err || { echo "FAIL $m"; tail $O/$n.err; exit 1; }
  python3 -c "import json; l=json.loads([x for x in open('$O/$n.json') if x.startswith('{')][-1]); print('$m', l['value'], l['ms_per_step'], l['breakdown']['verified'], l['roofline']['kernel'][:60], (l['roofline_decode'] or {}).get('kernel_ms'))"
done
echo "all done"
