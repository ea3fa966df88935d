# A/B: the small-object elimination with / without the progress-based wave priority (build/noprio: -DRLNC_SMALL_PRIO=0)
set -o pipefail
O=gpurun_out/r05_prio
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_parity.py -k "small or decode" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for rep in 1 2 3; do
  for lib in rlnc_amd/librlnc_hip.so build/noprio/librlnc_hip.so; do
    RLNC_LIB_PATH=$PWD/$lib timeout -k 10 120 python scripts/elim_small_probe.py 2>/dev/null | sed "s#^{#{\"lib\": \"$lib\", #" >> $O/ab.jsonl || exit 1
    RLNC_LIB_PATH=$PWD/$lib CONFIGS=0 timeout -k 10 120 python scripts/bench_configs.py 2>/dev/null | sed "s#^{#{\"lib\": \"$lib\", #" >> $O/ab.jsonl || exit 1
  done
done
python3 -c "
import json
for l in open('$O/ab.jsonl'):
    r=json.loads(l); print(r['lib'], r.get('ms', r.get('decode_ms')), r.get('what', 'cfg0 decode'))
"
