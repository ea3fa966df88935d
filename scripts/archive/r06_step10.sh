# round 6: the decode plan validation (r06_step9.sh), then the wave-priority A/B (r06_step8.sh), in one call
# the encode-plan test, then the bench line with it and without plans (--no-plan), interleaved
set -o pipefail
O=gpurun_out/r06_s9
mkdir -p $O
timeout -k 10 300 python -u -m pytest -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py -k "plan_written_ahead" > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for rep in 1 2; do
  for mode in plan noplan; do
    extra=""; [ $mode = noplan ] && extra="--no-plan"
    timeout -k 10 300 python bench.py --no-cpu-baseline --no-ceiling $extra > $O/bench_${mode}_$rep.json 2> $O/bench_${mode}_$rep.err || { tail $O/bench_${mode}_$rep.err; exit 1; }
    python3 -c "import json; l=json.loads([x for x in open('$O/bench_${mode}_$rep.json') if x.startswith('{')][-1]); b=l['breakdown']; print('$mode', $rep, l['value'], l['ms_per_step'], l['roofline']['kernel_ms'], b['decode_ms'], b['decode_apply_ms'], b['verified'])"
  done
done
bash scripts/archive/r06_step8.sh || exit $?
