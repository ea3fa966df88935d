# A/B of the large get_decoded_data copy-out: pre-faulting the caller's buffer (RLNC_COPY_TOUCH) on / off
set -o pipefail
O=gpurun_out/r05_copyout
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_piece.py tests/test_gpu_cpp.py tests/test_gpu_boundary.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for rep in 1 2; do for t in 1 0; do
  RLNC_COPY_TRACE=1 RLNC_COPY_TOUCH=$t OBJ_BENCH_ONLY=decode timeout -k 10 300 build/object_api_bench 2> $O/trace_$t.err | grep '"data_bytes": 3355\|"data_bytes": 1677' | sed "s/^{/{\"touch\": $t, \"rep\": $rep, /" >> $O/ab.jsonl || exit 1
  grep copy_trace $O/trace_$t.err | sed "s/^{/{\"touch\": $t, /"
done; done
python3 -c "
import json
for l in open('$O/ab.jsonl'):
    r=json.loads(l); print(r['touch'], r['rep'], r['data_bytes']>>20, r['k'], 'get', r['get_decoded_data_median_us'])
"
