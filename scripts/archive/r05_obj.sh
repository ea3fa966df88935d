# the object-API grid (five benches x 15 shapes), and the large decodes' copy-out phases (RLNC_COPY_TRACE)
set -o pipefail
O=${1:-gpurun_out/r05_obj}
mkdir -p $O
timeout -k 10 500 build/object_api_bench > $O/object_api_bench.jsonl 2> $O/object_api_bench.err || { tail $O/object_api_bench.err; exit 1; }
for k in 16 256; do
  RLNC_COPY_TRACE=1 OBJ_BENCH_ONLY=decode OBJ_BENCH_K=$k timeout -k 10 200 build/object_api_bench > $O/trace_k$k.jsonl 2> $O/trace_k$k.err || { tail $O/trace_k$k.err; exit 1; }
done
cat $O/trace_k*.err | grep copy_trace
grep '"decode"' $O/object_api_bench.jsonl | cut -c1-260
