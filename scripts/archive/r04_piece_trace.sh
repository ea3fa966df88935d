# round-4 GPU step: host-side breakdown of the call-latency path (RLNC_PIECE_TRACE) for the 1 MB encode and recode
# rows at k = 16 / 32 / 64 (a fresh Recoder per recode sample, as the reference's bench)
set -o pipefail
mkdir -p gpurun_out/trace
export OBJ_BENCH_SMALL=1 RLNC_PIECE_TRACE=1
for k in ${TRACE_KS:-16 32 64}; do
  for only in ${TRACE_OPS:-encode recode}; do
    echo "== k=$k $only" >> gpurun_out/trace/trace.txt
    OBJ_BENCH_K=$k OBJ_BENCH_ONLY=$only timeout -k 10 60 build/object_api_bench --quick >> gpurun_out/trace/trace.txt 2>&1 || exit 1
  done
done
grep -v amdgpu gpurun_out/trace/trace.txt
