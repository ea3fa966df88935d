# round-5 GPU step 3: small-elimination timeline and NW A/B (diagnostic build), host page-fault microbenchmark,
# large get_decoded_data copy-out A/B (huge pages, threads) on the decode rows of the object-API grid
set -o pipefail
O=${1:-gpurun_out/r05c}
mkdir -p $O
AB=$PWD/rlnc_amd/librlnc_hip_ab.so
RLNC_LIB_PATH=$AB timeout -k 10 120 python scripts/elim_small_prof.py > $O/elim_prof.jsonl 2> $O/elim_prof.err || { tail $O/elim_prof.err; exit 1; }
cat $O/elim_prof.jsonl
for nw in 1 2 4 8; do
  RLNC_LIB_PATH=$AB RLNC_SMALL_NW=$nw timeout -k 10 120 python scripts/elim_small_probe.py 2>/dev/null | sed "s/^{/{\"nw\": $nw, /" >> $O/elim_nw.jsonl || exit 1
done
cat $O/elim_nw.jsonl
timeout -k 10 200 build/ubench_fault > $O/fault.jsonl 2>&1 || exit 1
cat $O/fault.jsonl
for hp in 1 0; do for th in 8 16 4; do
  RLNC_COPY_HUGEPAGE=$hp RLNC_COPY_THREADS=$th OBJ_BENCH_ONLY=decode timeout -k 10 300 build/object_api_bench 2>/dev/null | grep '"data_bytes": 3355\|"data_bytes": 1677' | sed "s/^{/{\"hugepage\": $hp, \"threads\": $th, /" >> $O/copyout_ab.jsonl || exit 1
done; done
echo "all done"
