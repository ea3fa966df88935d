# piece-path A/B at the 1 MB rows: waves per workgroup (RLNC_PIECE_WAVES; default = n_in rounded up to a power of two,
# at most 16)
set -o pipefail
mkdir -p gpurun_out
rm -f gpurun_out/piece_ab.txt
export OBJ_BENCH_SMALL=1
for cfg in "RLNC_PIECE_WAVES=0" "RLNC_PIECE_WAVES=4" "RLNC_PIECE_WAVES=8" "RLNC_PIECE_WAVES=2" "RLNC_PIECE_WAVES=0"; do
  for only in encode recode; do
    echo "== $cfg $only" >> gpurun_out/piece_ab.txt
    env $cfg OBJ_BENCH_ONLY=$only timeout -k 10 60 build/object_api_bench --quick >> gpurun_out/piece_ab.txt 2>&1
  done
done
