# round-4 GPU step: HBM traffic of configs[0]'s small products (4,096 objects x 16 x 4 KiB, encode + decode): two
# separate PMC passes (FETCH_SIZE, WRITE_SIZE), each rocprofv3 --kernel-trace --pmc only, program after --
set -u
R=$PWD
OUT=$R/gpurun_out/pmc_cfg0
rm -rf "$OUT"; mkdir -p "$OUT"
export TMPDIR=/tmp CONFIGS=0 ROUNDS=1
cd /tmp
i=0
for group in FETCH_SIZE WRITE_SIZE; do
  i=$((i+1))
  timeout -k 10 -s KILL 120 rocprofv3 --kernel-trace --pmc $group -d "$OUT/p$i" -o run --output-format csv -- \
      python3 "$R/scripts/bench_configs.py" > "$OUT/p$i.log" 2>&1
  rc=$?; echo "pmc pass $i ($group) rc=$rc"
  [ $rc -ne 0 ] && exit $rc
done
python3 "$R/scripts/pmc_summary.py" "$OUT" > "$OUT/summary.jsonl" 2>&1; grep -E "bsj|rref|final_len" "$OUT/summary.jsonl"
