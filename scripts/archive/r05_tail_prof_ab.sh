# round-5: configs[0] kernel traces with and without the payload-tail answer on one box (elimination cost of the tail)
set -o pipefail
export TMPDIR=/tmp
O=${1:-gpurun_out/r05_tail_prof_ab}
mkdir -p $O
for f in 1 0 1 0; do
  RLNC_FUSED_SCAN=$f ROUNDS=2 CONFIGS=0 timeout -k 10 200 rocprofv3 --kernel-trace -d $O/f$f -o run -- python3 scripts/bench_configs.py >> $O/run_f$f.log 2>&1 || exit 1
done
