# round-5: configs[0] kernel trace (encode then decode), per-kernel medians
set -o pipefail
export TMPDIR=/tmp
O=${1:-gpurun_out/r05_cfg0_prof}
mkdir -p $O
ROUNDS=2 CONFIGS=0 timeout -k 10 200 rocprofv3 --kernel-trace -d $O/trace -o run -- python3 scripts/bench_configs.py > $O/run.log 2>&1 || exit 1
