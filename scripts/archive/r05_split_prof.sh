# round-5: kernel durations of configs[0] (encode, then decode) under the shipped and the split 2-wave program
set -o pipefail
export TMPDIR=/tmp
for v in base split; do
  if [ $v = base ]; then l=$PWD/rlnc_amd/librlnc_hip.so; else l=$PWD/build/w2var/split/librlnc_hip.so; fi
  RLNC_LIB_PATH=$l ROUNDS=2 CONFIGS=0 timeout -k 10 200 rocprofv3 --kernel-trace -d gpurun_out/r05_split_prof/$v -o run -- python3 scripts/bench_configs.py > gpurun_out/r05_split_prof/$v.log 2>&1 || exit 1
done
