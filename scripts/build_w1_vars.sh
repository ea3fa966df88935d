#!/usr/bin/env bash
# Round-5 A/B for the configs[0] shape: products of 9-16 rows as two 1-wave row tiles (64-thread workgroups, no
# per-row barrier, each wave its own DMA) instead of one 2-wave tile (the elimination then leaves the product's
# block offsets to the offset kernel: its stream is laid out for one row tile); w1s5: the same with a 5-slot source ring.
set -eu
cd "$(dirname "$0")/.."
ROOT=$(pwd)
build() {  # name gen-args...
  name=$1; shift
  out=$ROOT/build/w2var/$name
  mkdir -p "$out/obj"
  python3 rlnc_amd/csrc/gen_bsjump.py --out "$out/bitslice_jump.inc" "$@"
  sed 's/return n_out <= 8 ? 1 : n_out <= 16 ? 2 : 4;/return n_out <= 16 ? 1 : 4;/; s/return bsj_waves(n_out) <= 2 ? kBsjWaveRows \* bsj_waves(n_out) : 0;/return n_out <= kBsjWaveRows ? kBsjWaveRows : 0;/' rlnc_amd/csrc/kernels.hip > "$out/kernels.hip"
  scripts/diag_build.sh "$out" "bitslice_jump.inc=$out/bitslice_jump.inc" "kernels.hip=$out/kernels.hip" > /dev/null
}
build w1 &
build w1s5 --slots1 5 &
wait
ls -la build/w2var/w1*/librlnc_hip.so
