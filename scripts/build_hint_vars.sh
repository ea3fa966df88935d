#!/usr/bin/env bash
# Builds librlnc_hip.so variants of the bit-sliced jump program with cache-policy modifiers on the source DMA
# loads and/or the tile stores (gen_bsjump.py --load-hint / --store-hint) into build/var/<name>/, on the CPU here;
# scripts/bsj_layout_ab.sh VARIANTS="..." swaps them in on the GPU box (parity tests, then bench A/B).
set -eu
cd "$(dirname "$0")/.."
ROOT=$(pwd)
build() {  # name load-hint store-hint
  out=$ROOT/build/var/$1
  mkdir -p "$out/obj"
  python3 rlnc_amd/csrc/gen_bsjump.py --out "$out/bitslice_jump.inc" --load-hint "$2" --store-hint "$3"
  scripts/diag_build.sh "$out" "bitslice_jump.inc=$out/bitslice_jump.inc"
}
build stnt "" "nt" &
build ldnt "nt" "" &
build bothnt "nt" "nt" &
[ -n "${SKIP_SC1:-}" ] || build stsc1 "" "sc1" &
wait
