#!/usr/bin/env bash
# Round-5 diagnosis: what the combination sets cost the 1- / 2-wave programs on the configs[0] shape.  Timing-only
# variants (wrong bytes): nocombo = no composite entries (11 XORs x 4 sets a source row), nosets = that and the
# transposes replaced by moves.
set -eu
cd "$(dirname "$0")/.."
ROOT=$(pwd)
build() {  # name gen-args...
  name=$1; shift
  out=$ROOT/build/w2var/$name
  mkdir -p "$out/obj"
  python3 rlnc_amd/csrc/gen_bsjump.py --out "$out/bitslice_jump.inc" "$@"
  scripts/diag_build.sh "$out" "bitslice_jump.inc=$out/bitslice_jump.inc" > /dev/null
  rm -rf "$out/src" "$out/obj" "$out/bitslice_jump.inc"
}
build nocombo --diag nocombo &
build nosets --diag nocombo,notrans &
wait
ls -la build/w2var/*/librlnc_hip.so
