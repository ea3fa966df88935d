#!/usr/bin/env bash
# Round-5 A/B: the split 2-wave program (gen_bsjump.py --w2split: waves split the byte groups instead of the rows)
# into build/w2var/split/ (a complete library: the parity suite runs on it).
set -eu
cd "$(dirname "$0")/.."
out=$(pwd)/build/w2var/split
mkdir -p "$out/obj"
python3 rlnc_amd/csrc/gen_bsjump.py --w2split --out "$out/bitslice_jump.inc"
scripts/diag_build.sh "$out" "bitslice_jump.inc=$out/bitslice_jump.inc" > /dev/null
rm -rf "$out/src" "$out/obj" "$out/bitslice_jump.inc"
ls -la "$out/librlnc_hip.so"
