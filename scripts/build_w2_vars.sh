#!/usr/bin/env bash
# Round-5 diagnosis of the 2-wave bit-sliced program on the configs[0] shape (16 x 4 KiB per object): variants of
# gen_bsjump.py into build/w2var/<name>/ (timing-only ones, marked *, compute wrong bytes):
#   slots5   a 5-slot source ring (4 rows in flight instead of 2)
#   nosmem*  every row reuses the prologue's block offsets (no per-row scalar load of the offset stream)
#   novm*    no source DMA (the program's compute and stores alone)
set -eu
cd "$(dirname "$0")/.."
ROOT=$(pwd)
build() {  # name gen-args...
  name=$1; shift
  out=$ROOT/build/w2var/$name
  mkdir -p "$out/obj"
  python3 rlnc_amd/csrc/gen_bsjump.py --out "$out/bitslice_jump.inc" "$@"
  scripts/diag_build.sh "$out" "bitslice_jump.inc=$out/bitslice_jump.inc" > /dev/null
}
build slots5 --slots2 5 &
build nosmem --diag nosmem &
build novm --diag novm &
build slots5nosmem --slots2 5 --diag nosmem &
wait
ls -la build/w2var/*/librlnc_hip.so
