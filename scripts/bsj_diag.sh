#!/usr/bin/env bash
# Diagnostic builds of the jump variant (gen_bsjump.py --diag / --stride / --align) into build/diag_<name>/:
# DIAGS="name:generator-args ..." e.g. "inline:--diag=inline s160:--stride=160+--align=6" (+ separates arguments).  Timing only.
set -eu
cd "$(dirname "$0")/.."
ROOT=$(pwd)
for spec in $DIAGS; do
  name=${spec%%:*}; args=${spec#*:}; args=${args//+/ }
  out=$ROOT/build/diag_$name
  mkdir -p "$out/obj"
  python3 rlnc_amd/csrc/gen_bsjump.py $args --out "$out/bitslice_jump.inc"
  scripts/diag_build.sh "$out" "bitslice_jump.inc=$out/bitslice_jump.inc"
done
