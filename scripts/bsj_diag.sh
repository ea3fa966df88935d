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
  make -s -C rlnc_amd/csrc OUT="$out/librlnc_hip.so" OBJDIR="$out/obj" \
       CXXFLAGS="-O3 -std=c++17 -fPIC -Wall -Wextra -Wno-unused-parameter -DRLNC_BSJ_ASM_FILE=\\\"$out/bitslice_jump.inc\\\""
  echo "built $out/librlnc_hip.so"
done
