#!/usr/bin/env bash
# Timing diagnostics of gf_matmul_bs_kernel: builds librlnc_hip.so variants whose inner program drops the
# source loads ("novm") and/or the per-step index reloads ("nosmem") — WRONG results, timing only — into
# build/diag_<name>/, on the CPU here.  On the GPU box: RLNC_LIB_PATH=build/diag_<name>/librlnc_hip.so
# RLNC_DIAG=1 python scripts/sweep.py --configs 5:0 (RLNC_DIAG skips the cross-variant equality check).
set -eu
cd "$(dirname "$0")/.."
ROOT=$(pwd)
for d in ${DIAGS:-novm nosmem novm,nosmem}; do
  name=${d//,/_}
  out=$ROOT/build/diag_$name
  mkdir -p "$out/obj"
  python3 rlnc_amd/csrc/gen_bitslice.py --diag "$d" --out "$out/bitslice_asm.inc"
  AB=1 scripts/diag_build.sh "$out" "bitslice_asm.inc=$out/bitslice_asm.inc"  # variant 5 lives in the A/B build
done
