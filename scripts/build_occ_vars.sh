#!/usr/bin/env bash
# Round-5 A/B: is the 2-wave bit-sliced program (configs[0] shape) latency- or issue-bound?  Its workgroups given
# extra dynamic LDS so fewer fit on a CU: occ1 = 60,000 B (2 workgroups = 1 wave per SIMD instead of 2), occctl =
# 20,000 B (still VGPR-limited at 2 waves per SIMD: the control).
set -eu
cd "$(dirname "$0")/.."
ROOT=$(pwd)
build() {  # name dynamic-lds-bytes
  out=$ROOT/build/w2var/$1
  mkdir -p "$out/obj"
  sed "s/hipLaunchKernelGGL(gf_matmul_bsj_kernel<2>, grid, dim3(128), 0, s/hipLaunchKernelGGL(gf_matmul_bsj_kernel<2>, grid, dim3(128), $2, s/" rlnc_amd/csrc/kernels.hip > "$out/kernels.hip"
  grep -q "dim3(128), $2, s" "$out/kernels.hip"
  scripts/diag_build.sh "$out" "kernels.hip=$out/kernels.hip" > /dev/null
  rm -rf "$out/src" "$out/obj" "$out/kernels.hip"
}
build occ1 60000 &
build occctl 20000 &
wait
ls -la build/w2var/*/librlnc_hip.so
