#!/usr/bin/env bash
# Diagnostic library builds without diagnostic code in the shipped sources: copy rlnc_amd/csrc into <out>/src/csrc,
# substitute files (name=path: e.g. a generated bitslice_jump.inc variant, or kernels.hip=<variant>),
# build <out>/librlnc_hip.so there (AB=1: the A/B library, make ab), extra compiler flags after --.
#   scripts/diag_build.sh build/diag_x bitslice_jump.inc=build/diag_x/bitslice_jump.inc -- -DFOO
set -eu
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
out=$1; shift
mkdir -p "$out" && out=$(cd "$out" && pwd)
rm -rf "$out/src" && mkdir -p "$out/src/csrc"
cp -p rlnc_amd/csrc/*.hip rlnc_amd/csrc/*.hpp rlnc_amd/csrc/*.cpp rlnc_amd/csrc/*.inc rlnc_amd/csrc/*.py rlnc_amd/csrc/Makefile "$out/src/csrc/"
rm -rf "$out/include" && cp -r include "$out/include"  # the sources include ../../include/rlnc_hip.h
flags=""
while [ $# -gt 0 ]; do
  if [ "$1" = "--" ]; then shift; flags="$*"; break; fi
  cp "${1#*=}" "$out/src/csrc/${1%%=*}"
  shift
done
cxx="-O3 -std=c++17 -fPIC -Wall -Wextra -Wno-unused-parameter $flags"
if [ "${AB:-0}" = 1 ]; then
  make -s -C "$out/src/csrc" ab AB_OUT="$out/librlnc_hip.so" AB_OBJDIR="$out/obj" CXXFLAGS="$cxx"
else
  make -s -C "$out/src/csrc" OUT="$out/librlnc_hip.so" OBJDIR="$out/obj" CXXFLAGS="$cxx"
fi
echo "built $out/librlnc_hip.so"
