#!/bin/bash
# build liblqro variant from a patched copy of csrc: variant.sh <out.so> <patch.py> [-Dflags]
# patch.py edits files in the directory given as argv[1]
set -e
ROOT="$(cd "$(dirname "$0")/.." && pwd)"
out=$1; patch=$2; shift 2
tmp=$(mktemp -d)
mkdir -p "$tmp/lqr-obstacles_amd" "$tmp/include"
cp -r "$ROOT/lqr-obstacles_amd/csrc" "$tmp/lqr-obstacles_amd/"
cp "$ROOT/include/lqro.h" "$tmp/include/"
python3 "$patch" "$tmp/lqr-obstacles_amd/csrc"
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -fno-fast-math -fPIC -shared "$@" \
  -o "$ROOT/lqr-obstacles_amd/$out" "$tmp/lqr-obstacles_amd/csrc/lqro_runtime.hip" "$tmp/lqr-obstacles_amd/csrc/lqro_synth.cpp"
rm -rf "$tmp"
