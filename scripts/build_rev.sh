#!/bin/bash
# build liblqro from a git revision: build_rev.sh <rev> <out.so>   (A/B baselines)
set -e
ROOT="$(cd "$(dirname "$0")/.." && pwd)"
tmp=$(mktemp -d)
git -C "$ROOT" archive "$1" lqr-obstacles_amd/csrc include | tar -x -C "$tmp"
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -fno-fast-math -fPIC -shared \
  -o "$ROOT/lqr-obstacles_amd/$2" "$tmp/lqr-obstacles_amd/csrc/lqro_runtime.hip" "$tmp/lqr-obstacles_amd/csrc/lqro_synth.cpp"
rm -rf "$tmp"
