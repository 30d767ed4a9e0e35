#!/bin/bash
# build a diagnostic variant of liblqro.so: build_variant.sh <out-name> [-Dflags...]
set -e
cd "$(dirname "$0")/../lqr-obstacles_amd"
out=$1; shift
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -fno-fast-math -fPIC -shared "$@" \
  -o "$out" csrc/lqro_runtime.hip csrc/lqro_synth.cpp
