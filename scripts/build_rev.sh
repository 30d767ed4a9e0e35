#!/bin/bash
# build liblqro from a git revision: build_rev.sh <rev> <out.so>   (A/B baselines)
# (revisions before the split into objects are built as one hipcc command)
set -e
ROOT="$(cd "$(dirname "$0")/.." && pwd)"
tmp=$(mktemp -d)
git -C "$ROOT" archive "$1" lqr-obstacles_amd/csrc include | tar -x -C "$tmp"
if [ -f "$tmp/lqr-obstacles_amd/csrc/lqro_pair_inst.hip" ]; then
  python3 - "$ROOT" "$tmp" "$2" <<'P'
import os, sys
root, tmp, out = sys.argv[1:]
sys.path.insert(0, root)
import __graft_entry__ as g
objs = g.lib_objects(build_dir=os.path.join(tmp, "build"), csrc=os.path.join(tmp, "lqr-obstacles_amd", "csrc"))
g.link_objects(os.path.join(root, "lqr-obstacles_amd", out), objs)
P
else
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -fno-fast-math -fPIC -shared \
    -o "$ROOT/lqr-obstacles_amd/$2" "$tmp/lqr-obstacles_amd/csrc/lqro_runtime.hip" "$tmp/lqr-obstacles_amd/csrc/lqro_synth.cpp"
fi
rm -rf "$tmp"
