#!/bin/bash
# build a diagnostic variant of liblqro.so: build_variant.sh <out-name> [-Dflags...]
# (the same objects as __graft_entry__.build_lib, compiled with the extra flags
# into build/<out-name>/)
set -e
cd "$(dirname "$0")/.."
out=$1; shift
python3 - "$out" "$@" <<'P'
import os, sys
sys.path.insert(0, os.getcwd())
import __graft_entry__ as g
out, flags = sys.argv[1], sys.argv[2:]
objs = g.lib_objects(flags, build_dir=os.path.join("build", out))
g.link_objects(os.path.join("lqr-obstacles_amd", out), objs)
P
