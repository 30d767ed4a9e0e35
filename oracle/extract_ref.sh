#!/bin/sh
# Build-time extraction of the reference's own per-pair path functions into a
# scratch directory OUTSIDE the repository (default /tmp/lqro_ref_extract, see
# Makefile), so that no reference source sits in the tree that is pushed to
# the GPU box.  Used only to compile the
# reference itself as an oracle (oracle/_ref/libref.so, see Makefile).
#
# The reference's translation unit (LQRObstacles.cpp) cannot be compiled as a
# whole here: it needs <tchar.h> and the Win32 Callisto visualisation library.
# We do NOT write stand-ins for those.  Instead the harness (ref_harness.cpp)
# compiles the line ranges that hold the path's functions, verbatim, against
# the reference's own headers (include/matrix.h, gjk.h, Vector3.h) and
# gjk.cpp.  The line ranges are pinned to the file hashes below.
set -e
REF="$1"
OUT="$2"
Q="$REF/QuadrotorHoverController"
mkdir -p "$OUT"

check() {
  h=$(sha256sum "$1" | cut -d' ' -f1)
  if [ "$h" != "$2" ]; then
    echo "extract_ref.sh: $1 does not match the pinned reference revision" >&2
    exit 3
  fi
}
check "$Q/LQRObstacles.cpp" f3d1ff4b5f9fed508336153459bc39e3807d6af1e373435d0caf72c666f97493
check "$Q/stdafx.h"         88c34fd8ce0264e84e1e0e99cb823197fa9911f2cbe9f38edccd61b18b1e0104
check "$Q/gjk.cpp"          25f56c142bd0854fb30fd5811bc5ea6e74ee8657bd686c2a713c2fde97fd0952

# stdafx.h:24-97   quatFromRot, errFromRot, rotFromQuat, skewSymmetric, hypot
sed -n '24,97p'    "$Q/stdafx.h"          > "$OUT/ref_stdafx_helpers.inc"
# LQRO:32-70       world/quadrotor constants and weight matrices (globals)
sed -n '32,70p'    "$Q/LQRObstacles.cpp"  > "$OUT/ref_globals.inc"
# LQRO:169-189     setup(): physical constants (Callisto part excluded)
sed -n '169,189p'  "$Q/LQRObstacles.cpp"  > "$OUT/ref_setup_body.inc"
# LQRO:1275-1286   _tmain: Qx, Qv, Qp, R, M, N
sed -n '1275,1286p' "$Q/LQRObstacles.cpp" > "$OUT/ref_weights_body.inc"
# LQRO:367-472     f, h, Jacobians, linearizeDiscretize
sed -n '367,472p'  "$Q/LQRObstacles.cpp"  > "$OUT/ref_model.inc"
# LQRO:487-1234    kalman filters, controlMatrices, controllers, GJK glue,
#                  findFG .. calculateNewV (propagate, LQRO:473-486, is left
#                  out: it needs the RNG, which is not on the path)
sed -n '487,1234p' "$Q/LQRObstacles.cpp"  > "$OUT/ref_path.inc"
echo "extracted reference ranges into $OUT"
