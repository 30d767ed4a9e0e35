#!/usr/bin/env python3
"""Golden fixture for the reference's pseudoInverse (include/matrix.h:450-477,
over jacobi2 :887-1037), the kernel of l in controlMatrices (LQRO:552).
TEST INFRASTRUCTURE, build container: oracle/_ref/libref.so ref_pinv16 on
seeded 16 x 16 matrices (full rank, rank deficient, symmetric, and the
controlMatrices matrix ~A - ~A*S*B*!(R+~B*S*B)*~B - I of the reference's own
model, which has eigenvalues at 0).  Writes tests/golden/pinv.npz.
"""
import ctypes as C
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path[:0] = [os.path.join(ROOT, "oracle")]
import pyoracle  # noqa: E402


def main():
    r = pyoracle.reflib()
    assert r is not None, "needs oracle/_ref/libref.so"
    rng = np.random.default_rng(552)
    ms = [rng.standard_normal((16, 16)),
          rng.standard_normal((16, 4)) @ rng.standard_normal((4, 16)),     # rank 4
          (lambda a: a + a.T)(rng.standard_normal((16, 16))),
          np.diag(np.r_[np.ones(12), np.zeros(4)]) + 1e-3 * rng.standard_normal((16, 16))]
    g = pyoracle.synthesize()
    A, B = g["A"], g["B"]
    # S of the velocity LQR is not an output; the matrix is rebuilt with L:
    # ~A - ~A*S*B*!(R+~B*S*B)*~B = ~A + ~L*~B... is not exact, so use ~(A + B L) - I
    ms.append((A + B @ g["L"]).T - np.eye(16))
    ins = np.array([np.ascontiguousarray(m, np.float64) for m in ms])
    outs = np.zeros_like(ins)
    for k in range(len(ins)):
        r.ref_pinv16(ins[k].ctypes.data_as(C.c_void_p), outs[k].ctypes.data_as(C.c_void_p))
    np.savez_compressed(os.path.join(HERE, "pinv.npz"), inputs=ins, outputs=outs)
    print(f"{len(ins)} matrices")


if __name__ == "__main__":
    main()
