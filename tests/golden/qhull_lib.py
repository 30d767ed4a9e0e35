"""Live Qhull (scipy's bundled qhull_r 2019.1) driven like qconvex.exe.
TEST INFRASTRUCTURE, build container only.

The reference's convexHull (LQRObstacles.cpp:867-880) runs
    qconvex n  TO "Planes.txt"        < pointList.txt
    qconvex Fv TO "facetVertices.txt" < pointList.txt
on the reachable points printed at 6 significant digits.  qconvex.exe is a
Win32 binary and is never run.  SURVEY.md §8c names scipy's bundled Qhull as
its stand-in: it reproduces the reference's own fixture (tests/golden/qhull)
facet for facet.  scipy's Python API only exposes the triangulated ('Qt')
hull, so this module calls the library's own entry points the way qconvex's
main does: qh_zero, qh_new_qhull(qh, 3, n, points, 0, "qhull <opts>", out,
err), qh_freeqhull, qh_memfreeshort.  The functions are local symbols of
scipy's extension module; their addresses are its load base (from
/proc/self/maps) plus the values `nm` lists.  With "n" / "Fv" the output is
exactly what qconvex prints for those options (qconvex_r.c: no other
defaults for 3-d input); with "T4" etc. the error stream carries Qhull's
build trace.

Nothing under lqr-obstacles_amd/ or bench.py imports this.
"""
import ctypes
import os
import subprocess
import tempfile

import numpy as np

_LIB = None


def _lib():
    global _LIB
    if _LIB is not None:
        return _LIB
    import scipy.spatial._qhull as mod
    path = os.path.realpath(mod.__file__)
    base = None
    with open("/proc/self/maps") as fh:
        for line in fh:
            parts = line.split()
            if len(parts) >= 6 and os.path.realpath(parts[5]) == path and int(parts[2], 16) == 0:
                base = int(parts[0].split("-")[0], 16)
                break
    if base is None:
        raise RuntimeError("scipy qhull module not mapped")
    syms = {}
    out = subprocess.run(["nm", path], capture_output=True, text=True, check=True).stdout
    for line in out.splitlines():
        p = line.split()
        if len(p) == 3 and p[2] in ("qh_new_qhull", "qh_zero", "qh_freeqhull", "qh_memfreeshort"):
            syms[p[2]] = base + int(p[0], 16)
    if len(syms) != 4:
        raise RuntimeError(f"qhull symbols not found: {sorted(syms)}")
    vp, ci = ctypes.c_void_p, ctypes.c_int
    libc = ctypes.CDLL(None)
    libc.fopen.restype = vp
    libc.fopen.argtypes = [ctypes.c_char_p, ctypes.c_char_p]
    libc.fclose.argtypes = [vp]
    libc.fflush.argtypes = [vp]
    _LIB = dict(
        new=ctypes.CFUNCTYPE(ci, vp, ci, ci, vp, ci, ctypes.c_char_p, vp, vp)(syms["qh_new_qhull"]),
        zero=ctypes.CFUNCTYPE(None, vp, vp)(syms["qh_zero"]),
        free=ctypes.CFUNCTYPE(None, vp, ci)(syms["qh_freeqhull"]),
        memfree=ctypes.CFUNCTYPE(None, vp, ctypes.POINTER(ci), ctypes.POINTER(ci))(syms["qh_memfreeshort"]),
        libc=libc,
    )
    return _LIB


def run(points, opts="n", want_err=False):
    """Run Qhull on `points` (n x 3 float64) with "qhull <opts>"; return the
    output text (and the error/trace text if want_err)."""
    L = _lib()
    pts = np.ascontiguousarray(points, dtype=np.float64)
    qh = ctypes.create_string_buffer(1 << 20)       # qhT is ~20 KB
    with tempfile.TemporaryDirectory() as td:
        fo, fe = os.path.join(td, "out"), os.path.join(td, "err")
        out = L["libc"].fopen(fo.encode(), b"w")
        err = L["libc"].fopen(fe.encode(), b"w")
        L["zero"](ctypes.addressof(qh), err)
        code = L["new"](ctypes.addressof(qh), 3, pts.shape[0], pts.ctypes.data, 0,
                        ("qhull " + opts).encode(), out, err)
        L["free"](ctypes.addressof(qh), 0)
        a, b = ctypes.c_int(), ctypes.c_int()
        L["memfree"](ctypes.addressof(qh), ctypes.byref(a), ctypes.byref(b))
        L["libc"].fclose(out)
        L["libc"].fclose(err)
        with open(fo) as fh:
            otext = fh.read()
        with open(fe) as fh:
            etext = fh.read()
    if code != 0:
        raise RuntimeError(f"qhull exit {code}: {etext[-2000:]}")
    return (otext, etext) if want_err else otext


def qconvex(points):
    """The two files the reference reads: (planes F x 4 as printed and read
    back by >>, facet vertex lists as printed by Fv)."""
    ntext = run(points, "n")
    vtext = run(points, "Fv")
    nt = ntext.split()
    dim, nf = int(nt[0]), int(nt[1])
    planes = np.array([float(t) for t in nt[2:2 + dim * nf]]).reshape(nf, dim)
    vt = vtext.split()
    nf2 = int(vt[0])
    fv, p = [], 1
    for _ in range(nf2):
        k = int(vt[p])
        fv.append([int(t) for t in vt[p + 1:p + 1 + k]])
        p += 1 + k
    assert nf == nf2
    return planes, fv, ntext, vtext


def read_pointlist(path):
    t = open(path).read().split()
    dim, n = int(t[0]), int(t[1])
    return np.array([float(v) for v in t[2:2 + dim * n]]).reshape(n, dim)
