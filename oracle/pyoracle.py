"""pyoracle — ctypes binding of oracle/liboracle.so.  TEST INFRASTRUCTURE ONLY.

The CPU restatement of the reference's per-pair path (see lqro_oracle.h).
Imported only by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline
leg, and only as the checker / the timed CPU baseline.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(HERE, "liboracle.so")
REF_LIB = os.path.join(HERE, "_ref", "libref.so")
REFERENCE = "/root/reference"

_o = None
_r = None


def build(ref: bool = True):
    """Compile liboracle.so (and oracle/_ref/libref.so where /root/reference exists)."""
    subprocess.run(["make", "-s", "-C", HERE, "liboracle.so"], check=True)
    if ref and os.path.isdir(REFERENCE):
        subprocess.run(["make", "-s", "-C", HERE, "ref"], check=True)


def _p(a):
    return a.ctypes.data_as(C.c_void_p)


def lib():
    global _o
    if _o is None:
        if not os.path.exists(LIB):
            build(ref=False)
        _o = C.CDLL(LIB)
        d = C.c_double
        _o.orc_gjk.restype = d
        _o.orc_round6.restype = d
        _o.orc_round6.argtypes = [d]
        _o.orc_pair.argtypes = [C.c_int] * 4 + [d] + [C.c_void_p] * 5 + [C.c_int, C.c_int] + [C.c_void_p] * 3
        _o.orc_step.argtypes = [C.c_int] * 5 + [d, d, C.c_int] + [C.c_void_p] * 5 + [C.c_int, C.c_int, C.c_void_p, C.c_void_p]
        _o.orc_step_mt.argtypes = _o.orc_step.argtypes + [C.c_int]
        _o.orc_step_faithful_mt.argtypes = _o.orc_step_mt.argtypes[:8] + [C.c_void_p] * 2 + \
            _o.orc_step_mt.argtypes[8:]
        _o.orc_newv.argtypes = [C.c_int, C.c_void_p, C.c_void_p, d, C.c_void_p]
        _o.orc_lp_chain.argtypes = [C.c_int, C.c_void_p, C.c_void_p, d]
        _o.orc_lp_chain.restype = C.c_longlong
        _o.orc_sphere.argtypes = [C.c_int, d, d, C.c_void_p]
        _o.orc_pinv.argtypes = [C.c_int, C.c_void_p, C.c_void_p]
        _o.orc_hull_branch.argtypes = [C.c_int, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p]
        _o.orc_hull.argtypes = [C.c_int, C.c_void_p, C.c_void_p, C.c_int]
        _o.orc_agent_step.argtypes = [C.c_void_p] * 17
        _o.orc_jacobi.argtypes = [C.c_int, C.c_void_p, C.c_void_p, C.c_void_p]
        _o.orc_set_neighbors.argtypes = [C.c_double, C.c_int]
        _o.orc_keyframe.argtypes = [C.c_double, C.c_void_p, C.c_void_p, C.c_void_p]
        _o.orc_quat_from_rot.argtypes = [C.c_void_p, C.c_void_p]
        _o.orc_neighbors.argtypes = [C.c_int, C.c_int, C.c_void_p, C.c_int, C.c_double, C.c_int,
                                     C.c_void_p]
    return _o


def reflib():
    """The reference's own functions (oracle/_ref/libref.so) or None."""
    global _r
    if _r is None:
        if not os.path.exists(REF_LIB):
            if not os.path.isdir(REFERENCE):
                return None
            build(ref=True)
        _r = C.CDLL(REF_LIB)
        _r.ref_gjk.restype = C.c_double
    return _r


# record layout == include/lqro.h lqro_pair_record
RECORD_DTYPE = np.dtype([
    ("i", "<i4"), ("j", "<i4"), ("n_reach", "<i4"), ("flags", "<i4"), ("gjk_iters", "<i4"),
    ("simplex_n", "<i4"), ("simplex", "<i4", (4,)), ("facet", "<i4", (3,)),
    ("n_facets", "<i4"), ("reach_hash", "<u8"), ("dist", "<f8"), ("normal", "<f8", (3,)),
    ("wpt_vrel", "<f8", (3,)), ("wpt_hull", "<f8", (3,)), ("plane_point", "<f4", (3,)),
    ("plane_normal", "<f4", (3,)),
])


class Model(C.Structure):
    _fields_ = [(n, C.c_double) for n in (
        "dt", "gravity", "mass", "inertia", "moment_const", "thrust_latency", "length",
        "j_step", "qv", "qp", "r", "pos_weight")]


def synthesize(model: Model | None = None, x_dim: int = 16) -> dict:
    """controlMatrices (LQRO:520-582); x_dim 12 = config 5's reduced model."""
    m = model
    if m is None:
        m = Model()
        lib().orc_model_default(C.byref(m))
    X = x_dim
    out = dict(A=np.zeros((X, X)), B=np.zeros((X, 4)), c=np.zeros(X), L=np.zeros((4, X)),
               E=np.zeros((4, 3)), l=np.zeros(4), Lh=np.zeros((3, X)), Eh=np.zeros((3, 3)))
    rc = lib().orc_synthesize_x(C.byref(m), X, *[_p(out[k]) for k in ("A", "B", "c", "L", "E", "l", "Lh", "Eh")])
    if rc != 0:
        raise ValueError(f"orc_synthesize_x: x_dim {X}")
    return out


def pinv(q: np.ndarray) -> np.ndarray:
    """pseudoInverse (MAT:450-477) of a square matrix."""
    q = np.ascontiguousarray(q, np.float64)
    out = np.zeros_like(q)
    lib().orc_pinv(q.shape[0], _p(q), _p(out))
    return out


def sphere(np_: int = 100, rxy: float = 0.26, rz: float = 0.75) -> np.ndarray:
    s = np.zeros((np_, 3))
    lib().orc_sphere(np_, rxy, rz, _p(s))
    return s


def tables(A, B, L, E, H: int, X: int = 16, U: int = 4):
    T = np.zeros((H, 9))
    N = np.zeros((H, 3, X))
    A, B, L, E = (np.ascontiguousarray(v, dtype=np.float64) for v in (A, B, L, E))
    rc = lib().orc_tables(X, U, H, _p(A), _p(B), _p(L), _p(E), _p(T), _p(N))
    if rc:
        raise RuntimeError(f"orc_tables: {rc}")
    return T, N


def pair(T, NCF, S, xi, xj, i=0, j=1, min_reach=4, vmax_reach=30.0, want_points=False):
    H = T.shape[0]
    NP = S.shape[0]
    X = NCF.shape[-1]
    rec = np.zeros(1, dtype=RECORD_DTYPE)
    idx = np.zeros(H * NP, np.int32)
    pts = np.zeros((H * NP, 3))
    xi = np.ascontiguousarray(xi, np.float64)
    xj = np.ascontiguousarray(xj, np.float64)
    rc = lib().orc_pair(X, H, NP, min_reach, vmax_reach, _p(T), _p(NCF), _p(S), _p(xi), _p(xj),
                        i, j, _p(rec), _p(idx), _p(pts))
    if rc:
        raise RuntimeError(f"orc_pair: {rc}")
    n = int(rec["n_reach"][0])
    if want_points:
        return rec[0], idx[:n].copy(), pts[:n].copy()
    return rec[0]


def step(T, NCF, S, x, vgoal, min_reach=4, vmax_reach=30.0, vmax_lp=100.0, rows=None,
         per_agent=False, threads=1, records=True):
    N, X = x.shape
    H = T.shape[-2]
    NP = S.shape[0]
    r0, r1 = rows if rows is not None else (0, N)
    newv = np.zeros((N, 3))
    recs = np.zeros((r1 - r0) * (N - 1), dtype=RECORD_DTYPE) if records else None
    x = np.ascontiguousarray(x, np.float64)
    vgoal = np.ascontiguousarray(vgoal, np.float64)
    rc = lib().orc_step_mt(N, X, H, NP, min_reach, vmax_reach, vmax_lp, int(per_agent), _p(T),
                           _p(NCF), _p(S), _p(x), _p(vgoal), r0, r1, _p(newv),
                           _p(recs) if recs is not None else None, threads)
    if rc:
        raise RuntimeError(f"orc_step: {rc}")
    return newv, recs


def step_faithful(A, B, L, E, S, x, vgoal, H, min_reach=4, vmax_reach=30.0, vmax_lp=100.0, rows=None,
                  per_agent=False, threads=1, records=True):
    """orc_step_faithful_mt: the step with the reference's per-pair cost
    (findFG per pair, LQRO:1401-1406; GJK twice for outside pairs,
    LQRO:1410/1414); results bit-identical to step().  The CPU baseline."""
    N, X = x.shape
    NP = S.shape[0]
    r0, r1 = rows if rows is not None else (0, N)
    newv = np.zeros((N, 3))
    recs = np.zeros((r1 - r0) * (N - 1), dtype=RECORD_DTYPE) if records else None
    A, B, L, E, x, vgoal = (np.ascontiguousarray(v, np.float64) for v in (A, B, L, E, x, vgoal))
    rc = lib().orc_step_faithful_mt(N, X, H, NP, min_reach, vmax_reach, vmax_lp, int(per_agent),
                                    _p(A), _p(B), _p(L), _p(E), _p(S), _p(x), _p(vgoal), r0, r1,
                                    _p(newv), _p(recs) if recs is not None else None, threads)
    if rc:
        raise RuntimeError(f"orc_step_faithful: {rc}")
    return newv, recs


def newv(planes6: np.ndarray, vgoal, vmax_lp=100.0):
    planes6 = np.ascontiguousarray(planes6, np.float32).reshape(-1, 6)
    v = np.ascontiguousarray(vgoal, np.float64)
    out = np.zeros(3)
    lib().orc_newv(planes6.shape[0], _p(planes6), _p(v), vmax_lp, _p(out))
    return out


def lp_chain(planes6: np.ndarray, vgoal, vmax_lp=100.0) -> int:
    """linearProgram4's sequential chain length for one plane list (0: no LP4)."""
    planes6 = np.ascontiguousarray(planes6, np.float32).reshape(-1, 6)
    v = np.ascontiguousarray(vgoal, np.float64)
    return int(lib().orc_lp_chain(planes6.shape[0], _p(planes6), _p(v), vmax_lp))


def round6(v: float) -> float:
    return lib().orc_round6(float(v))


def hull(points: np.ndarray) -> np.ndarray:
    points = np.ascontiguousarray(points, np.float64)
    n = points.shape[0]
    cap = 4 * n + 16
    f = np.zeros((cap, 3), np.int32)
    k = lib().orc_hull(n, _p(points), _p(f), cap)
    if k < 0:
        raise RuntimeError(f"orc_hull: {k}")
    return f[:k].copy()


def hull_branch(points_full: np.ndarray, vrel):
    points_full = np.ascontiguousarray(points_full, np.float64)
    v = np.ascontiguousarray(vrel, np.float64)
    d = np.zeros(1)
    nrm = np.zeros(3)
    fac = np.zeros(3, np.int32)
    k = lib().orc_hull_branch(points_full.shape[0], _p(points_full), _p(v), _p(d), _p(nrm), _p(fac))
    return k, float(d[0]), nrm, fac


def agent_step(st: dict, gains: dict, nrm, models=None, M=None, N=None,
               per_agent: bool = False):
    """orc_agent_step for every agent of st (same dict layout as
    lqro.agent_states), in place; returns u (n x 4).  models: None (the
    default model), or a list of 1 or n models with the lqro_model fields."""
    if models is None:
        m0 = Model()
        lib().orc_model_default(C.byref(m0))
        models = [m0]
    models = [Model(*[getattr(m, f) for f, _ in Model._fields_]) for m in models]
    M = np.ascontiguousarray(1e-9 * np.eye(16) if M is None else M, np.float64)
    N = np.ascontiguousarray(1e-9 * np.eye(6) if N is None else N, np.float64)
    n = st["x"].shape[0]
    nrm = np.ascontiguousarray(nrm, np.float64).reshape(n, 22)
    u = np.zeros((n, 4))
    for a in range(n):
        g = {k: np.ascontiguousarray(gains[k][a] if per_agent else gains[k], np.float64)
             for k in ("L", "E", "l", "Lh", "Eh")}
        row = {k: np.ascontiguousarray(st[k][a]) for k in st}
        m = models[a if len(models) > 1 else 0]
        lib().orc_agent_step(C.byref(m), _p(g["L"]), _p(g["E"]), _p(g["l"]), _p(g["Lh"]),
                             _p(g["Eh"]), _p(row["u_goal"]), _p(row["p_goal"]), _p(M), _p(N),
                             _p(nrm[a]), _p(row["x"]), _p(row["rot"]), _p(row["x_true"]),
                             _p(row["rot_true"]), _p(row["P"]), _p(row["vgoal"]), _p(u[a]))
        for k in ("x", "rot", "x_true", "rot_true", "P", "vgoal"):
            st[k][a] = row[k]
    return u


def jacobi(m):
    m = np.ascontiguousarray(m, np.float64)
    n = m.shape[0]
    V = np.zeros((n, n))
    D = np.zeros((n, n))
    lib().orc_jacobi(n, _p(m), _p(V), _p(D))
    return V, D


def set_neighbors(nbr_dist: float, max_nbr: int):
    """Neighbour culling for step() (0 = all pairs; process-wide)."""
    lib().orc_set_neighbors(float(nbr_dist), int(max_nbr))


def neighbors(x, i: int, nbr_dist: float, max_nbr: int) -> np.ndarray:
    x = np.ascontiguousarray(x, np.float64)
    sel = np.zeros(x.shape[0], np.uint8)
    lib().orc_neighbors(x.shape[0], x.shape[1], _p(x), i, nbr_dist * nbr_dist, max_nbr, _p(sel))
    return sel


def keyframes(t: float, x_true, rot_true) -> np.ndarray:
    """orc_keyframe per agent: n x 8 float32 (time, position, quaternion)."""
    x_true = np.ascontiguousarray(x_true, np.float64)
    rot_true = np.ascontiguousarray(rot_true, np.float64)
    n = x_true.shape[0]
    out = np.zeros((n, 8), np.float32)
    for a in range(n):
        lib().orc_keyframe(float(t), _p(x_true[a]), _p(rot_true[a]), _p(out[a]))
    return out


class _QhullOut(C.Structure):
    _fields_ = [("nfacets", C.c_int), ("nvertices", C.c_int), ("fv", C.POINTER(C.c_int)),
                ("plane", C.POINTER(C.c_double)), ("facet_id", C.POINTER(C.c_int)),
                ("status", C.c_int)] + [(k, C.c_int) for k in (
                    "st_addpoints", "st_partition", "st_horizon_max", "st_horizon_sum", "st_cop_max",
                    "st_old_append", "st_visible_max", "st_new_max", "st_partition_max", "st_facets_created")] + [
                ("distround", C.c_double)]


def qhull(points: np.ndarray, keep_going: bool = False):
    """orc_qhull: Qhull 2019.1's build restated (lqro_qhull.c) on n x 3
    points.  Returns (status, fv (F x 3, Fv order), planes (F x 4), facet ids);
    status != 0 means the hull needs Qhull's merging (not restated)."""
    o = lib()
    if not getattr(o, "_qh_init", False):
        o.orc_qhull.argtypes = [C.c_void_p, C.c_int, C.c_void_p]
        o.orc_qhull_ex.argtypes = [C.c_void_p, C.c_int, C.c_void_p, C.c_int]
        o.orc_qhull_free.argtypes = [C.c_void_p]
        o._qh_init = True
    points = np.ascontiguousarray(points, np.float64)
    out = _QhullOut()
    o.orc_qhull_ex(_p(points), points.shape[0], C.byref(out), int(keep_going))
    nf = out.nfacets
    if (out.status and not keep_going) or nf <= 0:
        st = out.status
        o.orc_qhull_free(C.byref(out))
        return st, None, None, None
    fv = np.ctypeslib.as_array(out.fv, shape=(nf, 3)).copy()
    pl = np.ctypeslib.as_array(out.plane, shape=(nf, 4)).copy()
    fid = np.ctypeslib.as_array(out.facet_id, shape=(nf,)).copy()
    st = out.status
    global last_qhull_stats
    last_qhull_stats = {k: getattr(out, k) for k, _ in _QhullOut._fields_ if k.startswith("st_")}
    o.orc_qhull_free(C.byref(out))
    return st, fv, pl, fid


def set_hull_rule(rule: int, round16: bool = True):
    """0: the canonical rule (default); 1: the reference's rule over Qhull's
    order (orc_hull_branch_ref), loop-carried normal resolved in row order.
    round16: planes read back as qconvex prints them (%.16g, LQRO:889-899:
    the reference's own rule and the GPU's, lqro_dec16.hpp; False keeps
    Qhull's doubles, for diagnostics).  Process-wide."""
    o = lib()
    o.orc_set_hull_rule.argtypes = [C.c_int, C.c_int]
    o.orc_set_hull_rule(int(rule), int(round16))


def carry_normal(n=None):
    """Get (n=None) or set the loop-carried normalVector entering the next step."""
    o = lib()
    o.orc_get_carry_normal.argtypes = [C.c_void_p]
    o.orc_set_carry_normal.argtypes = [C.c_void_p]
    if n is None:
        out = np.zeros(3)
        o.orc_get_carry_normal(_p(out))
        return out
    v = np.ascontiguousarray(n, np.float64)
    o.orc_set_carry_normal(_p(v))


def hull_branch_ref(points_full: np.ndarray, vrel):
    """orc_hull_branch_ref: (nfacets, dist, normal or None if stale, Fv triple, qstatus)."""
    o = lib()
    o.orc_hull_branch_ref.argtypes = [C.c_int] + [C.c_void_p] * 7
    points_full = np.ascontiguousarray(points_full, np.float64)
    v = np.ascontiguousarray(vrel, np.float64)
    d = np.zeros(1)
    nrm = np.zeros(3)
    fac = np.zeros(3, np.int32)
    st = np.zeros(2, np.int32)
    k = o.orc_hull_branch_ref(points_full.shape[0], _p(points_full), _p(v), _p(d), _p(nrm), _p(fac),
                              _p(st[:1]), _p(st[1:]))
    return k, float(d[0]), (None if st[0] else nrm), fac, int(st[1])


def hull_time(reset: bool = True):
    """(thread-seconds in the hull branch, inside-hull pairs) since the last reset."""
    o = lib()
    o.orc_hull_time.argtypes = [C.c_void_p, C.c_void_p, C.c_int]
    sec = C.c_double()
    cnt = C.c_longlong()
    o.orc_hull_time(C.byref(sec), C.byref(cnt), int(reset))
    return sec.value, cnt.value
