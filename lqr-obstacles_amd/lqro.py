"""lqro — Python host binding of liblqro.so (the MI355X LQR-Obstacle step).

This module mirrors the reference simulator's interface for the pair loop
(hihixuyang/LQR-Obstacles, QuadrotorHoverController/LQRObstacles.cpp, "LQRO"):

  * ``Quadrotor``  — the agent record the loop reads and writes (LQRO:73-165:
    ``x``, ``L``, ``E``, ``vGoal``, ``newV``);
  * ``Simulator.findMatrices()`` — controlMatrices at hover (LQRO:520-582,
    called per agent at LQRO:1370-1373);
  * ``Simulator.step()`` — the pair loop LQRO:1393-1436: every ordered pair's
    LQR-Obstacle, its half-plane, and each agent's new velocity
    (calculateNewV, LQRO:1435), computed by the HIP kernels.

All numerics run in liblqro.so (HIP for gfx950).  There is no CPU fallback:
if the library or a gfx950 device is missing, the calls raise.
"""
from __future__ import annotations

import ctypes as C
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "liblqro.so")

LQRO_OK = 0
LQRO_E_HULL = -8              # an inside-hull pair's hull could not be built (degenerate input or capacity; no half-plane)
LQRO_E_QHMERGE = -9           # the step ran, but a pair's winning facet may be one qconvex's pre-merge joins
LQRO_FLAG_RECORDS = 0x1
LQRO_FLAG_QHULL_ORDER = 0x2   # the reference's own hull rule over Qhull's build order (k_qhull)
REC_PLANE, REC_INSIDE, REC_BACKUP, REC_HULL, REC_HULLFAIL, REC_LOCAL = 0x01, 0x02, 0x04, 0x08, 0x10, 0x20
REC_STALE, REC_QHMERGE = 0x40, 0x80
REC_QHMERGE_WIN = 0x100       # with REC_QHMERGE: qconvex's pre-merge may have merged the winning facet
HULL_BUILD_DTYPE = np.dtype([("i", np.int32), ("j", np.int32), ("n_points", np.int32), ("insertions", np.int32),
                             ("facet_slots", np.int32), ("kernel", np.int32), ("t_start", np.uint64),
                             ("t_end", np.uint64)])


class Config(C.Structure):
    _fields_ = [
        ("n_agents", C.c_int32), ("x_dim", C.c_int32), ("u_dim", C.c_int32),
        ("horizon", C.c_int32), ("n_points", C.c_int32), ("min_reach", C.c_int32),
        ("xy_radius", C.c_double), ("z_radius", C.c_double),
        ("vmax_reach", C.c_double), ("vmax_lp", C.c_double),
        ("row_begin", C.c_int32), ("row_end", C.c_int32),
        ("device", C.c_int32), ("flags", C.c_int32), ("row_stride", C.c_int32),
    ]


class Model(C.Structure):
    _fields_ = [(n, C.c_double) for n in (
        "dt", "gravity", "mass", "inertia", "moment_const", "thrust_latency", "length",
        "j_step", "qv", "qp", "r", "pos_weight")]


class PairRecord(C.Structure):
    _fields_ = [
        ("i", C.c_int32), ("j", C.c_int32), ("n_reach", C.c_int32), ("flags", C.c_int32),
        ("gjk_iters", C.c_int32), ("simplex_n", C.c_int32), ("simplex", C.c_int32 * 4),
        ("facet", C.c_int32 * 3), ("n_facets", C.c_int32), ("reach_hash", C.c_uint64),
        ("dist", C.c_double), ("normal", C.c_double * 3), ("wpt_vrel", C.c_double * 3),
        ("wpt_hull", C.c_double * 3), ("plane_point", C.c_float * 3),
        ("plane_normal", C.c_float * 3),
    ]


RECORD_DTYPE = np.dtype([
    ("i", "<i4"), ("j", "<i4"), ("n_reach", "<i4"), ("flags", "<i4"), ("gjk_iters", "<i4"),
    ("simplex_n", "<i4"), ("simplex", "<i4", (4,)), ("facet", "<i4", (3,)),
    ("n_facets", "<i4"), ("reach_hash", "<u8"), ("dist", "<f8"), ("normal", "<f8", (3,)),
    ("wpt_vrel", "<f8", (3,)), ("wpt_hull", "<f8", (3,)), ("plane_point", "<f4", (3,)),
    ("plane_normal", "<f4", (3,)),
])
assert RECORD_DTYPE.itemsize == C.sizeof(PairRecord) == 168

# every symbol include/lqro.h declares
EXPORTS = (
    "lqro_config_default", "lqro_model_default", "lqro_synthesize_gains", "lqro_sphere",
    "lqro_create", "lqro_destroy", "lqro_set_gains", "lqro_step", "lqro_step_device",
    "lqro_get_records", "lqro_get_stats", "lqro_get_timings", "lqro_status_string",
    "lqro_version", "lqro_calculate_new_v", "lqro_synthesize_gains_batch",
    "lqro_dynamics_step", "lqro_dynamics_step_device", "lqro_normals", "lqro_set_neighbors",
    "lqro_synthesize_gains_x", "lqro_synthesize_gains_batch_x",
    "lqro_set_carry_normal", "lqro_get_carry_normal",
    "lqro_step_device_begin", "lqro_step_device_end",
    "lqro_get_stats_ex", "lqro_get_hull_failures", "lqro_get_hull_builds", "lqro_get_qhmerge_pairs",
)

NORMALS_PER_AGENT = 22   # LQRO_NORMALS_PER_AGENT: 16 propagate + 6 observation


class Agents(C.Structure):
    """lqro_agents: per-agent state, gains and noise of the step after the
    pair loop (LQRO:1437-1446)."""
    _fields_ = [(n, C.c_void_p) for n in (
        "x", "rot", "x_true", "rot_true", "P", "vgoal", "u", "u_goal", "p_goal",
        "L", "E", "l", "Lh", "Eh", "M", "N", "normals", "keyframes")] + [("time", C.c_double)]

_lib = None


def lib() -> C.CDLL:
    """Load liblqro.so (raises if it was not built: no fallback path)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise RuntimeError(f"liblqro.so not built at {LIB_PATH}; run __graft_entry__.build()")
        L = C.CDLL(LIB_PATH)
        vp, i32, i64, dbl = C.c_void_p, C.c_int32, C.c_int64, C.c_double
        L.lqro_status_string.restype = C.c_char_p
        L.lqro_config_default.argtypes = [C.POINTER(Config), i32, i32, i32]
        L.lqro_model_default.argtypes = [C.POINTER(Model)]
        L.lqro_synthesize_gains.argtypes = [C.POINTER(Model)] + [vp] * 7
        L.lqro_synthesize_gains_batch.argtypes = [C.POINTER(Model), i32] + [vp] * 7 + [i32]
        L.lqro_synthesize_gains_x.argtypes = [C.POINTER(Model), i32] + [vp] * 8
        L.lqro_synthesize_gains_batch_x.argtypes = [C.POINTER(Model), i32, i32] + [vp] * 8 + [i32]
        L.lqro_sphere.argtypes = [i32, dbl, dbl, vp]
        L.lqro_create.argtypes = [C.POINTER(Config), C.POINTER(vp)]
        L.lqro_destroy.argtypes = [vp]
        L.lqro_destroy.restype = None
        L.lqro_set_gains.argtypes = [vp, vp, vp, vp, vp, i32]
        L.lqro_step.argtypes = [vp, vp, vp, vp]
        L.lqro_step_device.argtypes = [vp, vp, vp, vp, vp]
        L.lqro_step_device_begin.argtypes = [vp, vp, vp, vp, vp]
        L.lqro_step_device_end.argtypes = [vp, vp, vp, vp]
        L.lqro_get_records.argtypes = [vp, vp, i64, C.POINTER(i64)]
        L.lqro_get_stats.argtypes = [vp, vp]
        L.lqro_get_stats_ex.argtypes = [vp, vp, i32]
        L.lqro_get_hull_failures.argtypes = [vp, vp, i64, C.POINTER(i64)]
        if hasattr(L, "lqro_get_qhmerge_pairs"):   # (older libraries in A/B runs lack it)
            L.lqro_get_qhmerge_pairs.argtypes = [vp, vp, i64, C.POINTER(i64)]
        L.lqro_get_timings.argtypes = [vp, vp]
        L.lqro_calculate_new_v.argtypes = [vp, vp, i32, vp, dbl, vp, i32]
        L.lqro_dynamics_step.argtypes = [C.POINTER(Model), i32, i32, i32, C.POINTER(Agents), i32]
        L.lqro_dynamics_step_device.argtypes = [vp, i32, i32, i32, C.POINTER(Agents), vp]
        L.lqro_normals.argtypes = [C.POINTER(C.c_uint32), i64, vp]
        L.lqro_set_neighbors.argtypes = [vp, dbl, i32]
        L.lqro_set_carry_normal.argtypes = [vp, vp]
        L.lqro_get_carry_normal.argtypes = [vp, vp]
        _lib = L
    return _lib


class LqroError(RuntimeError):
    pass


class HullFailure(LqroError):
    """lqro_step returned LQRO_E_HULL: inside-hull pairs whose hull could not
    be built (degenerate or too few points, or every hull kernel's capacity
    exceeded) got no half-plane (the reference's qconvex
    always returns a hull, LQRO:879-880).  .pairs: their (i, j); .newv: the
    step's new velocities, computed without those planes."""

    def __init__(self, msg, pairs, newv):
        super().__init__(msg)
        self.pairs, self.newv = pairs, newv


class QhullMergeSuspect(LqroError):
    """lqro_step returned LQRO_E_QHMERGE: the step completed, but for some
    inside-hull pairs the winning facet may be one that qconvex's default
    pre-merge joins into a merged facet (LQRO_REC_QHMERGE_WIN; convexHull
    then measures from the merged facet's first Fv vertex with its merged
    plane, LQRO:925-939, 956-967).  Qhull's merging is not restated, so those
    pairs' half-planes are not pinned to the reference.  .pairs: their (i, j);
    .newv: the step's new velocities."""

    def __init__(self, msg, pairs, newv):
        super().__init__(msg)
        self.pairs, self.newv = pairs, newv


def _check(rc: int, what: str):
    if rc != LQRO_OK:
        msg = lib().lqro_status_string(rc).decode()
        raise LqroError(f"{what}: {msg} ({rc})")


def _p(a: np.ndarray):
    return a.ctypes.data_as(C.c_void_p)


def default_model() -> Model:
    m = Model()
    lib().lqro_model_default(C.byref(m))
    return m


def gain_shapes(x_dim: int = 16) -> dict:
    """controlMatrices' outputs in the reference's argument order (LQRO:520)."""
    X = x_dim
    return dict(A=(X, X), B=(X, 4), c=(X,), L=(4, X), E=(4, 3), l=(4,), Lh=(3, X), Eh=(3, 3))


GAIN_SHAPES = gain_shapes(16)


def synthesize_gains(model: Model | None = None, x_dim: int = 16) -> dict:
    """controlMatrices at hover (LQRO:520-582): A, B, c, L, E, l, Lh, Eh.
    x_dim = 12: BASELINE config 5's reduced model (rotor-force states
    dropped, F = u; lqro_synthesize_gains_x)."""
    m = model or default_model()
    shp = gain_shapes(x_dim)
    out = {k: np.zeros(s) for k, s in shp.items()}
    _check(lib().lqro_synthesize_gains_x(C.byref(m), x_dim, *[_p(out[k]) for k in shp]),
           "lqro_synthesize_gains_x")
    return out


def synthesize_gains_batch(models, device: int = 0, x_dim: int = 16) -> dict:
    """controlMatrices for heterogeneous agents, on the GPU (one agent per
    lane): arrays with a leading agent axis, bit-identical to
    synthesize_gains(models[k], x_dim); L and E feed
    Context.set_gains(per_agent=1)."""
    n = len(models)
    arr = (Model * n)(*models)
    shp = gain_shapes(x_dim)
    out = {k: np.zeros((n,) + s) for k, s in shp.items()}
    _check(lib().lqro_synthesize_gains_batch_x(arr, n, x_dim, *[_p(out[k]) for k in shp], device),
           "lqro_synthesize_gains_batch_x")
    return out


def perturbed_models(n: int, rel: float = 0.01, seed: int | None = None) -> list:
    """n agent models with mass, inertia, arm length, moment constant, thrust
    latency and the cost weights qv, qp, r each scaled by a factor in
    [1 - rel, 1 + rel] (SplitMix64, seeded): the heterogeneous swarm of
    BASELINE config 5."""
    g = _splitmix(SEED_MODELS if seed is None else seed)
    base = default_model()
    out = []
    for _ in range(n):
        m = Model.from_buffer_copy(base)
        for f in ("mass", "inertia", "length", "moment_const", "thrust_latency", "qv", "qp", "r"):
            setattr(m, f, getattr(base, f) * (1.0 + rel * (2.0 * next(g) - 1.0)))
        out.append(m)
    return out


def create_spheres(n_points: int = 100, xy_radius: float = 0.26, z_radius: float = 0.75):
    """createSpheres (LQRO:735-750)."""
    s = np.zeros((n_points, 3))
    _check(lib().lqro_sphere(n_points, xy_radius, z_radius, _p(s)), "lqro_sphere")
    return s


def config(n_agents: int, horizon: int, n_points: int = 100, **kw) -> Config:
    c = Config()
    lib().lqro_config_default(C.byref(c), n_agents, horizon, n_points)
    for k, v in kw.items():
        setattr(c, k, v)
    return c


class Context:
    """One liblqro context: owns device buffers and a HIP stream."""

    def __init__(self, cfg: Config):
        self.cfg = cfg
        h = C.c_void_p()
        _check(lib().lqro_create(C.byref(cfg), C.byref(h)), "lqro_create")
        self._h = h
        rb, re = cfg.row_begin, cfg.row_end
        if rb == 0 and re == 0:
            re = cfg.n_agents
        self.rows = (rb, re)
        self.row_ids = np.arange(rb, re, max(cfg.row_stride, 1))   # the agents whose rows this computes

    def close(self):
        if self._h:
            lib().lqro_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def set_neighbors(self, neighbor_dist: float, max_neighbors: int):
        """Opt-in neighbour culling (lqro_set_neighbors; RVO2 computeNeighbors,
        AGT:74-81,153-174).  Changes results; max_neighbors <= 0 = all pairs."""
        _check(lib().lqro_set_neighbors(self._h, float(neighbor_dist), int(max_neighbors)),
               "lqro_set_neighbors")

    def set_gains(self, A, B, L, E, per_agent: bool = False):
        A, B, L, E = (np.ascontiguousarray(v, dtype=np.float64) for v in (A, B, L, E))
        X, U, n = self.cfg.x_dim, self.cfg.u_dim, self.cfg.n_agents
        lead = (n,) if per_agent else ()
        for name, v, shp in (("A", A, (X, X)), ("B", B, (X, U)), ("L", L, lead + (U, X)),
                             ("E", E, lead + (U, 3))):
            if v.shape != shp and not (per_agent is False and v.shape == (1,) + shp):
                raise LqroError(f"set_gains: {name} has shape {v.shape}, expected {shp}")
        _check(lib().lqro_set_gains(self._h, _p(A), _p(B), _p(L), _p(E), int(per_agent)),
               "lqro_set_gains")

    def step(self, x: np.ndarray, vgoal: np.ndarray) -> np.ndarray:
        x = np.ascontiguousarray(x, dtype=np.float64)
        vgoal = np.ascontiguousarray(vgoal, dtype=np.float64)
        n = self.cfg.n_agents
        if x.shape != (n, self.cfg.x_dim):
            raise LqroError(f"step: x has shape {x.shape}, expected {(n, self.cfg.x_dim)}")
        if vgoal.shape != (n, 3):
            raise LqroError(f"step: vgoal has shape {vgoal.shape}, expected {(n, 3)}")
        newv = np.zeros((self.cfg.n_agents, 3))
        rc = lib().lqro_step(self._h, _p(x), _p(vgoal), _p(newv))
        if rc == LQRO_E_HULL:
            pairs = self.hull_failures()
            raise HullFailure(f"lqro_step: {len(pairs)} inside-hull pair(s) without a half-plane: "
                              f"{[tuple(p) for p in pairs[:8]]}", pairs, newv)
        if rc == LQRO_E_QHMERGE:
            pairs = self.qhmerge_pairs()
            raise QhullMergeSuspect(f"lqro_step: {len(pairs)} inside-hull pair(s) whose winning facet qconvex may "
                                    f"merge: {[tuple(p) for p in pairs[:8]]}", pairs, newv)
        _check(rc, "lqro_step")
        return newv

    def hull_failures(self) -> np.ndarray:
        """(i, j) of the last step's pairs left without a half-plane (at most 64)."""
        out = np.zeros((64, 2), np.int64)
        n = C.c_int64()
        _check(lib().lqro_get_hull_failures(self._h, _p(out), 64, C.byref(n)), "lqro_get_hull_failures")
        return out[:min(n.value, 64)]

    def qhmerge_pairs(self) -> np.ndarray:
        """(i, j) of the last step's LQRO_REC_QHMERGE_WIN pairs (at most 64)."""
        out = np.zeros((64, 2), np.int64)
        n = C.c_int64()
        _check(lib().lqro_get_qhmerge_pairs(self._h, _p(out), 64, C.byref(n)), "lqro_get_qhmerge_pairs")
        return out[:min(n.value, 64)]

    def step_device(self, d_x: int, d_vgoal: int, d_newv: int, stream: int = 0):
        """Device pointers (e.g. torch tensor .data_ptr()) on the context's
        device, enqueued on `stream` (a hipStream_t handle such as
        torch.cuda.current_stream().cuda_stream; 0 = the null stream, which is
        torch's default stream), so it is ordered with the caller's work."""
        _check(lib().lqro_step_device(self._h, C.c_void_p(d_x), C.c_void_p(d_vgoal),
                                      C.c_void_p(d_newv), C.c_void_p(stream or None)),
               "lqro_step_device")

    def step_device_begin(self, d_x: int, d_vgoal: int, d_rowtab: int, stream: int = 0):
        """The first half of step_device for row shards in Qhull order: sweep
        and hulls; this context's rows of the (N, 4) row-normal table
        d_rowtab are written (lqro_step_device_begin)."""
        _check(lib().lqro_step_device_begin(self._h, C.c_void_p(d_x), C.c_void_p(d_vgoal),
                                            C.c_void_p(d_rowtab), C.c_void_p(stream or None)),
               "lqro_step_device_begin")

    def step_device_end(self, d_rowtab: int, d_newv: int, stream: int = 0):
        """The second half, once every rank's rows of d_rowtab are present:
        the facet-0 pairs' loop-carried normals, then the LP."""
        _check(lib().lqro_step_device_end(self._h, C.c_void_p(d_rowtab), C.c_void_p(d_newv),
                                          C.c_void_p(stream or None)), "lqro_step_device_end")

    def records(self) -> np.ndarray:
        n = len(self.row_ids) * (self.cfg.n_agents - 1)
        out = np.zeros(n, dtype=RECORD_DTYPE)
        got = C.c_int64()
        _check(lib().lqro_get_records(self._h, _p(out), n, C.byref(got)), "lqro_get_records")
        return out[:got.value]   # rows x K with neighbour culling on

    def stats(self) -> dict:
        s = np.zeros(12, dtype=np.int64)
        _check(lib().lqro_get_stats_ex(self._h, _p(s), 12), "lqro_get_stats_ex")
        keys = ("pairs", "planes", "inside", "hull_ok", "hull_fail", "gjk_backups",
                "sum_n_reach", "sum_gtests", "qhull_merged", "qhull_retried", "qhull_timeouts",
                "qhull_merge_win")
        return dict(zip(keys, (int(v) for v in s)))

    def hull_builds(self) -> np.ndarray:
        """LQRO_FLAG_QHULL_ORDER: the last step's hull builds (lqro_get_hull_builds):
        i, j, n_points, insertions, facet_slots, kernel (0 k_qhull, 1 k_qhull_big,
        2 a k_qhull build handed over), t_start / t_end in 100 MHz ticks."""
        out = np.zeros(16384, dtype=HULL_BUILD_DTYPE)
        n = C.c_int64()
        _check(lib().lqro_get_hull_builds(self._h, _p(out), len(out), C.byref(n)), "lqro_get_hull_builds")
        return out[:min(n.value, len(out))]

    def carry_normal(self, n=None):
        """LQRO_FLAG_QHULL_ORDER: get (n=None) the loop-carried normalVector
        (LQRO:1385) the last step left, or set the one entering the next."""
        if n is None:
            out = np.zeros(3)
            _check(lib().lqro_get_carry_normal(self._h, _p(out)), "lqro_get_carry_normal")
            return out
        v = np.ascontiguousarray(n, dtype=np.float64)
        _check(lib().lqro_set_carry_normal(self._h, _p(v)), "lqro_set_carry_normal")

    def debug_qhull(self, rounded: np.ndarray, full: np.ndarray, vrel, max_facets: int = 0):
        """Test hook: k_qhull on given points (rounded = qconvex's input, full =
        the distances' points): (record, build status bits[, facet list in
        Qhull's order, Fv triples, when max_facets > 0]).  self.debug_status:
        the hook's C-ABI status, LQRO_E_QHMERGE for a merge-suspect winner
        (lqro_step's rule)."""
        n = rounded.shape[0]
        pts = np.ascontiguousarray(np.concatenate([rounded.reshape(-1), full.reshape(-1)]), dtype=np.float64)
        v = np.ascontiguousarray(vrel, dtype=np.float64)
        rec = PairRecord()
        nf = C.c_int32()
        fn = lib().lqro_debug_hull_points
        fn.argtypes = [C.c_void_p, C.c_void_p, C.c_int32, C.c_void_p, C.c_int32, C.c_void_p, C.c_int32,
                       C.POINTER(C.c_int32), C.POINTER(PairRecord)]
        fl = np.zeros((max(max_facets, 1), 3), np.int32)
        rc = fn(self._h, _p(pts), n, _p(v), 2, _p(fl) if max_facets else None, max_facets, C.byref(nf),
                C.byref(rec))
        self.debug_status = rc
        if rc != LQRO_E_QHMERGE:
            _check(rc, "lqro_debug_hull_points")
        r = np.frombuffer(bytes(rec), dtype=RECORD_DTYPE)[0]
        if max_facets:
            end = np.nonzero(fl[:, 0] < 0)[0]
            return r, int(nf.value), fl[: end[0] if len(end) else max_facets]
        return r, int(nf.value)

    def timings(self) -> dict:
        t = np.zeros(4, dtype=np.float32)
        _check(lib().lqro_get_timings(self._h, _p(t)), "lqro_get_timings")
        return dict(pair_ms=float(t[0]), hull_ms=float(t[1]), lp_ms=float(t[2]),
                    step_ms=float(t[3]))


def calculate_new_v(plane_lists, vgoals, vmax_lp: float = 100.0, device: int = 0) -> np.ndarray:
    """calculateNewV (LQRO:1223-1234) for many agents at once on the GPU.
    plane_lists: sequence of (m_r, 6) float32 arrays (point, normal) in push
    order; vgoals: (n, 3)."""
    n = len(plane_lists)
    offs = np.zeros(n + 1, dtype=np.int64)
    for r, p in enumerate(plane_lists):
        offs[r + 1] = offs[r] + len(p)
    flat = np.zeros((max(int(offs[-1]), 1), 6), dtype=np.float32)
    for r, p in enumerate(plane_lists):
        if len(p):
            flat[offs[r]:offs[r + 1]] = np.asarray(p, dtype=np.float32).reshape(-1, 6)
    vg = np.ascontiguousarray(vgoals, dtype=np.float64).reshape(n, 3)
    out = np.zeros((n, 3))
    _check(lib().lqro_calculate_new_v(_p(flat), _p(offs), n, _p(vg), vmax_lp, _p(out), device),
           "lqro_calculate_new_v")
    return out


# ---------------------------------------------------------------------------
# Synthetic swarms: SplitMix64, seed "LQRO"
# ---------------------------------------------------------------------------
SEED = 0x4C51524F
SEED_MODELS = 0x4D4F444C   # "MODL"
_M64 = 0xFFFFFFFFFFFFFFFF


def _splitmix(seed: int):
    s = seed & _M64
    while True:
        s = (s + 0x9E3779B97F4A7C15) & _M64
        z = s
        z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & _M64
        z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & _M64
        yield ((z ^ (z >> 31)) >> 11) * 2.0 ** -53


def synthetic_swarm(n: int, x_dim: int = 16, seed: int = SEED, box: float | None = None):
    """N agents at constant density: position U[-L/2,L/2]^3 with L = 4 N^(1/3),
    velocity U[-1,1]^3, hover attitude, rotor forces at nominalInput
    (LQRO:188); vGoal U[-1,1]^3.  Draw order per agent: 3 position, 3
    velocity, 3 vGoal."""
    g = _splitmix(seed)
    side = box if box is not None else 4.0 * n ** (1.0 / 3.0)
    nominal = 9.80665 * 0.500 / 4
    x = np.zeros((n, x_dim))
    vg = np.zeros((n, 3))
    for i in range(n):
        for k in range(3):
            x[i, k] = (next(g) - 0.5) * side
        for k in range(3):
            x[i, 3 + k] = 2.0 * next(g) - 1.0
        if x_dim == 16:
            x[i, 12:16] = nominal
        for k in range(3):
            vg[i, k] = 2.0 * next(g) - 1.0
    return x, vg


def swap_scenario():
    """The scripted 4-quad swap of LQRO:1308-1331 at its first step: states
    (x = xInit, hover forces) and the position goals."""
    nominal = 9.80665 * 0.500 / 4
    pos = [(4.0, 0.0, 2.0), (-4.0, -0.0, 2.0), (0.0, 4.0, 2.0), (0.0, -4.0, 2.0)]
    goal = [(-4.0, 0.0, 2.0), (4.0, 0.0, 2.0), (0.0, -4.0, 2.0), (0.0, 4.0, 2.0)]
    x = np.zeros((4, 16))
    for i, p in enumerate(pos):
        x[i, :3] = p
        x[i, 12:16] = nominal
    return x, np.array(goal)


# ---------------------------------------------------------------------------
# The per-agent step after the pair loop (LQRO:1437-1446), SURVEY §8f next #1
# ---------------------------------------------------------------------------
AGENT_FIELDS = dict(x=(16,), rot=(3, 3), x_true=(16,), rot_true=(3, 3), P=(16, 16), vgoal=(3,),
                    u_goal=(4,), p_goal=(3,))


def normals(seed: int, count: int) -> tuple[np.ndarray, int]:
    """`count` draws of the reference's normal() (LQRO:340-350) on the MSVC
    rand() stream seeded with `seed` (srand); returns (draws, next seed)."""
    st = C.c_uint32(seed & 0xFFFFFFFF)
    out = np.zeros(count)
    _check(lib().lqro_normals(C.byref(st), count, _p(out)), "lqro_normals")
    return out, int(st.value)


def agent_states(x, u_goal=None, p_goal=None, p0: float = 1e-9) -> dict:
    """Host-side agent records for dynamics_step: the estimate x, Rot = I,
    xTrue = x, RotTrue = I, P = p0 I (Pinit, LQRO:1297), vGoal = 0, uGoal =
    hover thrust, pGoal = 0 (setupQuadrotors, LQRO:107-122, without its
    initial noise draw)."""
    x = np.ascontiguousarray(x, dtype=np.float64)
    n = x.shape[0]
    hover = default_model().gravity * default_model().mass / 4
    st = dict(x=x.copy(), rot=np.tile(np.eye(3), (n, 1, 1)), x_true=x.copy(),
              rot_true=np.tile(np.eye(3), (n, 1, 1)), P=np.tile(p0 * np.eye(16), (n, 1, 1)),
              vgoal=np.zeros((n, 3)),
              u_goal=np.full((n, 4), hover) if u_goal is None else np.array(u_goal, dtype=np.float64),
              p_goal=np.zeros((n, 3)) if p_goal is None else np.array(p_goal, dtype=np.float64))
    return st


def dynamics_step(st: dict, gains: dict, nrm: np.ndarray, models=None, M=None, N=None,
                  per_agent: bool = False, device: int = 0, keyframes: np.ndarray | None = None,
                  time: float = 0.0) -> np.ndarray:
    """lqro_dynamics_step: advances every agent of `st` in place (x, rot,
    x_true, rot_true, P; vgoal in = newV, out = findVGoal()) and returns u.
    keyframes: optional n x 8 float32 array that receives visualize's
    keyframe (time, xTrue position, quatFromRot(RotTrue)) at `time`.
    gains: L, E, l, Lh, Eh (one set, or a leading agent axis with
    per_agent=True).  nrm: n x 22 draws.  M, N default to the reference's
    1e-9 I (LQRO:1285-1286)."""
    n = st["x"].shape[0]
    models = [default_model()] if models is None else list(models)
    marr = (Model * len(models))(*models)
    M = 1e-9 * np.eye(16) if M is None else M
    N = 1e-9 * np.eye(6) if N is None else N
    for k, shp in AGENT_FIELDS.items():
        if st[k].shape != (n,) + shp or st[k].dtype != np.float64 or not st[k].flags.c_contiguous:
            raise LqroError(f"dynamics_step: {k} must be C-contiguous float64 {(n,) + shp}")
    keep = [np.ascontiguousarray(v, dtype=np.float64) for v in
            (gains["L"], gains["E"], gains["l"], gains["Lh"], gains["Eh"], M, N, nrm)]
    if keep[-1].size != n * NORMALS_PER_AGENT:
        raise LqroError("dynamics_step: need n x 22 normals")
    u = np.zeros((n, 4))
    a = Agents(*[_p(st[k]).value for k in ("x", "rot", "x_true", "rot_true", "P", "vgoal")],
               _p(u).value, _p(st["u_goal"]).value, _p(st["p_goal"]).value,
               *[_p(v).value for v in keep])
    if keyframes is not None:
        if keyframes.shape != (n, 8) or keyframes.dtype != np.float32 or not keyframes.flags.c_contiguous:
            raise LqroError("dynamics_step: keyframes must be C-contiguous float32 (n, 8)")
        a.keyframes = _p(keyframes).value
    a.time = float(time)
    _check(lib().lqro_dynamics_step(marr, len(models), n, int(per_agent), C.byref(a), device),
           "lqro_dynamics_step")
    return u


# ---------------------------------------------------------------------------
# Reference-shaped interface
# ---------------------------------------------------------------------------
class Quadrotor:
    """The fields of class Quadrotor (LQRO:73-165) that the pair loop and the
    agent update (LQRO:1437-1446) use."""

    def __init__(self, x, vGoal=None, pGoal=None):
        self.x = np.asarray(x, dtype=np.float64).copy()
        self.vGoal = np.zeros(3) if vGoal is None else np.asarray(vGoal, dtype=np.float64).copy()
        self.newV = np.zeros(3)
        self.pGoal = np.zeros(3) if pGoal is None else np.asarray(pGoal, dtype=np.float64).copy()
        self.L = None
        self.E = None
        self.l = np.zeros(4)   # feedforward (LQRO:557), set by findMatrices; the pair path never reads it
        self.Lh = None
        self.Eh = None
        # estimation state (setupQuadrotors, LQRO:107-122, without its noise draw)
        self.Rot = np.eye(3)
        self.xTrue = self.x.copy()
        self.RotTrue = np.eye(3)
        self.P = 1e-9 * np.eye(16)


class Simulator:
    """The per-step driver of LQRO:1391-1436 on the GPU: ``findMatrices``
    once, then ``step()`` each control step fills every ``Quadrotor.newV``."""

    def __init__(self, qlist, horizon: int = 45, n_points: int = 100, device: int = 0,
                 records: bool = False, model: Model | None = None, hull_rule: str = "reference"):
        self.qlist = list(qlist)
        self.model = model or default_model()
        # hull_rule "reference": the reference's own inside-hull rule (Qhull's
        # order, LQRO:925-968); "canonical": the faster deviating rule
        if hull_rule not in ("reference", "canonical"):
            raise ValueError(f"hull_rule {hull_rule!r}")
        flags = (LQRO_FLAG_RECORDS if records else 0) | (LQRO_FLAG_QHULL_ORDER if hull_rule == "reference" else 0)
        self.device = device
        self.t = 0                 # control steps taken (LQRO:1392)
        self.trajectory = []       # keyframes per step (update())
        self.ctx = Context(config(len(self.qlist), horizon, n_points, device=device,
                                  flags=flags))
        self.A = self.B = self.c = None

    def findMatrices(self):
        g = synthesize_gains(self.model)
        self.A, self.B, self.c = g["A"], g["B"], g["c"]
        for q in self.qlist:
            q.L, q.E, q.l, q.Lh, q.Eh = g["L"], g["E"], g["l"], g["Lh"], g["Eh"]
        Ls = np.stack([q.L for q in self.qlist])
        Es = np.stack([q.E for q in self.qlist])
        per_agent = not all(np.array_equal(Ls[0], l) for l in Ls) or \
            not all(np.array_equal(Es[0], e) for e in Es)
        if per_agent:
            self.ctx.set_gains(self.A, self.B, Ls, Es, per_agent=True)
        else:
            self.ctx.set_gains(self.A, self.B, Ls[0], Es[0])
        return g

    def step(self):
        x = np.stack([q.x for q in self.qlist])
        vg = np.stack([q.vGoal for q in self.qlist])
        newv = self.ctx.step(x, vg)
        for q, v in zip(self.qlist, newv):
            q.newV = v.copy()
        return newv

    def save_trajectory(self, path: str):
        """The keyframes update() recorded (Quadrotor::visualize's Callisto
        keys, LQRO:128-133): an .npz with `keyframes` (steps x agents x 8:
        time, xTrue position, quaternion) for offline diffing/plotting."""
        kf = np.stack(self.trajectory) if self.trajectory else np.zeros((0, len(self.qlist), 8),
                                                                        np.float32)
        np.savez_compressed(path, keyframes=kf, fields=np.array(
            ["time", "px", "py", "pz", "qx", "qy", "qz", "qw"]))

    def update(self, seed: int) -> int:
        """The agent loop after the pair loop (LQRO:1437-1446) on the GPU:
        vGoal = newV, findU, propagateU, kalmanFilter1, the observation draw,
        kalmanFilter2, vGoal = findVGoal.  Noise from the reference's rand()
        stream seeded with `seed`; returns the next seed."""
        n = len(self.qlist)
        nrm, seed = normals(seed, n * NORMALS_PER_AGENT)
        hover = self.model.gravity * self.model.mass / 4
        st = dict(x=np.stack([q.x for q in self.qlist]), rot=np.stack([q.Rot for q in self.qlist]),
                  x_true=np.stack([q.xTrue for q in self.qlist]),
                  rot_true=np.stack([q.RotTrue for q in self.qlist]),
                  P=np.stack([q.P for q in self.qlist]), vgoal=np.stack([q.newV for q in self.qlist]),
                  u_goal=np.full((n, 4), hover), p_goal=np.stack([q.pGoal for q in self.qlist]))
        gains = {k: np.stack([getattr(q, k) for q in self.qlist]) for k in ("L", "E", "l", "Lh", "Eh")}
        kf = np.zeros((n, 8), np.float32)
        dynamics_step(st, gains, nrm, models=[self.model], per_agent=True, device=self.device,
                      keyframes=kf, time=self.t * self.model.dt)
        self.trajectory.append(kf)
        self.t += 1
        for a, q in enumerate(self.qlist):
            q.x, q.Rot, q.xTrue, q.RotTrue, q.P = (st["x"][a].copy(), st["rot"][a].copy(),
                                                   st["x_true"][a].copy(), st["rot_true"][a].copy(),
                                                   st["P"][a].copy())
            q.vGoal = st["vgoal"][a].copy()
        return seed


# ---------------------------------------------------------------------------
# Multi-GPU: rows (agents i) block-sharded over ranks
# ---------------------------------------------------------------------------
ROW_MODES = ("block", "cyclic")


def row_shard(n_agents: int, rank: int, world: int) -> tuple[int, int]:
    """Rows [rb, re) owned by `rank`: balanced contiguous blocks (sizes
    differ by at most one).  Every pair (i, j) of row i is computed by the
    owner of i; no pair is split across ranks."""
    if not (0 <= rank < world) or n_agents < world:
        raise ValueError(f"cannot shard {n_agents} agents over {world} ranks")
    return rank * n_agents // world, (rank + 1) * n_agents // world


def shard_rows(n_agents: int, rank: int, world: int, mode: str = "block") -> dict:
    """The lqro_config fields of `rank`'s shard.  "block": row_shard's
    contiguous rows.  "cyclic": rows rank, rank + world, ... (row_stride =
    world) — agents that crowd into one region of the index space (a
    formation, the hull-heavy rows of SURVEY §8e) spread over every rank
    instead of loading one."""
    if mode not in ROW_MODES:
        raise ValueError(f"row mode {mode!r} not in {ROW_MODES}")
    if mode == "block":
        rb, re = row_shard(n_agents, rank, world)
        return dict(row_begin=rb, row_end=re, row_stride=0)
    if not (0 <= rank < world) or n_agents < world:
        raise ValueError(f"cannot shard {n_agents} agents over {world} ranks")
    return dict(row_begin=rank, row_end=n_agents, row_stride=world if world > 1 else 0)


def shard_row_ids(n_agents: int, rank: int, world: int, mode: str = "block") -> np.ndarray:
    f = shard_rows(n_agents, rank, world, mode)
    return np.arange(f["row_begin"], f["row_end"], max(f["row_stride"], 1))


def step_rows(ctx, dist, x, vgoal, newv, rowtab, rank: int, world: int, mode: str = "block", stream=None):
    """One pair-loop step of this rank's rows on torch device tensors, then
    the all-gather of newV.  In Qhull order with more than one rank the step
    is split around the all-gather of the (N, 4) row-normal table `rowtab`
    (lqro_step_device_begin / _end): the loop-carried normalVector
    (LQRO:1385) runs through the whole swarm's pairs in (i, j) order."""
    import torch
    st = stream if stream is not None else torch.cuda.current_stream(x.device)
    sid = st.cuda_stream
    if world > 1 and ctx.cfg.flags & LQRO_FLAG_QHULL_ORDER:
        ctx.step_device_begin(x.data_ptr(), vgoal.data_ptr(), rowtab.data_ptr(), sid)
        with torch.cuda.stream(st):
            allgather_rows(dist, rowtab, rank, world, mode=mode)
        ctx.step_device_end(rowtab.data_ptr(), newv.data_ptr(), sid)
    else:
        ctx.step_device(x.data_ptr(), vgoal.data_ptr(), newv.data_ptr(), sid)
    if world > 1:
        with torch.cuda.stream(st):
            allgather_rows(dist, newv, rank, world, mode=mode)


def allgather_rows(dist, full, rank: int, world: int, group=None, mode: str = "block"):
    """The per-step exchange: every rank holds its own rows of `full`
    (an (N, k) tensor, rows from shard_rows(mode)); afterwards every rank
    holds all rows.  One all-gather of equal ceil(N/world)-row chunks — RCCL
    over xGMI with the "nccl" backend, gloo on the CPU."""
    import torch

    n = full.shape[0]
    chunk = -(-n // world)

    def own(r):
        if mode == "cyclic":
            return full[r::world]
        b, e = row_shard(n, r, world)
        return full[b:e]

    if mode not in ROW_MODES:
        raise ValueError(f"row mode {mode!r} not in {ROW_MODES}")
    mine = own(rank)
    send = torch.zeros((chunk,) + tuple(full.shape[1:]), dtype=full.dtype, device=full.device)
    send[: mine.shape[0]] = mine
    recv = torch.empty((chunk * world,) + tuple(full.shape[1:]), dtype=full.dtype,
                       device=full.device)
    if dist.get_backend(group) == "nccl":
        dist.all_gather_into_tensor(recv, send, group=group)
    else:
        dist.all_gather(list(recv.chunk(world)), send, group=group)
    for r in range(world):
        dst = own(r)
        dst.copy_(recv[r * chunk: r * chunk + dst.shape[0]])
    return full


class DeviceLoop:
    """The whole control loop LQRO:1391-1446 on device buffers, for the rows
    this rank owns (rows="block": [rb, re); "cyclic": rank, rank + world, ...,
    gathered into contiguous copies around the dynamics): ``step()`` is the pair loop (lqro_step_device),
    ``update()`` the agent loop after it (vGoal = newV, lqro_dynamics_step_device
    on the own rows), then the single exchange per step: an all-gather of the
    new estimates x.  Every launch goes on `stream` (default:
    torch's current stream), so RCCL's stream waits order the exchange against
    the kernels and no device synchronisation is needed between the calls.

    The noise of step t is the reference's rand() stream for all N agents in
    agent order (LQRO:1437-1446 draws per agent in turn); each rank uses its
    own rows' draws, so a sharded run equals the single-context run bit for
    bit."""

    def __init__(self, x0, vgoal0, gains: dict, horizon: int, n_points: int = 100, *,
                 p_goal=None, rank: int = 0, world: int = 1, dist=None, device=None,
                 model: Model | None = None, seed: int = 1, stream=None, rows: str = "block",
                 flags: int = LQRO_FLAG_QHULL_ORDER):
        import torch
        self.torch = torch
        self.dev = torch.device("cuda", torch.cuda.current_device()) if device is None else device
        self.stream = stream if stream is not None else torch.cuda.current_stream(self.dev)
        n = x0.shape[0]
        self.n, self.rank, self.world, self.dist = n, rank, world, dist
        self.mode = rows
        sh = shard_rows(n, rank, world, rows)
        ids = shard_row_ids(n, rank, world, rows)
        self.rb, self.re = int(ids[0]), int(ids[-1]) + 1     # block mode: the own rows [rb, re)
        rows = len(ids)
        self.model = model or default_model()
        self.seed = seed
        f64 = dict(dtype=torch.float64, device=self.dev)
        self.ctx = Context(config(n, horizon, n_points, device=self.dev.index, flags=flags, **sh))
        self.ids_h = ids
        self.ids = torch.from_numpy(ids.astype(np.int64)).to(self.dev)
        self.ctx.set_gains(gains["A"], gains["B"], gains["L"], gains["E"])
        self.x = torch.from_numpy(np.ascontiguousarray(x0, np.float64)).to(self.dev)
        self.vgoal = torch.from_numpy(np.ascontiguousarray(vgoal0, np.float64)).to(self.dev)
        self.newv = torch.zeros((n, 3), **f64)
        self.flags = flags
        self.rowtab = torch.zeros((n, 4), **f64)   # per-row loop-carried normals (Qhull order, world > 1)
        eye3 = torch.eye(3, **f64).repeat(rows, 1, 1).contiguous()
        hover = self.model.gravity * self.model.mass / 4
        pg = np.zeros((n, 3)) if p_goal is None else np.asarray(p_goal, np.float64)
        self.own = dict(rot=eye3.clone(), x_true=self.x[self.ids].clone(), rot_true=eye3.clone(),
                        P=(1e-9 * torch.eye(16, **f64)).repeat(rows, 1, 1).contiguous(),
                        u_goal=torch.full((rows, 4), hover, **f64),
                        p_goal=torch.from_numpy(np.ascontiguousarray(pg[ids])).to(self.dev))
        self.g = {k: torch.from_numpy(np.ascontiguousarray(gains[k], np.float64)).to(self.dev)
                  for k in ("L", "E", "Lh", "Eh")}
        self.g["l"] = torch.from_numpy(np.ascontiguousarray(gains.get("l", np.zeros(4)), np.float64)).to(self.dev)
        self.M = 1e-9 * torch.eye(16, **f64)
        self.Nz = 1e-9 * torch.eye(6, **f64)
        self.model_d = torch.frombuffer(bytearray(bytes(self.model)), dtype=torch.uint8).to(self.dev)
        self.nrm = None
        self._nrm_host = None   # the next update's noise draws, pinned (drawn while the GPU runs)
        self.t = 0

    def _sid(self):
        return self.stream.cuda_stream

    def step(self, gather: bool = False):
        """The pair loop for the own rows; newV of the own rows on the device
        (all rows with gather=True: one all-gather of newV)."""
        if self.world > 1 and self.flags & LQRO_FLAG_QHULL_ORDER:
            # the loop-carried normal crosses the shards: the row-normal
            # table's all-gather between the hulls and the LP
            self.ctx.step_device_begin(self.x.data_ptr(), self.vgoal.data_ptr(), self.rowtab.data_ptr(),
                                       self._sid())
            with self.torch.cuda.stream(self.stream):
                allgather_rows(self.dist, self.rowtab, self.rank, self.world, mode=self.mode)
            self.ctx.step_device_end(self.rowtab.data_ptr(), self.newv.data_ptr(), self._sid())
        else:
            self.ctx.step_device(self.x.data_ptr(), self.vgoal.data_ptr(), self.newv.data_ptr(), self._sid())
        if gather and self.world > 1:
            with self.torch.cuda.stream(self.stream):
                allgather_rows(self.dist, self.newv, self.rank, self.world, mode=self.mode)
        return self.newv

    def own_rows(self, t):
        """The own rows of an (N, k) tensor, in row order."""
        return t[self.rb:self.re] if self.mode == "block" else t[self.ids]

    def update(self):
        """LQRO:1437-1446 for the own rows, then the all-gather of x."""
        torch = self.torch
        rb, re = self.rb, self.re
        block = self.mode == "block"
        if self._nrm_host is None:
            self._nrm_host = self._draw_normals()
        with torch.cuda.stream(self.stream):
            # pinned + non-blocking: no host wait on the stream's earlier work
            self.nrm = self._nrm_host.to(self.dev, non_blocking=True)
            if block:
                self.vgoal[rb:re].copy_(self.newv[rb:re])      # vGoal = newV (LQRO:1438)
                xs, vs = self.x[rb:re], self.vgoal[rb:re]
            else:                                              # cyclic rows: contiguous copies
                xs = self.x.index_select(0, self.ids)
                vs = self.newv.index_select(0, self.ids)
        o, g = self.own, self.g
        a = Agents(xs.data_ptr(), o["rot"].data_ptr(), o["x_true"].data_ptr(), o["rot_true"].data_ptr(),
                   o["P"].data_ptr(), vs.data_ptr(), None, o["u_goal"].data_ptr(), o["p_goal"].data_ptr(),
                   g["L"].data_ptr(), g["E"].data_ptr(), g["l"].data_ptr(), g["Lh"].data_ptr(),
                   g["Eh"].data_ptr(), self.M.data_ptr(), self.Nz.data_ptr(), self.nrm.data_ptr())
        a.time = self.t * self.model.dt
        _check(lib().lqro_dynamics_step_device(C.c_void_p(self.model_d.data_ptr()), 1, len(self.ids_h), 0,
                                               C.byref(a), C.c_void_p(self._sid() or None)),
               "lqro_dynamics_step_device")
        with torch.cuda.stream(self.stream):
            if not block:
                self.x.index_copy_(0, self.ids, xs)
                self.vgoal.index_copy_(0, self.ids, vs)
            if self.world > 1:
                allgather_rows(self.dist, self.x, self.rank, self.world, mode=self.mode)
        self.t += 1
        # the next step's draws (the reference's rand() stream, in agent order)
        # on the host while this step's kernels run
        self._nrm_host = self._draw_normals()

    def _draw_normals(self):
        nrm, self.seed = normals(self.seed, self.n * NORMALS_PER_AGENT)
        host = self.torch.from_numpy(np.ascontiguousarray(nrm.reshape(self.n, NORMALS_PER_AGENT)[self.ids_h]))
        return host.pin_memory()

    def close(self):
        self.ctx.close()
