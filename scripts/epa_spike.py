"""Research spike (CPU, not product): can the inside-hull branch find the
canonical facet from a LOCAL hull around vrel instead of the full hull?

EPA-style expansion: Q = hull of a few support points (26 directions),
grown until vrel is strictly inside it; then every Q-facet whose plane
distance from vrel is within V* + delta of the best certified rule value V*,
and every Q-facet sharing a vertex with one of those, is either certified (no
point of the pair's rounded set beyond it, the oracle's eps rule: a facet of
the full hull) or expanded (its furthest point joins Q).  delta = max
|P_full - P_rounded| bounds the gap between a facet's plane distance and the
rule's value (which uses the full-precision vertex).  Why the window is then
complete: D(u) = h(u) - u.vrel is positive and concave along
great-circle arcs inside a vertex's normal cone, so any direction with
D_Q <= W lies in the normal cone of a vertex of a window facet; those
vertices have only certified (full-hull) facets around them, so Q and the
full hull share their normal cones, and every full-hull facet with plane
distance <= W is a certified facet of Q.
Compared with the oracle's full-hull result (pyoracle.hull_branch) on the
inside pairs of tests/golden/hull_rule.npz (dense swarm, C3).
usage: epa_spike.py [dense|c3|both]"""
import os, sys, time
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "oracle"), os.path.join(ROOT, "lqr-obstacles_amd")]
import pyoracle, lqro

DIRS = np.array([(a, b, c) for a in (-1, 0, 1) for b in (-1, 0, 1) for c in (-1, 0, 1) if (a, b, c) != (0, 0, 0)],
                float)


def canon(t):
    t = list(t)
    while not (t[0] < t[1] and t[0] < t[2]):
        t = t[1:] + t[:1]
    return tuple(t)


def rule_value(R, P, v, t):
    a, b, c = (R[k].tolist() for k in t)   # orc_hull_branch's arithmetic, operation by operation
    e1 = [b[0] - a[0], b[1] - a[1], b[2] - a[2]]
    e2 = [c[0] - a[0], c[1] - a[1], c[2] - a[2]]
    n = [e1[1] * e2[2] - e1[2] * e2[1], e1[2] * e2[0] - e1[0] * e2[2], e1[0] * e2[1] - e1[1] * e2[0]]
    ln = (n[0] * n[0] + n[1] * n[1] + n[2] * n[2]) ** 0.5
    n = [n[0] / ln, n[1] / ln, n[2] / ln]
    p0 = P[t[0]].tolist()
    return abs(n[0] * (v[0] - p0[0]) + n[1] * (v[1] - p0[1]) + n[2] * (v[2] - p0[2])), n


def local(R, P, v, ring=True):
    """Returns (value, canonical triple, |V|, support queries), or None when
    vrel is not strictly inside the local hull (the full hull decides then).
    ring: also certify every facet sharing a vertex with a window facet — with
    vrel inside Q that makes the window complete."""
    scale = np.abs(R).max()
    eps = 1e-13 * (scale + 1.0)
    delta = np.sqrt(((P - R) ** 2).sum(1)).max() * (1 + 1e-9) + 1e-12
    V = sorted(set(int(np.argmax(R @ d)) for d in DIRS))
    queries = 0
    cert = {}                      # triple (as produced) -> rule value; P-facets
    while True:
        F = [tuple(V[k] for k in f) for f in pyoracle.hull(R[V])]
        info = {}
        for t in F:
            a, b, c = R[t[0]], R[t[1]], R[t[2]]
            n = np.cross(b - a, c - a)
            info[t] = (n @ (v - a) / np.sqrt(n @ n), n)   # signed: < 0 inside (outward normals)
        # vrel strictly inside Q first
        out = [t for t in F if info[t][0] >= 0]
        added = False
        for t in out:
            queries += 1
            n = info[t][1]
            d = (R - R[t[0]]) @ n
            k = int(np.argmax(d))
            if d[k] > 0 and d[k] * d[k] > eps * eps * (n @ n):
                V = sorted(set(V) | {k}); added = True; break
            return None            # a P-facet with vrel on or outside it
        if added:
            continue
        order = sorted(F, key=lambda t: -info[t][0])
        best = min(cert.values()) if cert else np.inf
        for t in order:            # certify the nearest facets until the window closes
            if -info[t][0] > best + delta:
                break
            if t in cert:
                continue
            queries += 1
            n = info[t][1]
            d = (R - R[t[0]]) @ n
            k = int(np.argmax(d))
            if d[k] > 0 and d[k] * d[k] > eps * eps * (n @ n):
                V = sorted(set(V) | {k}); added = True; break
            cert[t] = rule_value(R, P, v, canon(t))[0]
            best = min(best, cert[t])
        if added:
            continue
        if ring:
            win = [t for t in F if -info[t][0] <= best + delta]
            wv = {u for t in win for u in t}
            for t in F:
                if t in cert or not (set(t) & wv):
                    continue
                queries += 1
                n = info[t][1]
                d = (R - R[t[0]]) @ n
                k = int(np.argmax(d))
                if d[k] > 0 and d[k] * d[k] > eps * eps * (n @ n):
                    V = sorted(set(V) | {k}); added = True; break
                cert[t] = rule_value(R, P, v, canon(t))[0]
            if added:
                continue
        fin = [(val, canon(t)) for t, val in cert.items() if t in info]
        val, tb = min(fin)
        return val, tb, len(V), queries


def run(name, N, H, box, seed):
    fx = np.load(os.path.join(ROOT, "tests", "golden", "hull_rule.npz"))
    g = pyoracle.synthesize()
    T, NCF = pyoracle.tables(g["A"], g["B"], g["L"], g["E"], H)
    S = pyoracle.sphere(100)
    x, _ = lqro.synthetic_swarm(N, box=box, seed=seed)
    ok = 0
    nv, nq, nfull = [], [], []
    t_loc = t_full = 0.0
    for i, j in zip(fx[f"{name}_i"], fx[f"{name}_j"]):
        _, _, P = pyoracle.pair(T, NCF, S, x[i], x[j], int(i), int(j), want_points=True)
        R = np.vectorize(pyoracle.round6)(P)
        v = x[i, 3:6] - x[j, 3:6]
        t0 = time.time()
        k, d_full, n_full, fac = pyoracle.hull_branch(P, v)
        t1 = time.time()
        res = local(R, P, v)
        t2 = time.time()
        if res is None:
            print(f"  {name} ({i},{j}): vrel not inside the local hull -> full hull")
            res = (d_full, tuple(fac.tolist()), 0, 0)
        d_loc, t_best, nverts, q = res
        t_full += t1 - t0
        t_loc += t2 - t1
        same = d_loc == d_full and sorted(t_best) == sorted(fac.tolist())
        ok += same
        nv.append(nverts); nq.append(q)
        nfull.append(len({u for f in pyoracle.hull(R) for u in f}))
        if not same:
            print(f"  MISMATCH {name} ({i},{j}): full {d_full!r} {sorted(fac.tolist())}  local {d_loc!r} {sorted(t_best)}")
    print(f"{name}: {ok}/{len(nv)} inside pairs equal to the full hull's canonical facet and distance; "
          f"local vertices mean {np.mean(nv):.0f} max {max(nv)} vs full-hull vertices mean {np.mean(nfull):.0f}; "
          f"certification queries mean {np.mean(nq):.0f} max {max(nq)}; CPU s: local {t_loc:.1f} (scipy-free C hull per "
          f"round), full {t_full:.1f}", flush=True)


if __name__ == "__main__":
    which = sys.argv[1] if len(sys.argv) > 1 else "both"
    if which in ("dense", "both"):
        run("dense", 32, 45, 3.0, 11)
    if which in ("c3", "both"):
        run("c3", 1024, 100, None, lqro.SEED)
