import sys, os
sys.path[:0] = ["lqr-obstacles_amd", "oracle"]
import numpy as np, lqro, pyoracle as po
N, H, NP = 512, 100, 100
x, vg = lqro.synthetic_swarm(N, seed=3)
g = lqro.synthesize_gains()
outs = []
envs = [{"LQRO_HOT": "0"}, {"LQRO_HOT": "1", "LQRO_SIDE_HULL_CUS": "32"}, {"LQRO_HOT": "1", "LQRO_HOT_R": "0.5"}]
for env in envs:
    for k in ("LQRO_HOT", "LQRO_SIDE_HULL_CUS", "LQRO_HOT_R"):
        os.environ.pop(k, None)
    os.environ.update(env)
    c = lqro.Context(lqro.config(N, H, NP, flags=lqro.LQRO_FLAG_RECORDS))
    c.set_gains(g["A"], g["B"], g["L"], g["E"])
    v = c.step(x, vg); r = c.records(); c.close()
    outs.append((v, r))
(v0, r0), (v1, r1), (v2, r2) = outs
print("cfg3 rows differing:", np.where(~np.all(v0 == v2, axis=1))[0][:20])
rows = np.where(~np.all(v0 == v1, axis=1))[0]
print("rows differing:", rows[:20], len(rows))
for f in ("n_reach", "reach_hash", "flags", "facet", "dist", "normal", "plane_point", "plane_normal"):
    d = ~np.all(np.atleast_2d((r0[f] == r1[f]).reshape(len(r0), -1)), axis=1) if r0[f].ndim > 1 else (r0[f] != r1[f])
    print(f, int(d.sum()), np.where(d)[0][:5])
ins = (r0["flags"] & 2) != 0
print("inside", int(ins.sum()), "inside rows", sorted(set(r0["i"][ins].tolist()))[:30])
T, NCF = po.tables(g["A"], g["B"], g["L"], g["E"], H)
S = po.sphere(NP)
rv, rr = po.step(T, NCF, S, x, vg, threads=16)
print("oracle vs hot0 rows", np.where(~np.all(rv == v0, axis=1))[0][:10], "vs hot1", np.where(~np.all(rv == v1, axis=1))[0][:10])
for rw in rows[:5]:
    print(rw, v0[rw], v1[rw], rv[rw])
