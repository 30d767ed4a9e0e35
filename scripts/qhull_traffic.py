#!/usr/bin/env python3
"""HBM bytes per Qhull-order hull build (k_qhull + k_qhull_big), C3.

  run:        the C3 step in Qhull order, K times (the program the PMC passes
              profile); writes the builds it made (lqro_get_hull_builds) to OUT
  summarise:  FETCH_SIZE / WRITE_SIZE passes of `run` -> bytes per build,
              stamped with the liblqro.so measured (bench.py's `critical`
              object cites it only for that build)

  rocprofv3 --pmc FETCH_SIZE --output-format csv -d DIR_F -o run -- python3 scripts/qhull_traffic.py run OUT_F
  rocprofv3 --pmc WRITE_SIZE --output-format csv -d DIR_W -o run -- python3 scripts/qhull_traffic.py run OUT_W
  python3 scripts/qhull_traffic.py summarise DIR_F DIR_W OUT_F OUT.json

FETCH_SIZE / WRITE_SIZE are KiB summed over every k_qhull / k_qhull_big
launch of the run; FETCH_SIZE doubled (gfx950 correction, MI355X_MICROARCH.md
§HBM).  The algorithmic input of a build is its points, rounded and full
precision: 48 B per point (the per-build figure is reported beside it).
"""
import csv
import glob
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "lqr-obstacles_amd"))


def run(out, steps=3):
    import lqro
    N, H = 1024, 100
    x, vg = lqro.synthetic_swarm(N)
    g = lqro.synthesize_gains()
    ctx = lqro.Context(lqro.config(N, H, 100, flags=lqro.LQRO_FLAG_QHULL_ORDER))
    ctx.set_gains(g["A"], g["B"], g["L"], g["E"])
    builds, points, per_step = 0, 0, []
    for _ in range(steps):
        ctx.step(x, vg)
        b = ctx.hull_builds()
        builds += len(b)
        points += int(b["n_points"].sum())
        per_step.append([len(b), int(b["n_points"].sum())])
    ctx.close()
    json.dump({"steps": steps, "builds": builds, "points": points, "per_step": per_step}, open(out, "w"))


def launches_kib(d, counter):
    """[(dispatch id, KiB)] of every k_qhull / k_qhull_big launch, in dispatch order"""
    f = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)[0]
    rows = []
    for r in csv.DictReader(open(f)):
        if r["Counter_Name"] == counter and ("k_qhull" in r["Kernel_Name"]):
            rows.append((int(r["Dispatch_Id"]), float(r["Counter_Value"])))
    return sorted(rows)


def total_kib(d, counter, skip=0):
    rows = launches_kib(d, counter)[skip:]
    return sum(v for _, v in rows), len(rows)


def summarise(dir_f, dir_w, run_json, out):
    rj = json.load(open(run_json))
    fk, nf = total_kib(dir_f, "FETCH_SIZE")
    wk, nw = total_kib(dir_w, "WRITE_SIZE")
    fb, wb = fk * 1024 * 2, wk * 1024
    with open(os.path.join(ROOT, "lqr-obstacles_amd", "liblqro.stamp.json")) as fh:
        stamp = json.load(fh)
    # the steady steps: a context's first two steps run the plain schedule
    # (k_qhull + k_qhull_big after the sweep: two launches each); the later
    # ones the overlapped one (the side's k_qhull, the main stream's k_qhull
    # and k_qhull_big: three launches each)
    st = {}
    ps = rj.get("per_step")
    if ps and rj["steps"] > 2:
        fs, nfs = total_kib(dir_f, "FETCH_SIZE", skip=4)
        ws, nws = total_kib(dir_w, "WRITE_SIZE", skip=4)
        bs = sum(b for b, _ in ps[2:])
        pts = sum(q for _, q in ps[2:])
        if nfs == nws == 3 * (rj["steps"] - 2) and bs > 0:
            st = {"steady_steps": rj["steps"] - 2, "steady_builds": bs,
                  "steady_fetch_bytes_per_build": fs * 1024 * 2 / bs,
                  "steady_write_bytes_per_build": ws * 1024 / bs,
                  "steady_hbm_bytes_per_build": (fs * 1024 * 2 + ws * 1024) / bs,
                  "steady_algorithmic_bytes_per_build": 48.0 * pts / bs}
    res = {"n_agents": 1024, "horizon": 100, "steps": rj["steps"], "builds": rj["builds"],
           "launches": [nf, nw],
           "fetch_bytes_per_build": fb / rj["builds"], "write_bytes_per_build": wb / rj["builds"],
           "hbm_bytes_per_build": (fb + wb) / rj["builds"],
           "algorithmic_bytes_per_build": 48.0 * rj["points"] / rj["builds"], **st,
           "method": "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE in separate passes of scripts/qhull_traffic.py run "
                     "(C3, Qhull order); every k_qhull / k_qhull_big launch summed, divided by the builds "
                     "(lqro_get_hull_builds); FETCH_SIZE x2 (gfx950 correction); steady_*: the steps after the "
                     "first two (plain schedule), launches in dispatch order",
           "build": stamp}
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    if sys.argv[1] == "run":
        run(sys.argv[2], int(sys.argv[3]) if len(sys.argv) > 3 else 4)
    else:
        summarise(*sys.argv[2:6])
