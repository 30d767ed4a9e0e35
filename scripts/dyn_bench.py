#!/usr/bin/env python3
"""Time k_dyn (lqro_dynamics_step_device: the per-agent step after the pair
loop, LQRO:1437-1446) on device-resident buffers, beside the oracle's
per-agent CPU time, and report how close the GPU is to the oracle.
Writes gpurun_out/dyn_bench.json."""
import ctypes as C
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "lqr-obstacles_amd"), os.path.join(ROOT, "oracle"),
                os.path.join(ROOT, "tests")]
import numpy as np  # noqa: E402

import lqro  # noqa: E402
import pyoracle  # noqa: E402
from dyn_cases import trajectory_start  # noqa: E402
from test_gpu_dyn import STATE, _Hip  # noqa: E402


def states(n, seed):
    cs = trajectory_start(n, seed)
    st = lqro.agent_states(cs["x"], p_goal=cs["p_goal"])
    st["rot"][:] = cs["rot"]
    st["rot_true"][:] = cs["rot"]
    st["P"][:] = cs["P"]
    st["vgoal"][:] = cs["vgoal"]
    return st


def main():
    L = lqro.lib()
    g = pyoracle.synthesize()
    g["l"] = np.array([0.01, -0.02, 0.03, -0.04])
    out = {"kernel": "k_dyn", "unit": "agents/s", "runs": []}
    for n in (1024, 4096, 16384):
        st = states(n, 5)
        nrm, _ = lqro.normals(1, n * lqro.NORMALS_PER_AGENT)
        hip = _Hip()
        d = {k: hip.put(v) for k, v in st.items()}
        gd = {k: hip.put(np.ascontiguousarray(g[k], np.float64)) for k in ("L", "E", "l", "Lh", "Eh")}
        a = lqro.Agents(*[d[k] for k in STATE], None, d["u_goal"], d["p_goal"],
                        *[gd[k] for k in ("L", "E", "l", "Lh", "Eh")], hip.put(1e-9 * np.eye(16)),
                        hip.put(1e-9 * np.eye(6)), hip.put(nrm))
        md = hip.put(np.frombuffer(bytes(lqro.default_model()), dtype=np.uint8))
        assert L.lqro_dynamics_step_device(C.c_void_p(md), 1, n, 0, C.byref(a), None) == 0
        hip.sync()
        first = {k: hip.get(d[k], st[k]) for k in STATE}
        reps = 10
        t0 = time.perf_counter()
        for _ in range(reps):
            assert L.lqro_dynamics_step_device(C.c_void_p(md), 1, n, 0, C.byref(a), None) == 0
        hip.sync()
        ms = (time.perf_counter() - t0) / reps * 1e3
        hip.free()
        row = {"agents": n, "ms_per_step": ms, "agents_per_s": n / ms * 1e3}
        if n == 1024:
            ref = {k: v.copy() for k, v in st.items()}
            sub = 256
            refs = {k: v[:sub].copy() for k, v in ref.items()}
            t0 = time.perf_counter()
            pyoracle.agent_step(refs, g, nrm[: sub * 22])
            row["oracle_ms_per_agent_1core"] = (time.perf_counter() - t0) / sub * 1e3
            rel = 0.0
            same = 0
            tot = 0
            for k in STATE:
                a_, b_ = first[k][:sub], refs[k]
                scale = np.maximum(np.abs(b_), 1e-3 * np.abs(b_).max() + 1e-300)
                rel = max(rel, float((np.abs(a_ - b_) / scale).max()))
                same += int(np.sum(a_.view(np.uint64) == b_.view(np.uint64)))
                tot += a_.size
            row["max_rel_err_vs_oracle"] = rel
            row["bit_identical_fraction"] = same / tot
        out["runs"].append(row)
        print(json.dumps(row), flush=True)
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    with open(os.path.join(ROOT, "gpurun_out", "dyn_bench.json"), "w") as f:
        json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
