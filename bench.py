#!/usr/bin/env python3
"""bench.py — agent-pair LQR-obstacle evals/sec on MI355X.

Workload (BASELINE.json configs[2], "C3"): 1024 quadrotors, horizon 100,
100 points per sampled ellipsoid, 16-D state — the largest single-GPU config.
One step = the whole pair loop of LQRObstacles.cpp:1393-1436 over all
1024*1023 ordered pairs (sweep + reachable filter + GJK + in-kernel hull +
half-plane) and the per-agent new-velocity LP, with agent states, goals and
gains already resident in HBM.  Computed in fp64 with the reference's
operation order (results bit-identical to the reference CPU path).

Multi-GPU (python -m torch.distributed.run --nproc-per-node G bench.py --gpus G):
rows (agents i) are block-sharded over ranks, each rank runs its rows' pairs,
then one RCCL all-gather of the new velocities (the per-step state exchange,
SURVEY.md §8e).  Weak scaling: the swarm grows to round(1024 sqrt(G)) agents
so that every GPU keeps C3's ~1.05 M pairs per step (the path is all-pairs,
O(N^2)); --agents fixes N instead (e.g. --agents 4096 at G = 8 is C4).

Prints ONE JSON line (rank 0).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "lqr-obstacles_amd"))

N_AGENTS, HORIZON, N_POINTS, X_DIM = 1024, 100, 100, 16
FP64_VALU_PEAK_TFLOPS = 78.6     # MI355X FP64 vector (spec), MI355X_MICROARCH.md
HBM_PEAK_GBS = 8000.0


def sweep_flops_per_pair(X=X_DIM, H=HORIZON, NP=N_POINTS) -> int:
    """SURVEY.md §8d's algorithmic work per agent-pair, the unit of the
    metric: F_pair = X + H*(6X + 11*NP) (dx; off_t = W_t*dx; per point 3 adds
    + 3 subs + 5 for |d|^2).  GJK and hull are data-dependent and excluded."""
    return X + H * (6 * X + 11 * NP)


def exact_order_flops_per_pair(X=X_DIM, H=HORIZON, NP=N_POINTS) -> int:
    """What the reference-order sweep evaluates if no slice is pruned
    (informational): Translate_k (6X per k), then per point u = s + tr (3),
    Transform*u accumulated from 0.0 (18), reachable test (8)."""
    return H * (6 * X) + H * NP * (3 + 18 + 8)


def algorithmic_bytes_per_pair(X=X_DIM) -> int:
    """Compulsory HBM bytes per pair: read x_i, x_j (fp64), write one 32-B
    half-plane slot."""
    return 2 * X * 8 + 32


def lib_sha256() -> str:
    import hashlib
    with open(os.path.join(ROOT, "lqr-obstacles_amd", "liblqro.so"), "rb") as f:
        return hashlib.sha256(f.read()).hexdigest()


def pmc_traffic(kernel: str = "k_pair"):
    """HBM bytes per launch of `kernel` from the committed PMC passes
    (profiles/*_pmc_traffic.json, written by scripts/pmc_traffic.py from
    separate rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE runs of this bench at
    N=1, FETCH_SIZE doubled per the gfx950 correction).  Only a file whose
    build stamp is the liblqro.so this bench runs is cited; None otherwise."""
    import glob
    sha = lib_sha256()
    for path in sorted(glob.glob(os.path.join(ROOT, "profiles", "*_pmc_traffic.json")), reverse=True):
        with open(path) as f:
            d = json.load(f)
        if d.get("build", {}).get("lib_sha256") != sha:
            continue
        k = d.get("kernels", {}).get(kernel)
        if not k or d.get("n_agents") != N_AGENTS or d.get("horizon") != HORIZON:
            continue
        return k["hbm_bytes_per_launch"], os.path.relpath(path, ROOT)
    return None


def qhull_traffic():
    """HBM bytes per Qhull-order hull build from the committed PMC passes
    (profiles/*_qhull_traffic.json, scripts/qhull_traffic.py), cited only
    when its build stamp is the liblqro.so this bench runs."""
    import glob
    sha = lib_sha256()
    for path in sorted(glob.glob(os.path.join(ROOT, "profiles", "*_qhull_traffic.json")), reverse=True):
        with open(path) as f:
            d = json.load(f)
        if d.get("build", {}).get("lib_sha256") == sha:
            return d, os.path.relpath(path, ROOT)
    return None


def critical_path(ctx):
    """The step's critical path in the default rule: its Qhull-order hull
    builds (k_qhull, lqro_get_hull_builds of the last timed step, the GPU's
    100 MHz clock): the slowest build, the mean, microseconds per insertion,
    and the HBM bytes per build from the stamped PMC passes."""
    b = ctx.hull_builds()
    if len(b) == 0:
        return None
    dur = (b["t_end"].astype(np.int64) - b["t_start"].astype(np.int64)) / 1e5      # ms
    k = int(np.argmax(dur))
    t0 = int(b["t_start"].min())
    tr = qhull_traffic()
    return {"kernel": "k_qhull", "builds": int(len(b)),
            "builds_k_qhull_big": int((b["kernel"] == 1).sum()),
            "slowest_build_ms": float(dur[k]), "slowest_build_pair": [int(b["i"][k]), int(b["j"][k])],
            "slowest_build_insertions": int(b["insertions"][k]), "slowest_build_points": int(b["n_points"][k]),
            "slowest_us_per_insertion": float(dur[k] * 1e3 / max(1, b["insertions"][k])),
            "mean_build_ms": float(dur.mean()),
            "mean_us_per_insertion": float(dur.sum() * 1e3 / max(1, int(b["insertions"].sum()))),
            "last_build_end_ms": float((int(b["t_end"].max()) - t0) / 1e5),
            # (the steady steps' builds, as the timed step's; the first two
            # steps' plain-schedule builds beside it)
            "hbm_bytes_per_build": (tr[0].get("steady_hbm_bytes_per_build", tr[0]["hbm_bytes_per_build"])
                                    if tr else None),
            "hbm_bytes_per_build_all_steps": tr[0]["hbm_bytes_per_build"] if tr else None,
            "algorithmic_bytes_per_build": (tr[0].get("steady_algorithmic_bytes_per_build",
                                                      tr[0]["algorithmic_bytes_per_build"]) if tr else None),
            "traffic_source": tr[1] if tr else None,
            "note": "LQRO:867-969 per inside-hull pair (qconvex's build restated in-kernel); times from each "
                    "build's job start to its half-plane, s_memrealtime; last_build_end_ms from the first build's start"}


def cpu_model() -> str:
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def usable_cores() -> tuple:
    """Cores this process can run on: its CPU affinity, capped by the cgroup
    CPU quota when one is set (the GPU box gives each GPU a share of a large
    host); (cores, affinity count, quota or None)."""
    aff = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    quota = None
    try:
        q, period = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            quota = max(1, int(int(q) / int(period)))
    except (OSError, ValueError):
        pass
    return (min(aff, quota) if quota else aff), aff, quota


def cpu_baseline(x, vg, gains, hull_rule="qhull", seconds_target=10.0):
    """The reference-faithful CPU restatement (oracle/, orc_step_faithful_mt:
    the reference's per-pair findFG recursion, LQRO:1401-1406, its two GJK
    runs per outside pair, LQRO:1410/1414, and — hull_rule "qhull" — Qhull's
    own build for the inside-hull pairs, oracle/lqro_qhull.c, as qconvex
    computes them; calibrated against the reference's own code compiled in
    the build container) on the host cores, BASELINE.md §3:
    C3 rows on 1 core and on every usable core (~seconds_target each, the
    hull branch's time and inside-hull pairs reported apart), C1 and C2 whole
    steps, C4 and C5 extrapolated from measured per-pair rates (labelled)."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import pyoracle  # test infrastructure, used here only as the timed CPU baseline
    import lqro

    cores, aff, quota = usable_cores()
    pyoracle.set_hull_rule(1 if hull_rule == "qhull" else 0)
    S = pyoracle.sphere(N_POINTS)

    def timed(xx, vv, g, H, rows, threads, per_agent=False):
        pyoracle.hull_time(reset=True)
        t0 = time.perf_counter()
        pyoracle.step_faithful(g["A"], g["B"], g["L"], g["E"], pyoracle.sphere(N_POINTS), xx, vv, H,
                               rows=rows, threads=threads, records=False, per_agent=per_agent)
        dt = time.perf_counter() - t0
        hs, hc = pyoracle.hull_time(reset=True)
        return dt, hs, hc

    def rate(threads, row0):
        # calibrate on one row per thread, then scale the sample to the target
        dt, _, _ = timed(x, vg, gains, HORIZON, (row0, row0 + threads), threads)
        more = int(max(0, min(N_AGENTS - row0 - threads, (seconds_target - dt) / max(dt, 1e-9) * threads)))
        more = (more // threads) * threads
        rows, secs, hs, hc = threads, dt, 0.0, 0
        if more > 0:
            secs, hs, hc = timed(x, vg, gains, HORIZON, (row0 + threads, row0 + threads + more), threads)
            rows = more
        return rows * (N_AGENTS - 1) / secs, rows, secs, hs, hc

    one, rows1, _, _, _ = rate(1, 0)
    allc, rows_all, secs_all, hsec, hcnt = rate(cores, 64)
    small = {}
    for name, N, H in (("c1", 4, 50), ("c2", 64, 50)):
        xx, vv = lqro.synthetic_swarm(N)
        dt, _, hc = timed(xx, vv, gains, H, (0, N), min(cores, N))
        small[name] = {"agents": N, "horizon": H, "pairs": N * (N - 1), "ms_per_step": dt * 1e3,
                       "evals_per_s": N * (N - 1) / dt, "inside_hull_pairs": hc, "threads": min(cores, N),
                       "kind": "measured"}
    # C5: 12-D reduced model, per-agent gains, H = 200 — a sample of rows, extrapolated
    N5 = 16384
    x5, v5 = lqro.synthetic_swarm(N5, x_dim=12)
    ms = [pyoracle.synthesize(pyoracle.Model(*[getattr(m, f) for f, _ in pyoracle.Model._fields_]), x_dim=12)
          for m in lqro.perturbed_models(64)]
    g0 = pyoracle.synthesize(x_dim=12)
    g5 = dict(A=g0["A"], B=g0["B"], L=np.repeat(np.array([m["L"] for m in ms]), N5 // 64, axis=0),
              E=np.repeat(np.array([m["E"] for m in ms]), N5 // 64, axis=0))
    dt5, _, hc5 = timed(x5, v5, g5, 200, (0, cores), cores, per_agent=True)
    r5 = cores * (N5 - 1) / dt5
    pairs4, pairs5 = 4096 * 4095, N5 * (N5 - 1)
    small["c4"] = {"agents": 4096, "horizon": 100, "pairs": pairs4, "ms_per_step": pairs4 / allc * 1e3,
                   "kind": "extrapolated from the C3 per-pair rate on all cores"}
    small["c5"] = {"agents": N5, "horizon": 200, "x_dim": 12, "pairs": pairs5, "ms_per_step": pairs5 / r5 * 1e3,
                   "sample": f"{cores} rows x {N5 - 1} pairs in {dt5:.1f} s ({hc5} inside-hull pairs)",
                   "kind": "extrapolated from a sampled per-pair rate on all cores"}
    pyoracle.set_hull_rule(0)
    return {"value": allc, "unit": "agent-pair evals/s", "cores": cores, "kind": "port",
            "mode": "reference-faithful (per-pair findFG, GJK twice per outside pair, " +
                    ("Qhull's build for inside-hull pairs" if hull_rule == "qhull" else "canonical hull rule") +
                    "; bit-identical results to the GPU path's rule)",
            "cores_1": one, "cores_all": allc, "cpu_model": cpu_model(), "host_cpus_visible": os.cpu_count(),
            "cpu_affinity": aff, "cgroup_cpu_quota": quota,
            "c3_hull_seconds_all_cores": hsec, "c3_hull_fraction": hsec / max(secs_all * cores, 1e-9),
            "c3_sample_inside_hull_pairs": hcnt,
            "configs": small,
            "sample": f"C3 step rows: {rows1} rows on 1 core, {rows_all} rows on {cores} threads "
                      f"({N_AGENTS - 1} pairs per row)"}


def hull_flags(lqro, rule: str) -> int:
    """qhull: the reference's own inside-hull rule over Qhull's build order
    (LQRO_FLAG_QHULL_ORDER, k_qhull: results equal the reference loop over
    Qhull); canonical: this build's faster canonical facet rule (a measured
    deviation)."""
    return lqro.LQRO_FLAG_QHULL_ORDER if rule == "qhull" else 0


def closed_loop(lqro, torch, dev, x, vg, gains, reps, world=1, dist=None, rank=0, mode="block", flags=0):
    """The whole control step on the GPU, measured after the timed steps:
    lqro.DeviceLoop — the pair step, then the agent loop LQRO:1437-1446
    (k_dynw: findU, propagate, kalmanFilter1/2, findVGoal) on this rank's
    rows, then the one all-gather of x (N > 1), all on torch's current stream
    with no synchronisation between the calls (x and vGoal never leave HBM).
    Reported beside the headline, not in `value`.  Its own context and
    buffers start from the bench's swarm, so the roofline probe after it sees
    the timed steps' inputs."""
    loop = lqro.DeviceLoop(x, vg, dict(gains, l=np.zeros(4)), HORIZON, N_POINTS,
                           rank=rank, world=world, dist=dist, device=dev, rows=mode, flags=flags)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    it_ms, its, dms = [], [], []
    for _ in range(reps):
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        loop.step()
        tm = loop.ctx.timings()
        e0.record(loop.stream)
        loop.update()
        e1.record(loop.stream)
        torch.cuda.synchronize(dev)
        it_ms.append((time.perf_counter() - t0) * 1e3)
        dms.append(e0.elapsed_time(e1))
        its.append({"pair_ms": round(tm["pair_ms"], 3), "hull_ms": round(tm["hull_ms"], 3),
                    "lp_ms": round(tm["lp_ms"], 3), "inside": loop.ctx.stats()["inside"]})
    loop.close()
    return {"kernel": "k_dynw", "agents": len(loop.ids_h),
            "dynamics_plus_gather_ms": float(np.mean(dms)),
            "pair_step_plus_dynamics_ms": float(np.mean(it_ms)),
            "iteration_ms": [round(t, 3) for t in it_ms], "iterations": its,
            "note": "closed loop LQRO:1391-1446 on device buffers (lqro.DeviceLoop); "
                    "dynamics_plus_gather_ms from events on the launch stream"}


def config_runs(lqro, torch, dev, local, world, rank, dist, steps, mode="block", flags=0):
    """BASELINE configs 4 and 5 beside the headline (never in `value`):
    strong scaling — the whole swarm's rows sharded over the ranks, the
    per-step exchange as in the headline; max over ranks of the time for
    `steps` steps.  C4: 4096 quadrotors, H = 100, shared gains.  C5: 16384
    agents of the 12-DoF reduced model, per-agent gains of ±1 %-perturbed
    models (synthesised on the GPU), H = 200."""
    out = {}
    for name, N, H, X in (("c4", 4096, 100, 16), ("c5", 16384, 200, 12)):
        sh = lqro.shard_rows(N, rank, world, mode)
        x, vg = lqro.synthetic_swarm(N, x_dim=X)
        if name == "c5":
            g = lqro.synthesize_gains_batch(lqro.perturbed_models(N), device=local, x_dim=X)
            g0 = lqro.synthesize_gains(x_dim=X)      # the shared linearisation (LQRO:1265-1266)
            gains, per_agent = dict(A=g0["A"], B=g0["B"], L=g["L"], E=g["E"]), True
        else:
            gains, per_agent = lqro.synthesize_gains(), False
        ctx = lqro.Context(lqro.config(N, H, N_POINTS, x_dim=X, device=local, flags=flags, **sh))
        ctx.set_gains(gains["A"], gains["B"], gains["L"], gains["E"], per_agent=per_agent)
        d_x = torch.from_numpy(x).to(dev)
        d_vg = torch.from_numpy(vg).to(dev)
        d_newv = torch.zeros((N, 3), dtype=torch.float64, device=dev)

        rowtab = torch.zeros((N, 4), dtype=torch.float64, device=dev)

        def step():
            lqro.step_rows(ctx, dist, d_x, d_vg, d_newv, rowtab, rank, world, mode)
        for _ in range(2):   # untimed warmup: the schedule follows the work of the step two before
            step()
        torch.cuda.synchronize(dev)
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        for _ in range(steps):
            step()
        torch.cuda.synchronize(dev)
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize(dev)
        el = time.perf_counter() - t0
        st = ctx.stats()
        ctx.close()
        if world > 1:
            t = torch.tensor([el], dtype=torch.float64, device=dev)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            el = float(t.item())
        out[name] = {"n_agents": N, "horizon": H, "x_dim": X, "per_agent_gains": per_agent,
                     "pairs_per_step": N * (N - 1), "steps": steps, "ms_per_step": el / steps * 1e3,
                     "evals_per_s": N * (N - 1) * steps / el, "scaling": "strong",
                     "rank0_inside_hull": st["inside"], "rank0_hull_failures": st["hull_fail"]}
        if world == 1:
            out[name]["rank_shard_g8"] = rank_shard_run(lqro, torch, dev, local, N, H, X, gains, per_agent, x, vg,
                                                        steps, flags, out[name]["ms_per_step"])
    return out


def rank_shard_run(lqro, torch, dev, local, N, H, X, gains, per_agent, x, vg, steps, flags, whole_ms, G=8):
    """Every rank's work at G = 8, on this GPU, one shard after the other:
    rows [g N/8, (g+1) N/8) with the full schedule of a rank
    (lqro_step_device_begin, the row-normal table, _end; the all-gathers
    themselves are not timed: no other rank).  The 8-GPU step is the slowest
    rank's and cannot be shorter than the slowest shard's step here, so
    whole_ms / max is the strong-scaling ceiling this build has at 8 GPUs
    (SURVEY §8e)."""
    d_x = torch.from_numpy(x).to(dev)
    d_vg = torch.from_numpy(vg).to(dev)
    d_newv = torch.zeros((N, 3), dtype=torch.float64, device=dev)
    rowtab = torch.zeros((N, 4), dtype=torch.float64, device=dev)
    s = torch.cuda.current_stream(dev).cuda_stream
    shards = []
    for g in range(G):
        rows = (g * N // G, (g + 1) * N // G)
        ctx = lqro.Context(lqro.config(N, H, N_POINTS, x_dim=X, device=local, flags=flags,
                                       row_begin=rows[0], row_end=rows[1]))
        ctx.set_gains(gains["A"], gains["B"], gains["L"], gains["E"], per_agent=per_agent)

        def step():
            ctx.step_device_begin(d_x.data_ptr(), d_vg.data_ptr(), rowtab.data_ptr(), s)
            ctx.step_device_end(rowtab.data_ptr(), d_newv.data_ptr(), s)
        for _ in range(2):   # (the schedule follows the inside-hull count of the step two before)
            step()
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        for _ in range(steps):
            step()
        torch.cuda.synchronize(dev)
        el = time.perf_counter() - t0
        st = ctx.stats()
        crit = critical_path(ctx) if flags & lqro.LQRO_FLAG_QHULL_ORDER else None
        ctx.close()
        shards.append({"rows": list(rows), "ms_per_step": el / steps * 1e3, "inside_hull": st["inside"],
                       "hull_failures": st["hull_fail"],
                       "slowest_build_ms": crit["slowest_build_ms"] if crit else None})
    ms = [q["ms_per_step"] for q in shards]
    worst = int(np.argmax(ms))
    return {"shards": G, "pairs_per_shard_step": (N // G) * (N - 1), "steps": steps,
            "max_ms_per_step": max(ms), "mean_ms_per_step": float(np.mean(ms)),
            "slowest_shard_rows": shards[worst]["rows"],
            "strong_scaling_ceiling_g8": whole_ms / max(ms),
            "hull_failures": sum(q["hull_failures"] for q in shards),
            "per_shard": [{k: (round(v, 3) if isinstance(v, float) else v) for k, v in q.items()} for q in shards],
            "note": "every rank's rows of the 8-GPU strong-scaled swarm, one shard after the other on this one GPU; "
                    "the ceiling is the whole swarm's step on this GPU over the slowest shard's"}


CPP_BENCH = os.path.join(ROOT, "tests", "cpp", "lqro_bench_main")


def cpp_host_run(lqro, x, vg, steps, warmup, world, rank, local, dist):
    """The C++ multi-GPU host (include/lqro_sharded.hpp, lqro::ShardedSimulator)
    on the same swarm: one child process per rank (tests/cpp/lqro_bench_main,
    built by __graft_entry__.build), its own RCCL communicators, K iterations
    of the reference's agent loop LQRO:1391-1446 — the pair loop (world > 1:
    begin, row-normal all-gather, end), the dynamics and the all-gather of x —
    timed between two barriers, max over ranks.  Returns rank 0's result (a
    dict; {"error": ...} if the child failed)."""
    import subprocess
    import tempfile
    N = x.shape[0]
    token = [f"{os.getpid()}_{time.time_ns()}"]
    if world > 1:
        dist.broadcast_object_list(token, src=0)
    tmp = tempfile.gettempdir()
    uid = os.path.join(tmp, f"lqro_bench_uid_{token[0]}")
    inp = os.path.join(tmp, f"lqro_bench_in_{token[0]}_{rank}.bin")
    with open(inp, "wb") as f:
        np.array([N, HORIZON, N_POINTS, steps], np.int32).tofile(f)
        np.array([0x4C51524F], np.uint32).tofile(f)
        for a in (x, vg, -x[:, :3]):
            np.ascontiguousarray(a, np.float64).tofile(f)
    try:
        r = subprocess.run([CPP_BENCH, inp, uid, str(rank), str(world), str(local), str(warmup), str(steps)],
                           capture_output=True, text=True, timeout=600)
    except (OSError, subprocess.TimeoutExpired) as e:
        return {"error": repr(e)[:300]}
    finally:
        os.remove(inp)
    if world > 1:
        dist.barrier()
    if rank == 0 and os.path.exists(uid):
        os.remove(uid)
    if r.returncode != 0:
        return {"error": f"rank {rank}: exit {r.returncode}: {r.stderr.strip()[-300:]}"}
    if rank != 0:
        return {}
    kv = dict(t.split("=", 1) for t in r.stdout.split() if "=" in t)
    el = float(kv["elapsed_s"])
    return {"value": N * (N - 1) * steps / el, "ms_per_step": float(kv["ms_per_step"]), "steps": steps,
            "warmup": warmup, "n_agents": N, "world": world,
            "max_rank_inside_hull": int(float(kv["max_rank_inside"])),
            "max_rank_hull_failures": int(float(kv["max_rank_hull_fail"])),
            "host": "C++ lqro::ShardedSimulator (include/lqro_sharded.hpp), one process per GPU, RCCL",
            "step": "pair loop + dynamics + x all-gather (LQRO:1391-1446), host-synchronised per iteration"}


def canonical_rule_run(lqro, torch, dev, sh, gains, d_x, d_vg, d_newv, stream, steps, N, world, rank, mode):
    """The canonical hull rule (no LQRO_FLAG_QHULL_ORDER, k_lhull) on the
    timed steps' inputs, beside the headline: its step time, and the rows
    whose newV it moves beyond 1e-5 (relative) from the reference rule's
    newV of the last timed step — the deviation the default rule would
    carry.  Never in `value`."""
    ref = d_newv.clone()
    c = lqro.Context(lqro.config(N, HORIZON, N_POINTS, device=dev.index, flags=0, **sh))
    c.set_gains(gains["A"], gains["B"], gains["L"], gains["E"])
    out = torch.zeros_like(d_newv)
    for _ in range(2):
        c.step_device(d_x.data_ptr(), d_vg.data_ptr(), out.data_ptr(), stream.cuda_stream)
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(steps):
        c.step_device(d_x.data_ptr(), d_vg.data_ptr(), out.data_ptr(), stream.cuda_stream)
    torch.cuda.synchronize(dev)
    el = time.perf_counter() - t0
    c.close()
    rows = lqro.shard_row_ids(N, rank, world, mode)
    a, b = out[rows].cpu().numpy(), ref[rows].cpu().numpy()
    rel = np.abs(a - b).max(1) / np.maximum(np.abs(b).max(1), 1e-30)
    return {"ms_per_step": el / steps * 1e3, "evals_per_s": len(rows) * (N - 1) * steps / el,
            "hull_rule_rows_off": int((rel > 1e-5).sum()), "rows": len(rows),
            "max_rel_newv_diff": float(rel.max()) if len(rel) else 0.0,
            "note": "canonical facet rule (k_lhull), same inputs; rows_off = rows whose newV differs from "
                    "the reference rule's beyond 1e-5 relative (this rank's rows)"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--agents", type=int, default=0,
                    help="swarm size (default: round(1024 sqrt(world)), C3's pairs per GPU)")
    ap.add_argument("--no-roofline-probe", action="store_true")
    ap.add_argument("--no-configs", action="store_true", help="skip the C4 / C5 strong-scaling runs")
    ap.add_argument("--rows", choices=("auto", "block", "cyclic"), default=os.environ.get("LQRO_ROWS", "auto"),
                    help="row sharding over ranks: contiguous blocks, cyclic (row_stride = world), or auto: "
                         "blocks unless the warm-up steps' inside-hull pairs per rank differ by more than 10 %%")
    ap.add_argument("--hull-rule", choices=("qhull", "canonical"), default=os.environ.get("LQRO_HULL_RULE", "qhull"),
                    help="inside-hull rule: the reference's (Qhull's build order, default) or the canonical one")
    ap.add_argument("--host", choices=("python", "cpp"), default=os.environ.get("LQRO_BENCH_HOST", "python"),
                    help="whose timed steps are `value`: the Python host (lqro.step_rows) or the C++ host "
                         "(lqro::ShardedSimulator, a child process per rank); the other is reported beside it")
    ap.add_argument("--no-host-cpp", action="store_true", help="skip the C++ host run (python host only)")
    args = ap.parse_args()

    import torch
    import lqro

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    # one process per GPU; more ranks than GPUs (a rehearsal on a smaller box)
    # share them round-robin.  LQRO_BENCH_BACKEND=gloo rehearses the exchange
    # without RCCL (the driver's runs use the default, RCCL).
    local = int(os.environ.get("LOCAL_RANK", "0")) % max(1, torch.cuda.device_count())
    backend = os.environ.get("LQRO_BENCH_BACKEND", "nccl")
    if args.gpus != world and world > 1:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world}")
    dist = None
    if world > 1:
        import torch.distributed as dist
        torch.cuda.set_device(local)
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend)
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)

    N = args.agents if args.agents > 0 else int(round(N_AGENTS * world ** 0.5))
    x, vg = lqro.synthetic_swarm(N)
    gains = lqro.synthesize_gains()
    flags = hull_flags(lqro, args.hull_rule)
    d_x = torch.from_numpy(x).to(dev)
    d_vg = torch.from_numpy(vg).to(dev)
    d_newv = torch.zeros((N, 3), dtype=torch.float64, device=dev)
    stream = torch.cuda.current_stream(dev)
    rowtab = torch.zeros((N, 4), dtype=torch.float64, device=dev)

    def make_ctx(mode):
        c = lqro.Context(lqro.config(N, HORIZON, N_POINTS, device=local, flags=flags,
                                     **lqro.shard_rows(N, rank, world, mode)))
        c.set_gains(gains["A"], gains["B"], gains["L"], gains["E"])
        return c

    # row sharding: an inside-hull pair costs ~50x a plain one and follows the
    # swarm's geometry, so "auto" keeps contiguous blocks unless the warm-up
    # steps show one rank holding > 10 % more of them than the mean (then
    # cyclic rows spread them)
    mode = "block" if args.rows == "auto" else args.rows
    ctx = make_ctx(mode)
    rows_auto = None

    def step():
        # (Qhull order, world > 1: split around the row-normal all-gather)
        lqro.step_rows(ctx, dist, d_x, d_vg, d_newv, rowtab, rank, world, mode, stream)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize(dev)
    if args.rows == "auto" and world > 1:
        mine = float(ctx.stats()["inside"])
        cmax = torch.tensor([mine], dtype=torch.float64, device=dev)
        csum = torch.tensor([mine], dtype=torch.float64, device=dev)
        dist.all_reduce(cmax, op=dist.ReduceOp.MAX)
        dist.all_reduce(csum)
        mean = float(csum.item()) / world
        imb = float(cmax.item()) / mean if mean > 0 else 1.0
        rows_auto = {"block_inside_max_rank": float(cmax.item()), "block_inside_mean": mean, "imbalance": imb,
                     "chose": "cyclic" if imb > 1.10 else "block"}
        if imb > 1.10:
            ctx.close()
            mode = "cyclic"
            ctx = make_ctx(mode)
            for _ in range(max(1, args.warmup)):
                step()
            torch.cuda.synchronize(dev)
    args.rows = mode
    sh = lqro.shard_rows(N, rank, world, mode)
    rows = len(lqro.shard_row_ids(N, rank, world, mode))
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    pair_ms, step_dev_ms = [], []
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
        tm = ctx.timings()          # HIP events on the launch stream (waits for this step)
        pair_ms.append(tm["pair_ms"])
        step_dev_ms.append(tm["step_ms"])
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    elapsed = time.perf_counter() - t0
    st = ctx.stats()
    crit = critical_path(ctx) if flags & lqro.LQRO_FLAG_QHULL_ORDER else None
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
        c = torch.tensor([st["inside"], st["hull_fail"]], dtype=torch.int64, device=dev)
        dist.all_reduce(c)
        st["inside"], st["hull_fail"] = int(c[0]), int(c[1])

    pairs_step = N * (N - 1)
    value = pairs_step * args.steps / elapsed
    ms_step = elapsed / args.steps * 1e3
    sweep_ms = float(np.mean(pair_ms))
    # Roofline of the dominant kernel, k_pair.  In the timed steps k_pair runs
    # as two launches beside the hull (hot pairs + rows on a side stream, rows
    # on the main stream), so its own duration is measured right after, on
    # this rank's same rows, with the overlap off (LQRO_HOT=0: one k_pair
    # launch over all pairs, HIP events on its launch stream).
    # the closed loop runs before the probe creates a second context (whose
    # stream can share a hardware queue with this context's side stream)
    ctx.close()   # one context at a time: a second one's streams can share hardware queues
    other = None
    if args.hull_rule == "qhull":
        other = canonical_rule_run(lqro, torch, dev, sh, gains, d_x, d_vg, d_newv, stream, args.steps, N, world, rank,
                                   args.rows)
    closed = closed_loop(lqro, torch, dev, x, vg, gains, min(args.steps, 5), world, dist, rank, args.rows, flags)
    host_cpp = None
    if args.host == "cpp" or not args.no_host_cpp:
        if args.rows != "block" or args.hull_rule != "qhull":
            host_cpp = {"error": "the C++ host shards rows in blocks with the reference's hull rule"}
        else:
            host_cpp = cpp_host_run(lqro, x, vg, args.steps if args.host == "cpp" else min(args.steps, 5),
                                    args.warmup if args.host == "cpp" else 1, world, rank, local, dist)
    pk_ms = sweep_ms
    probe = "sweep (k_prio + k_pair launches + overlapped side hull), timed steps"
    if not args.no_roofline_probe:
        os.environ["LQRO_HOT"] = "0"
        pctx = lqro.Context(lqro.config(N, HORIZON, N_POINTS, device=local, flags=0, **sh))   # k_pair only
        del os.environ["LQRO_HOT"]
        pctx.set_gains(gains["A"], gains["B"], gains["L"], gains["E"])
        pk = []
        for k in range(1 + min(args.steps, 5)):
            pctx.step_device(d_x.data_ptr(), d_vg.data_ptr(), d_newv.data_ptr(), stream.cuda_stream)
            if k:
                pk.append(pctx.timings()["pair_ms"])
        pctx.close()
        pk_ms = float(np.mean(pk))
        probe = f"k_pair alone (LQRO_HOT=0 probe, {len(pk)} launches after the timed steps)"
    pairs_launch = rows * (N - 1)
    tflops = sweep_flops_per_pair() * pairs_launch / (pk_ms * 1e-3) / 1e12
    gbs = algorithmic_bytes_per_pair() * pairs_launch / (pk_ms * 1e-3) / 1e9
    traffic = pmc_traffic() if world == 1 else None
    out = {
        "metric": "agent-pair LQR-obstacle evals/sec",
        "value": value,
        "unit": "agent-pair evals/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": ms_step,
        "higher_is_better": True,
        "scaling": "weak" if world > 1 else "none",   # (weak: the swarm grows with the ranks; N = 1: no scaling)
        "vs_baseline": None,
        "dtype": "f64",
        "data": "synthetic (SplitMix64 swarm, seed 0x4C51524F, constant density)",
        "config": {
            "workload": (f"C3: 1024 quadrotors" if N == N_AGENTS else f"{N} quadrotors (C3 pairs per GPU)") +
                        ", horizon 100, 100 points/ellipsoid, 16-D state; "
                        "reference-exact fp64 pair sweep+GJK+hull+half-plane, fp32 LP"
                        + ("" if args.hull_rule == "qhull" else " (canonical hull rule)"),
            "n_agents": N, "horizon": HORIZON, "n_points": N_POINTS, "x_dim": X_DIM,
            "pairs_per_step": pairs_step,
            "rows_auto": rows_auto,
            "parallelism": f"rows sharded ({args.rows}) over {world} rank(s)" +
                           ((" + RCCL all-gather of newV" if backend == "nccl" else f" + {backend} all-gather of newV")
                            if world > 1 else ""),
        },
        "roofline": {
            "bound": "valu-fp64",
            "kernel": "k_pair",
            "achieved": tflops,
            "peak": FP64_VALU_PEAK_TFLOPS,
            "unit": "TFLOP/s",
            "frac": tflops / FP64_VALU_PEAK_TFLOPS,
            "traffic": traffic[0] if traffic else None,
            "traffic_unit": "bytes/launch",
            "traffic_source": traffic[1] if traffic else None,
            "flops_per_pair": sweep_flops_per_pair(),
            "flops_per_pair_exact_order": exact_order_flops_per_pair(),
            "pairs_per_launch": pairs_launch,
            "kernel_ms": pk_ms,
            "kernel_ms_source": probe,
            "hbm_algorithmic_gbs": gbs,
            "hbm_frac": gbs / HBM_PEAK_GBS,
        },
        "critical": crit,
        "step_device_ms": float(np.mean(step_dev_ms)),
        "sweep_ms": sweep_ms,
        "closed_loop": closed,
        "inside_hull_pairs_per_step": st["inside"],
        "hull_failures": st["hull_fail"],
        "hull_rule_canonical": other,
        "hull_rule": ("reference: Qhull's facet order and first Fv vertex, strict <, loop-carried normal "
                      "(LQRO:925-968; k_qhull, LQRO_FLAG_QHULL_ORDER)" if args.hull_rule == "qhull" else
                      "canonical (a measured deviation from the reference's rule, DESIGN §5.2)"),
    }
    if host_cpp is not None:
        out["host_cpp"] = host_cpp
        if args.host == "cpp":
            if "value" not in host_cpp and rank == 0:
                raise SystemExit(f"--host cpp: {host_cpp.get('error')}")
            if rank == 0:
                out["host_python"] = {"value": value, "ms_per_step": ms_step}
                out["value"], out["ms_per_step"] = host_cpp["value"], host_cpp["ms_per_step"]
                out["config"]["host"] = "cpp"
    if not args.no_configs:
        out["configs"] = config_runs(lqro, torch, dev, local, world, rank, dist, 2, args.rows, flags)
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cb = cpu_baseline(x, vg, gains, args.hull_rule)
        out["cpu_baseline"] = cb
        out["gpu_over_cpu"] = value / cb["value"]
    if rank == 0:
        print(json.dumps(out), flush=True)
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
