"""Row shards in Qhull order (LQRO_FLAG_QHULL_ORDER): the reference's
loop-carried normalVector (LQRObstacles.cpp:1385) runs through every pair of
the swarm in (i, j) order, so a facet-0 pair at the top of a shard takes the
normal the previous shard's rows left.  lqro_step_device_begin / _end split
the step around the exchange of each row's last normal (an all-gather in a
multi-rank run, here assembled in one process from G shard contexts on one
GPU); every shard's records and new velocities must equal one context over
all rows, bit for bit, over steps (the carry into the next step included)."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _full(lqro_mod, gains, x, vg, H, steps):
    c = lqro_mod.Context(lqro_mod.config(x.shape[0], H, 100,
                                         flags=lqro_mod.LQRO_FLAG_RECORDS | lqro_mod.LQRO_FLAG_QHULL_ORDER))
    c.set_gains(gains["A"], gains["B"], gains["L"], gains["E"])
    out = []
    for _ in range(steps):
        v = c.step(x, vg)
        out.append((v, c.records(), c.carry_normal()))
    c.close()
    return out


def _shards_vs_full(lqro_mod, gains, x, vg, H, steps, world, mode):
    from test_gpu_dyn import _Hip   # device buffers through liblqro's own HIP runtime
    N = x.shape[0]
    ref = _full(lqro_mod, gains, x, vg, H, steps)
    hip = _Hip()
    d_x, d_vg = hip.put(x), hip.put(vg)
    ctxs = []
    for g in range(world):
        c = lqro_mod.Context(lqro_mod.config(N, H, 100, flags=lqro_mod.LQRO_FLAG_RECORDS | lqro_mod.LQRO_FLAG_QHULL_ORDER,
                                             **lqro_mod.shard_rows(N, g, world, mode)))
        c.set_gains(gains["A"], gains["B"], gains["L"], gains["E"])
        ctxs.append(c)
    try:
        zt, zv = np.zeros((N, 4)), np.zeros((N, 3))
        for t in range(steps):
            tabs = [hip.put(zt) for _ in range(world)]
            newv = [hip.put(zv) for _ in range(world)]
            for g, c in enumerate(ctxs):
                c.step_device_begin(d_x, d_vg, tabs[g], 0)
            hip.sync()
            whole = np.zeros((N, 4))
            for g in range(world):   # the all-gather: each rank's own rows
                ids = lqro_mod.shard_row_ids(N, g, world, mode)
                whole[ids] = hip.get(tabs[g], zt)[ids]
            d_whole = hip.put(whole)
            for g, c in enumerate(ctxs):
                c.step_device_end(d_whole, newv[g], 0)
            hip.sync()
            v_ref, r_ref, carry_ref = ref[t]
            for g, c in enumerate(ctxs):
                ids = lqro_mod.shard_row_ids(N, g, world, mode)
                got = hip.get(newv[g], zv)[ids]
                assert np.array_equal(got.view(np.uint64), v_ref[ids].view(np.uint64)), (t, g)
                rr = c.records().reshape(len(ids), N - 1)
                want = r_ref.reshape(N, N - 1)[ids]
                for f in ("flags", "facet", "dist", "normal", "plane_point", "plane_normal"):
                    assert np.array_equal(rr[f], want[f]), (t, g, f)
                assert np.array_equal(c.carry_normal(), carry_ref), (t, g)
    finally:
        for c in ctxs:
            c.close()
        hip.free()
    return ref


@pytest.mark.parametrize("world,mode", [(2, "block"), (3, "block"), (3, "cyclic")])
def test_shards_match_one_context(lqro_mod, gains, world, mode):
    x, vg = lqro_mod.synthetic_swarm(32, box=3.0, seed=11)
    ref = _shards_vs_full(lqro_mod, gains, x, vg, 45, 2, world, mode)
    assert sum(int((r["flags"] & lqro_mod.REC_STALE).astype(bool).sum()) for _, r, _ in ref) > 0


def test_shards_match_one_context_c3(lqro_mod, gains, monkeypatch):
    """The same at C3's size (two shards of 512 rows): the overlap schedule,
    the speculative builds (third step) and the early LP run inside
    lqro_step_device_begin, the early rows' newV reaching the caller's buffer
    through _end."""
    for k in ("LQRO_EARLY_LP", "LQRO_QSIDE", "LQRO_HOT", "LQRO_HOT_SPLIT", "LQRO_HOT_SPEC", "LQRO_QHULL_SPARE"):
        monkeypatch.delenv(k, raising=False)
    x, vg = lqro_mod.synthetic_swarm(1024)
    _shards_vs_full(lqro_mod, gains, x, vg, 100, 3, 2, "block")


def test_begin_end_call_order(lqro_mod, gains):
    from test_gpu_dyn import _Hip
    N, H = 8, 20
    x, vg = lqro_mod.synthetic_swarm(N)
    c = lqro_mod.Context(lqro_mod.config(N, H, 50))
    c.set_gains(gains["A"], gains["B"], gains["L"], gains["E"])
    hip = _Hip()
    d_x, d_vg = hip.put(x), hip.put(vg)
    tab, nv = hip.put(np.zeros((N, 4))), hip.put(np.zeros((N, 3)))
    try:
        with pytest.raises(RuntimeError):
            c.step_device_end(tab, nv, 0)      # no begin
        c.step_device_begin(d_x, d_vg, tab, 0)
        with pytest.raises(RuntimeError):
            c.step_device(d_x, d_vg, nv, 0)   # a step in the middle
        c.step_device_end(tab, nv, 0)
        hip.sync()
        got = hip.get(nv, np.zeros((N, 3)))
        assert np.array_equal(got.view(np.uint64), c.step(x, vg).view(np.uint64))
    finally:
        c.close()
        hip.free()


def test_c4_eight_shards_match_one_context(lqro_mod, gains, monkeypatch):
    """C4 (4096 quadrotors, H = 100) as the 8-GPU strong-scaled run splits it:
    the 8 block shards of 512 rows, each through lqro_step_device_begin, the
    row-normal table assembled from the 8 (the all-gather), then _end — over
    three steps (the third in the speculative-build steady state), each shard
    entered with the normal the step before left.  Every row's newV, every
    row's last normal in the table and every shard's carried normal equal one
    whole-swarm context's bit for bit (LQRO:1385: the loop-carried
    normalVector runs through all 16.8 M pairs across the shards), and the
    shards' inside-hull counts add up to the whole swarm's."""
    from test_gpu_dyn import _Hip
    for k in ("LQRO_EARLY_LP", "LQRO_QSIDE", "LQRO_HOT", "LQRO_HOT_SPLIT", "LQRO_HOT_SPEC", "LQRO_QHULL_SPARE"):
        monkeypatch.delenv(k, raising=False)
    N, H, G, steps = 4096, 100, 8, 3
    x, vg = lqro_mod.synthetic_swarm(N)
    hip = _Hip()
    d_x, d_vg = hip.put(x), hip.put(vg)
    zt, zv = np.zeros((N, 4)), np.zeros((N, 3))
    whole = lqro_mod.Context(lqro_mod.config(N, H, 100, flags=lqro_mod.LQRO_FLAG_QHULL_ORDER))
    whole.set_gains(gains["A"], gains["B"], gains["L"], gains["E"])
    ctxs = []
    for g in range(G):
        c = lqro_mod.Context(lqro_mod.config(N, H, 100, flags=lqro_mod.LQRO_FLAG_QHULL_ORDER,
                                             **lqro_mod.shard_rows(N, g, G, "block")))
        c.set_gains(gains["A"], gains["B"], gains["L"], gains["E"])
        ctxs.append(c)
    try:
        for t in range(steps):
            w_tab, w_nv = hip.put(zt), hip.put(zv)
            whole.step_device_begin(d_x, d_vg, w_tab, 0)
            whole.step_device_end(w_tab, w_nv, 0)
            hip.sync()
            ref_tab, ref_nv = hip.get(w_tab, zt), hip.get(w_nv, zv)
            ref_carry, ref_st = whole.carry_normal(), whole.stats()
            assert ref_st["hull_fail"] == 0 and ref_st["inside"] > 500, ref_st
            tabs = [hip.put(zt) for _ in range(G)]
            nvs = [hip.put(zv) for _ in range(G)]
            for g, c in enumerate(ctxs):
                c.step_device_begin(d_x, d_vg, tabs[g], 0)
            hip.sync()
            tab = np.zeros((N, 4))
            for g in range(G):   # the all-gather: each rank's own rows
                ids = lqro_mod.shard_row_ids(N, g, G, "block")
                tab[ids] = hip.get(tabs[g], zt)[ids]
            assert np.array_equal(tab.view(np.uint64), ref_tab.view(np.uint64)), t
            d_tab = hip.put(tab)
            for g, c in enumerate(ctxs):
                c.step_device_end(d_tab, nvs[g], 0)
            hip.sync()
            inside = 0
            for g, c in enumerate(ctxs):
                ids = lqro_mod.shard_row_ids(N, g, G, "block")
                got = hip.get(nvs[g], zv)[ids]
                assert np.array_equal(got.view(np.uint64), ref_nv[ids].view(np.uint64)), (t, g)
                assert np.array_equal(c.carry_normal(), ref_carry), (t, g)
                st = c.stats()
                assert st["hull_fail"] == 0 and st["qhull_timeouts"] == 0, (t, g, st)
                inside += st["inside"]
            assert inside == ref_st["inside"], (t, inside, ref_st["inside"])
    finally:
        whole.close()
        for c in ctxs:
            c.close()
        hip.free()
