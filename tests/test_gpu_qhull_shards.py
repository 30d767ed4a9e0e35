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


@pytest.mark.parametrize("world,mode", [(2, "block"), (3, "block"), (3, "cyclic")])
def test_shards_match_one_context(lqro_mod, gains, world, mode):
    import torch
    N, H, steps = 32, 45, 2
    x, vg = lqro_mod.synthetic_swarm(N, box=3.0, seed=11)
    ref = _full(lqro_mod, gains, x, vg, H, steps)
    assert sum(int((r["flags"] & lqro_mod.REC_STALE).astype(bool).sum()) for _, r, _ in ref) > 0
    dev = torch.device("cuda", 0)
    d_x = torch.from_numpy(x).to(dev)
    d_vg = torch.from_numpy(vg).to(dev)
    ctxs = []
    for g in range(world):
        c = lqro_mod.Context(lqro_mod.config(N, H, 100, flags=lqro_mod.LQRO_FLAG_RECORDS | lqro_mod.LQRO_FLAG_QHULL_ORDER,
                                             **lqro_mod.shard_rows(N, g, world, mode)))
        c.set_gains(gains["A"], gains["B"], gains["L"], gains["E"])
        ctxs.append(c)
    try:
        for t in range(steps):
            tabs = [torch.zeros((N, 4), dtype=torch.float64, device=dev) for _ in range(world)]
            newv = [torch.zeros((N, 3), dtype=torch.float64, device=dev) for _ in range(world)]
            for g, c in enumerate(ctxs):
                c.step_device_begin(d_x.data_ptr(), d_vg.data_ptr(), tabs[g].data_ptr(), 0)
            torch.cuda.synchronize()
            whole = torch.zeros((N, 4), dtype=torch.float64, device=dev)
            for g in range(world):   # the all-gather: each rank's own rows
                ids = torch.from_numpy(lqro_mod.shard_row_ids(N, g, world, mode).astype(np.int64)).to(dev)
                whole[ids] = tabs[g][ids]
            for g, c in enumerate(ctxs):
                c.step_device_end(whole.data_ptr(), newv[g].data_ptr(), 0)
            torch.cuda.synchronize()
            v_ref, r_ref, carry_ref = ref[t]
            for g, c in enumerate(ctxs):
                ids = lqro_mod.shard_row_ids(N, g, world, mode)
                got = newv[g].cpu().numpy()[ids]
                assert np.array_equal(got.view(np.uint64), v_ref[ids].view(np.uint64)), (t, g)
                rr = c.records().reshape(len(ids), N - 1)
                want = r_ref.reshape(N, N - 1)[ids]
                for f in ("flags", "facet", "dist", "normal", "plane_point", "plane_normal"):
                    assert np.array_equal(rr[f], want[f]), (t, g, f)
                assert np.array_equal(c.carry_normal(), carry_ref), (t, g)
    finally:
        for c in ctxs:
            c.close()


def test_begin_end_call_order(lqro_mod, gains):
    import torch
    N, H = 8, 20
    x, vg = lqro_mod.synthetic_swarm(N)
    c = lqro_mod.Context(lqro_mod.config(N, H, 50))
    c.set_gains(gains["A"], gains["B"], gains["L"], gains["E"])
    dev = torch.device("cuda", 0)
    d_x, d_vg = torch.from_numpy(x).to(dev), torch.from_numpy(vg).to(dev)
    tab = torch.zeros((N, 4), dtype=torch.float64, device=dev)
    nv = torch.zeros((N, 3), dtype=torch.float64, device=dev)
    try:
        with pytest.raises(RuntimeError):
            c.step_device_end(tab.data_ptr(), nv.data_ptr(), 0)      # no begin
        c.step_device_begin(d_x.data_ptr(), d_vg.data_ptr(), tab.data_ptr(), 0)
        with pytest.raises(RuntimeError):
            c.step_device(d_x.data_ptr(), d_vg.data_ptr(), nv.data_ptr(), 0)   # a step in the middle
        c.step_device_end(tab.data_ptr(), nv.data_ptr(), 0)
        torch.cuda.synchronize()
        assert np.array_equal(nv.cpu().numpy().view(np.uint64), c.step(x, vg).view(np.uint64))
    finally:
        c.close()
