"""The multi-rank HIP path on one GPU: 2 gloo ranks share
cuda:0, each owns a block of rows (or every other row: cyclic sharding) with its own liblqro context and runs the
device-resident closed loop (lqro.DeviceLoop: lqro_step_device ->
lqro_dynamics_step_device on its rows -> all-gather of x) on torch's default
stream with NO device synchronisation between the calls.  The gathered x and
the own rows' newV must equal a single-context run bit for bit — this checks
that the exchange is ordered against the kernels that produce its input
(stream semantics of lqro_step_device)."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu

N, H, NP, ITERS = 48, 30, 50, 3


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _run(lqro, x0, vg0, g, rank=0, world=1, dist=None, mode="block"):
    import torch
    loop = lqro.DeviceLoop(x0, vg0, g, H, NP, p_goal=-x0[:, :3], rank=rank, world=world, dist=dist, seed=11,
                           rows=mode)
    newv = []
    for _ in range(ITERS):
        loop.step()
        newv.append(loop.own_rows(loop.newv).clone())
        loop.update()
    torch.cuda.synchronize()
    out = loop.x.cpu().numpy(), torch.stack(newv).cpu().numpy(), loop.ids_h
    loop.close()
    return out


def _worker(rank, world, port, out_path, mode):
    import sys
    import torch
    import torch.distributed as dist
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, os.path.join(root, "lqr-obstacles_amd"))
    import lqro
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    x0, vg0 = lqro.synthetic_swarm(N, seed=77, box=5.0)
    g = lqro.synthesize_gains()
    x, nv, ids = _run(lqro, x0, vg0, g, rank, world, dist, mode)
    np.savez(f"{out_path}.{rank}.npz", x=x, newv=nv, rows=ids)
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("mode", ["block", "cyclic"])
def test_two_ranks_closed_loop_match_single_context(tmp_path, lqro_mod, mode):
    world = 2
    out = str(tmp_path / "loop")
    mp.spawn(_worker, args=(world, _free_port(), out, mode), nprocs=world, join=True)
    x0, vg0 = lqro_mod.synthetic_swarm(N, seed=77, box=5.0)
    g = lqro_mod.synthesize_gains()
    x_ref, nv_ref, _ = _run(lqro_mod, x0, vg0, g)
    assert not np.array_equal(x_ref, x0), "the loop did not move the agents"
    for r in range(world):
        d = np.load(f"{out}.{r}.npz")
        ids = d["rows"]
        assert np.array_equal(ids, lqro_mod.shard_row_ids(N, r, world, mode))
        assert np.array_equal(d["x"].view(np.uint64), x_ref.view(np.uint64)), f"rank {r}: gathered x"
        assert np.array_equal(d["newv"].view(np.uint64), nv_ref[:, ids].view(np.uint64)), f"rank {r}: newV"
