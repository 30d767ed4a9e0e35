"""The multi-rank path on the CPU (gloo, world_size 2): rows sharded with
lqro.shard_rows (contiguous blocks, or cyclic: row_stride = world), each rank computes its rows, one all-gather
(lqro.allgather_rows) assembles newV on every rank; the result equals the
single-process step.  The per-rank compute here is the oracle (no GPU in this
container); the GPU ranks run the same sharding/gather code in bench.py."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, N, H, NP, out_path, mode):
    import sys
    import torch
    import torch.distributed as dist
    here = os.path.dirname(os.path.abspath(__file__))
    root = os.path.dirname(here)
    sys.path[:0] = [os.path.join(root, "lqr-obstacles_amd"), os.path.join(root, "oracle")]
    import lqro
    import pyoracle
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    x, vg = lqro.synthetic_swarm(N, seed=21)
    g = pyoracle.synthesize()
    T, NCF = pyoracle.tables(g["A"], g["B"], g["L"], g["E"], H)
    S = pyoracle.sphere(NP)
    full = torch.zeros((N, 3), dtype=torch.float64)
    for i in lqro.shard_row_ids(N, rank, world, mode):
        newv, _ = pyoracle.step(T, NCF, S, x, vg, rows=(int(i), int(i) + 1), records=False)
        full[i] = torch.from_numpy(newv[i])
    lqro.allgather_rows(dist, full, rank, world, mode=mode)
    np.save(f"{out_path}.{rank}.npy", full.numpy())
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("mode", ["block", "cyclic"])
@pytest.mark.parametrize("N", [12, 13])
def test_gloo_two_ranks_match_single(tmp_path, N, mode):
    world, H, NP = 2, 20, 40
    out = str(tmp_path / "newv")
    mp.spawn(_worker, args=(world, _free_port(), N, H, NP, out, mode), nprocs=world, join=True)
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    sys.path[:0] = [os.path.join(os.path.dirname(here), "lqr-obstacles_amd")]
    import lqro
    import pyoracle
    x, vg = lqro.synthetic_swarm(N, seed=21)
    g = pyoracle.synthesize()
    T, NCF = pyoracle.tables(g["A"], g["B"], g["L"], g["E"], H)
    ref, _ = pyoracle.step(T, NCF, pyoracle.sphere(NP), x, vg, records=False)
    for r in range(world):
        got = np.load(f"{out}.{r}.npy")
        assert np.array_equal(got, ref), r
