"""The C++ multi-rank host (include/lqro_sharded.hpp): lqro_step_device,
lqro_dynamics_step_device and one ncclAllGather of x per iteration of the
reference's agent loop (LQRObstacles.cpp:1391-1446), compiled with hipcc
against liblqro.so and RCCL (tests/cpp/lqro_sharded_main.cpp,
__graft_entry__.build_cpp_sharded).  On the GPU a world-size-1 communicator
must replay lqro::Simulator's trajectory bit for bit (newV and x, every
step), and so must G = 2, 3 ranks in one process (threads on one GPU, the
exchange in-process since RCCL takes one rank per GPU) through the world > 1
path: lqro_step_device_begin, the row-normal table exchange,
lqro_step_device_end, the dynamics, the exchange of x — with uneven row
blocks.  The Python multi-rank path is covered by tests/test_distributed.py
(gloo, CPU) and tests/test_gpu_0_multirank.py.  On the CPU the binary must
link and fail loudly (no gfx950 device) before RCCL is touched."""
import os
import subprocess

import numpy as np
import pytest

from conftest import ROOT

BIN = os.path.join(ROOT, "tests", "cpp", "lqro_sharded_main")


@pytest.fixture(scope="module")
def sharded(lqro_mod):
    if not os.path.exists(BIN):
        import __graft_entry__ as ge
        ge.build_cpp_sharded()
    return BIN


def _write_input(path, x, vg, pg, H, NP, steps, seed):
    N = x.shape[0]
    with open(path, "wb") as f:
        np.array([N, H, NP, steps], np.int32).tofile(f)
        np.array([seed], np.uint32).tofile(f)
        for a in (x, vg, pg):
            np.ascontiguousarray(a, np.float64).tofile(f)


def test_sharded_host_links_and_fails_loudly_without_gpu(sharded, tmp_path):
    import torch
    if torch.cuda.device_count() > 0:
        pytest.skip("a GPU is present (the -m gpu test covers the run)")
    _write_input(tmp_path / "in.bin", np.zeros((4, 16)), np.zeros((4, 3)), np.zeros((4, 3)), 10, 20, 1, 1)
    r = subprocess.run([sharded, str(tmp_path / "in.bin"), str(tmp_path / "out.bin")], capture_output=True,
                       text=True, timeout=60)
    assert r.returncode == 1 and "no gfx950 device" in r.stderr, r.stderr


@pytest.mark.gpu
@pytest.mark.parametrize("world", [1, 2, 3])
def test_sharded_host_matches_simulator(sharded, lqro_mod, tmp_path, world):
    # 97 agents: blocks of 48/49 (G = 2) and 32/32/33 (G = 3); a dense box so
    # inside-hull pairs (and facet-0 normals carried across shards) occur
    N, H, NP, steps, seed = 97, 45, 100, 3, 11
    x, vg = lqro_mod.synthetic_swarm(N, box=6.0, seed=11)
    pg = -x[:, :3]
    _write_input(tmp_path / "in.bin", x, vg, pg, H, NP, steps, seed)
    args = [sharded, str(tmp_path / "in.bin"), str(tmp_path / "out.bin")] + ([str(world)] if world > 1 else [])
    r = subprocess.run(args, capture_output=True, text=True, timeout=180)
    assert r.returncode == 0, r.stderr
    out = np.fromfile(tmp_path / "out.bin", np.float64).reshape(steps, 2, N * 19)
    for t in range(steps):
        a, b = out[t, 0], out[t, 1]
        assert np.array_equal(a.view(np.uint64), b.view(np.uint64)), f"step {t}: max |d| {np.abs(a - b).max()}"
        assert np.all(np.isfinite(a))
