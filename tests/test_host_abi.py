"""The C-ABI library on the CPU: it loads, exports every entry point
include/lqro.h declares, and its host-side code (setup-time gain synthesis,
createSpheres) is bit-exact against the reference's golden outputs.  No
compute call reaches a GPU here; without one, lqro_create must fail loudly
(LQRO_E_NODEVICE) — there is no CPU fallback."""
import ctypes as C
import os
import re

import numpy as np
import pytest

from conftest import GOLDEN, ROOT


def _header_functions():
    src = open(os.path.join(ROOT, "include", "lqro.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(lqro_[a-z0-9_]+)\s*\(", src)))


def test_exports_every_header_symbol(lqro_mod):
    names = _header_functions()
    assert len(names) >= 15
    L = lqro_mod.lib()
    for n in names:
        assert hasattr(L, n), n
    assert sorted(lqro_mod.EXPORTS) == names


def test_lib_is_gfx950_code_object(lqro_mod):
    """The shared object carries a gfx950 HIP fat binary."""
    blob = open(lqro_mod.LIB_PATH, "rb").read()
    assert b"gfx950" in blob
    assert b"__hip_fatbin" in blob or b".hip_fatbin" in blob


def test_version_and_status_strings(lqro_mod):
    L = lqro_mod.lib()
    assert L.lqro_version() >= 1
    for rc in (0, -1, -2, -3, -4, -5, -6, -7, -8, -9):
        s = L.lqro_status_string(rc)
        assert s and len(s) >= 2 and s != b"unknown", rc
    assert b"merge" in L.lqro_status_string(lqro_mod.LQRO_E_QHMERGE)


def test_config_default(lqro_mod):
    c = lqro_mod.Config()
    lqro_mod.lib().lqro_config_default(C.byref(c), 1024, 100, 100)
    assert (c.n_agents, c.x_dim, c.u_dim, c.horizon, c.n_points, c.min_reach) == \
        (1024, 16, 4, 100, 100, 4)                                     # LQRO:9-14, 1409
    assert (c.xy_radius, c.z_radius, c.vmax_reach, c.vmax_lp) == (0.26, 0.75, 30.0, 100.0)


def test_host_gains_bit_exact(lqro_mod):
    """lqro_synthesize_gains (host C++ in liblqro.so) == the reference's
    controlMatrices, bit for bit."""
    ref = np.load(os.path.join(GOLDEN, "gains.npz"))
    got = lqro_mod.synthesize_gains()
    for k in ("A", "B", "c", "L", "E", "Lh", "Eh"):
        assert np.array_equal(got[k].view(np.uint64), ref[k].view(np.uint64)), k



def test_host_reduced_model_gains_bit_exact(lqro_mod, oracle):
    """lqro_synthesize_gains_x(x_dim = 12), config 5's reduced model (host
    C++), == the oracle's restatement, for the default and a perturbed model;
    x_dim = 16 is the reference's synthesis."""
    for m in (lqro_mod.default_model(), lqro_mod.perturbed_models(3)[2]):
        om = oracle.Model(*[getattr(m, f) for f, _ in m._fields_])
        for X in (12, 16):
            got = lqro_mod.synthesize_gains(m, x_dim=X)
            ref = oracle.synthesize(om, x_dim=X)
            for k in ref:
                assert got[k].shape == ref[k].shape
                assert np.array_equal(got[k].view(np.uint64), ref[k].view(np.uint64)), (X, k)
    with pytest.raises(lqro_mod.LqroError):
        lqro_mod.synthesize_gains(x_dim=13)
    with pytest.raises(ValueError):
        oracle.synthesize(x_dim=13)


@pytest.mark.parametrize("np_", [100, 50])
def test_host_sphere_bit_exact(lqro_mod, np_):
    ref = np.load(os.path.join(GOLDEN, "gains.npz"))[f"sphere{np_}"]
    got = lqro_mod.create_spheres(np_)
    assert np.array_equal(got.view(np.uint64), ref.view(np.uint64))


def test_bad_config_rejected(lqro_mod):
    L = lqro_mod.lib()
    h = C.c_void_p()
    bad = lqro_mod.config(1, 50, 100)              # one agent: no pairs
    assert L.lqro_create(C.byref(bad), C.byref(h)) == -1
    bad = lqro_mod.config(8, 0, 100)
    assert L.lqro_create(C.byref(bad), C.byref(h)) == -1
    bad = lqro_mod.config(8, 257, 100)             # horizon beyond the per-lane slice slots
    assert L.lqro_create(C.byref(bad), C.byref(h)) == -1
    bad = lqro_mod.config(8, 50, 257)              # points beyond the 4 reachable-mask words
    assert L.lqro_create(C.byref(bad), C.byref(h)) == -1
    assert L.lqro_create(None, C.byref(h)) == -1


def test_no_device_fails_loudly(lqro_mod):
    import torch
    if torch.cuda.is_available():
        pytest.skip("a GPU is present")
    with pytest.raises(lqro_mod.LqroError):
        lqro_mod.Context(lqro_mod.config(8, 50, 100))
    with pytest.raises(lqro_mod.LqroError):
        lqro_mod.calculate_new_v([np.zeros((1, 6), np.float32)], np.zeros((1, 3)))


def test_missing_library_raises(lqro_mod, monkeypatch):
    monkeypatch.setattr(lqro_mod, "_lib", None)
    monkeypatch.setattr(lqro_mod, "LIB_PATH", "/nonexistent/liblqro.so")
    with pytest.raises(RuntimeError):
        lqro_mod.lib()


def test_record_layout(lqro_mod, oracle):
    assert lqro_mod.RECORD_DTYPE == oracle.RECORD_DTYPE
    assert C.sizeof(lqro_mod.PairRecord) == 168


def test_row_shard_partition(lqro_mod):
    for n, w in ((1024, 8), (1000, 8), (64, 2), (9, 4), (4096, 8), (5, 5)):
        got = [lqro_mod.row_shard(n, r, w) for r in range(w)]
        assert got[0][0] == 0 and got[-1][1] == n
        assert all(a[1] == b[0] for a, b in zip(got, got[1:]))
        assert all(e > b for b, e in got)
    with pytest.raises(ValueError):
        lqro_mod.row_shard(3, 0, 4)


@pytest.mark.parametrize("mode", ["block", "cyclic"])
def test_shard_rows_partition(lqro_mod, mode):
    """Every agent's row belongs to exactly one rank, in either mode; the
    config fields are what the C-ABI reads (row_stride 0 = contiguous)."""
    for n, w in ((1024, 8), (1000, 8), (64, 2), (9, 4), (4096, 8), (5, 5), (7, 1)):
        ids = [lqro_mod.shard_row_ids(n, r, w, mode) for r in range(w)]
        assert np.array_equal(np.sort(np.concatenate(ids)), np.arange(n))
        assert max(len(i) for i in ids) - min(len(i) for i in ids) <= 1
        for r in range(w):
            f = lqro_mod.shard_rows(n, r, w, mode)
            cfg = lqro_mod.config(n, 10, 10, **f)
            assert cfg.row_stride == f["row_stride"]
    with pytest.raises(ValueError):
        lqro_mod.shard_rows(8, 0, 2, "striped")


def test_swarm_generator_is_stable(lqro_mod):
    """The synthetic swarm is part of the bench contract."""
    x, vg = lqro_mod.synthetic_swarm(4)
    assert x.shape == (4, 16) and vg.shape == (4, 3)
    assert np.all(np.abs(x[:, 3:6]) <= 1) and np.all(np.abs(vg) <= 1)
    assert np.all(x[:, 12:16] == 9.80665 * 0.5 / 4)
    side = 4.0 * 4 ** (1 / 3)
    assert np.all(np.abs(x[:, :3]) <= side / 2)
    x2, _ = lqro_mod.synthetic_swarm(4)
    assert np.array_equal(x, x2)


def test_small_pivot_routines(tmp_path):
    """lqro_synth.hpp's register-held pivoted routines (solve_sm, inverse_sm:
    N <= 4, used by k_dynw's per-lane 3x3 work without private memory) equal
    the indexed transcriptions of operator% / operator! (MAT:370-442,
    603-671) bit for bit, ties and singular matrices included
    (tests/cpp/small_pivot_check.cpp, host code)."""
    import subprocess
    exe = str(tmp_path / "spc")
    src = os.path.join(ROOT, "tests", "cpp", "small_pivot_check.cpp")
    subprocess.run(["/opt/rocm/bin/hipcc", "-std=c++17", "-O2", "-ffp-contract=off", "-fno-fast-math", "-x", "hip",
                    "--offload-arch=gfx950", src, "-o", exe], check=True, capture_output=True, timeout=300)
    r = subprocess.run([exe], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0 and r.stdout.startswith("ok"), r.stdout + r.stderr
