"""GJK's backup procedure (gjk.cpp:663-706) pinned to the reference: the C3
pairs whose GJK takes the backup (tests/golden/gjk_backup.npz, made by
make_golden_backup.py from the reference's own pair body and gjk_distance).
The oracle (CPU) and the GPU path must reproduce the reference bit for bit:
n_reach, the inside flag, GJK's squared distance and witnesses, and for an
outside pair the distance, normal and fp32 half-plane."""
import os

import numpy as np
import pytest

from conftest import GOLDEN

FIX = os.path.join(GOLDEN, "gjk_backup.npz")


def _check(rec, d, k):
    assert rec["n_reach"] == d["n_reach"][k]
    assert rec["flags"] & 4, "the backup procedure did not run"
    inside = bool(rec["flags"] & 2)
    assert inside == (d["status"][k] == 1)
    bits = lambda a: np.asarray(a, np.float64).view(np.uint64)  # noqa: E731
    assert np.array_equal(bits(rec["wpt_vrel"]), bits(d["gjk_wpt_vrel"][k]))
    assert np.array_equal(bits(rec["wpt_hull"]), bits(d["gjk_wpt_hull"][k]))
    if not inside:
        assert bits(rec["dist"]) == bits(d["dist"][k])
        assert np.array_equal(bits(rec["normal"]), bits(d["normal"][k]))
        pl = np.concatenate([rec["plane_point"], rec["plane_normal"]]).astype(np.float32)
        assert np.array_equal(pl.view(np.uint32), d["plane"][k].view(np.uint32))


def test_oracle_backup_pairs_match_reference(oracle, gains):
    d = np.load(FIX)
    H, NP = int(d["H"]), int(d["NP"])
    T, NCF = oracle.tables(gains["A"], gains["B"], gains["L"], gains["E"], H)
    S = oracle.sphere(NP)
    assert len(d["xi"]) >= 1
    for k in range(len(d["xi"])):
        rec = oracle.pair(T, NCF, S, d["xi"][k], d["xj"][k])
        _check(rec, d, k)
        # the squared distance GJK returned, through dist = sqrt(sqd) (LQRO:843)
        if d["status"][k] == 0:
            assert np.sqrt(d["gjk_sqd"][k]) == d["dist"][k]


@pytest.mark.gpu
def test_gpu_backup_pairs_match_reference(lqro_mod, gains):
    d = np.load(FIX)
    H, NP = int(d["H"]), int(d["NP"])
    for k in range(len(d["xi"])):
        x = np.stack([d["xi"][k], d["xj"][k]])
        ctx = lqro_mod.Context(lqro_mod.config(2, H, NP, flags=lqro_mod.LQRO_FLAG_RECORDS))
        ctx.set_gains(gains["A"], gains["B"], gains["L"], gains["E"])
        ctx.step(x, np.zeros((2, 3)))
        recs = ctx.records()
        ctx.close()
        _check(recs[0], d, k)
