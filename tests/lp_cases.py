"""Random plane sets for the new-velocity LP (shared by CPU and GPU tests)."""
import numpy as np


def random_cases(n_cases: int, seed: int = 1, max_planes: int = 60):
    """Mix of feasible and infeasible sets so that linearProgram4 runs."""
    rng = np.random.default_rng(seed)
    cases, goals = [], []
    for t in range(n_cases):
        m = int(rng.integers(0, max_planes))
        nrm = rng.normal(size=(m, 3))
        nrm /= np.linalg.norm(nrm, axis=1, keepdims=True)
        kind = t % 3
        if kind == 0:     # half-planes through points near the origin: often infeasible
            pts = rng.normal(size=(m, 3)) * rng.uniform(0.05, 2.0)
        elif kind == 1:   # LQR-obstacle-like: v_i - d n with moderate d
            pts = rng.normal(size=3) - rng.uniform(0.0, 3.0, size=(m, 1)) * nrm
        else:             # far planes: mostly feasible, exercises the speed sphere
            pts = -rng.uniform(10.0, 120.0, size=(m, 1)) * nrm
        cases.append(np.concatenate([pts, nrm], 1).astype(np.float32))
        goals.append(rng.normal(size=3) * rng.uniform(0.1, 150.0))
    return cases, np.array(goals)
