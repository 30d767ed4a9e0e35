"""Seeded agent states for the dynamics/estimation step tests (test data
only): positions, velocities, body rates and rotor forces around hover,
attitudes from random axis-angle rotations, covariances SPD around Pinit."""
from __future__ import annotations

import numpy as np

HOVER = 9.80665 * 0.5 / 4   # nominalInput (LQRO:188)


def rotation(axis_angle: np.ndarray) -> np.ndarray:
    th = float(np.linalg.norm(axis_angle))
    if th == 0.0:
        return np.eye(3)
    k = axis_angle / th
    K = np.array([[0, -k[2], k[1]], [k[2], 0, -k[0]], [-k[1], k[0], 0]])
    return np.eye(3) + np.sin(th) * K + (1 - np.cos(th)) * (K @ K)


def random_agent_cases(n: int, seed: int, rot_err: bool = True) -> dict:
    rng = np.random.default_rng(seed)
    x = np.zeros((n, 16))
    x[:, 0:3] = rng.uniform(-3, 3, (n, 3))
    x[:, 3:6] = rng.uniform(-1, 1, (n, 3))
    if rot_err:   # nonzero only between a propagate and its reset; exercised anyway
        x[: n // 2, 6:9] = rng.uniform(-0.02, 0.02, (n // 2, 3))
    x[:, 9:12] = rng.uniform(-0.5, 0.5, (n, 3))
    x[:, 12:16] = HOVER + rng.uniform(-0.1, 0.1, (n, 4))
    rot = np.stack([rotation(rng.normal(size=3) * rng.uniform(0, 0.4)) for _ in range(n)])
    rot[0] = np.eye(3)   # the sinangle == 0 branch of both controllers
    B = rng.normal(size=(n, 16, 16))
    P = 1e-9 * np.eye(16) + 1e-10 * np.einsum("nij,nkj->nik", B, B)
    vgoal = rng.uniform(-1, 1, (n, 3))
    p_goal = rng.uniform(-3, 3, (n, 3))
    u_goal = np.full((n, 4), HOVER)
    z = np.concatenate([x[:, 9:12], x[:, 0:3]], axis=1) + 3e-5 * rng.normal(size=(n, 6))
    return dict(x=x, rot=rot, P=P, vgoal=vgoal, p_goal=p_goal, u_goal=u_goal, z=z)


def trajectory_start(n: int, seed: int) -> dict:
    """States as they stand at a step boundary (rotation error reset to 0)."""
    cs = random_agent_cases(n, seed, rot_err=False)
    return cs


def quat_cases() -> np.ndarray:
    """Rotations for quatFromRot: random ones, the identity, half turns about
    each axis and near-half turns (where 1 + trace terms reach 0 and the
    std::max(., 0) clamp and the sign tests matter)."""
    rng = np.random.default_rng(0x5154)
    rs = [rotation(rng.normal(size=3) * rng.uniform(0, 3.1)) for _ in range(40)]
    rs.append(np.eye(3))
    for ax in np.eye(3):
        rs.append(rotation(ax * np.pi))
        rs.append(rotation(ax * (np.pi - 1e-9)))
        rs.append(rotation(-ax * (np.pi - 1e-9)))
    rs.append(rotation(np.array([1.0, 1.0, 0.0]) / np.sqrt(2) * np.pi))
    return np.stack(rs)
