import sys, os, time
sys.path[:0] = ["lqr-obstacles_amd", "tests", "oracle"]
import numpy as np, lqro, pyoracle as po
from lp_cases import random_cases
for seed, mp in [(1, 60), (2, 200), (3, 1100)]:
    cases, goals = random_cases(300 if mp < 500 else 60, seed=seed, max_planes=mp)
    t = time.time()
    got = lqro.calculate_new_v(cases, goals)
    ref = np.array([po.newv(c, g) for c, g in zip(cases, goals)])
    print(seed, mp, "time %.2f" % (time.time() - t), "bad", int((~np.all(got == ref, axis=1)).sum()), flush=True)
