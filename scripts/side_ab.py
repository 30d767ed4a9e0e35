"""Step time vs number of CUs running k_hull beside k_pair (LQRO_SIDE_HULL_CUS)."""
import os, subprocess, sys
here = os.path.dirname(os.path.abspath(__file__))
for side in sys.argv[1:] or ["0", "16", "32", "64"]:
    env = dict(os.environ, LQRO_SIDE_HULL_CUS=side)
    out = subprocess.run([sys.executable, os.path.join(here, "..", "bench.py"), "--no-cpu-baseline",
                          "--steps", "6", "--warmup", "2"], env=env, capture_output=True, text=True)
    import json
    try:
        d = json.loads(out.stdout.strip().splitlines()[-1])
        print(side, round(d["ms_per_step"], 2), round(d["roofline"]["kernel_ms"], 2), flush=True)
    except Exception:
        print(side, "failed", out.stderr[-500:], flush=True)
