#!/usr/bin/env python3
"""Per-launch SQ counters of one kernel from rocprofv3 --pmc passes of
bench.py (each pass a separate run; see scripts/gpu_profile.sh), plus the
executed-VALU figures they imply.

  pmc_sq.py OUT.json DIR [DIR ...] [--kernel k_pair]

For k_pair the full-grid launches (the LQRO_HOT=0 roofline probe) are kept,
as in pmc_traffic.py.  SQ_INSTS_VALU_*_F64 count wave instructions: executed
fp64 flops <= 64 x (2 FMA + ADD + MUL) per launch (inactive lanes counted).
SQ_WAVE_CYCLES / SQ_BUSY_CYCLES / SQ_WAIT_* / SQ_ACTIVE_INST_* are in
quad-cycles (MI355X_MICROARCH.md, PMC units)."""
import argparse
import collections
import csv
import glob
import json
import os
import re

from pmc_traffic import lib_stamp


def per_kernel(d, kernel):
    f = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)[0]
    acc = collections.defaultdict(lambda: collections.defaultdict(list))
    for r in csv.DictReader(open(f)):
        m = re.search(r"(k_[a-z0-9_]+)", r["Kernel_Name"])
        if not m or m.group(1) != kernel:
            continue
        acc[int(r["Grid_Size"])][r["Counter_Name"]].append(float(r["Counter_Value"]))
    if not acc:
        return {}, 0
    g = max(acc)
    return {c: sum(v) / len(v) for c, v in acc[g].items()}, g


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("out")
    ap.add_argument("dirs", nargs="+")
    ap.add_argument("--kernel", default="k_pair")
    ap.add_argument("--pairs", type=int, default=1024 * 1023)
    ap.add_argument("--kernel-ms", type=float, default=0.0, help="mean launch duration (kernel trace)")
    a = ap.parse_args()
    cnt, grid = {}, 0
    for d in a.dirs:
        c, g = per_kernel(d, a.kernel)
        cnt.update(c)
        grid = max(grid, g)
    out = {"kernel": a.kernel, "grid_size": grid, "counters_per_launch": cnt, "build": lib_stamp()}
    fma, add, mul = (cnt.get(f"SQ_INSTS_VALU_{k}_F64", 0.0) for k in ("FMA", "ADD", "MUL"))
    if fma or add or mul:
        fl = 64.0 * (2 * fma + add + mul)
        out["executed_fp64_flops_per_launch_upper"] = fl
        out["executed_fp64_flops_per_pair_upper"] = fl / a.pairs
        if a.kernel_ms > 0:
            out["executed_fp64_tflops_upper"] = fl / (a.kernel_ms * 1e-3) / 1e12
    wc = cnt.get("SQ_WAVE_CYCLES")
    if wc:
        for k in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_ACTIVE_INST_VALU"):
            if k in cnt:
                out[k.lower() + "_frac_of_wave_cycles"] = cnt[k] / wc
    with open(a.out, "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
