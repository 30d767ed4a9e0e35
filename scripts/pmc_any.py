#!/usr/bin/env python3
"""Per-kernel (name, grid) means of every counter in rocprofv3 --pmc CSV dirs.

  python3 scripts/pmc_any.py OUT.json DIR [DIR ...]

Each DIR is one `rocprofv3 --pmc ... --output-format csv -d DIR` pass; the
output maps "kernel grid" to {counter: mean per launch, launches: n}.
"""
import collections
import csv
import glob
import json
import os
import re
import sys


def main():
    out, dirs = sys.argv[1], sys.argv[2:]
    acc = collections.defaultdict(lambda: collections.defaultdict(list))
    for d in dirs:
        for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            for r in csv.DictReader(open(f)):
                m = re.search(r"(k_[a-z_0-9]+)", r["Kernel_Name"])
                key = "%s %s" % (m.group(1) if m else r["Kernel_Name"][:40], r["Grid_Size"])
                acc[key][r["Counter_Name"]].append(float(r["Counter_Value"]))
    res = {}
    for k, cs in acc.items():
        res[k] = {c: sum(v) / len(v) for c, v in cs.items()}
        res[k]["launches"] = max(len(v) for v in cs.values())
    with open(out, "w") as fh:
        json.dump(res, fh, indent=1, sort_keys=True)
    for k in sorted(res):
        if "qhull" in k or "pair" in k:
            print(k, {c: round(v) for c, v in res[k].items()})


if __name__ == "__main__":
    main()
