#!/usr/bin/env python3
"""Per-kernel mean of every counter collected by tools/pmc_sq.sh (one row per kernel)."""
import csv
import glob
import os
import sys
from collections import defaultdict


def short(name):
    return name.split("(")[0].replace("void ", "").strip()


def main():
    src = sys.argv[1]
    vals = defaultdict(lambda: defaultdict(list))
    for f in glob.glob(os.path.join(src, "**", "*counter_collection.csv"), recursive=True):
        with open(f) as fh:
            for row in csv.DictReader(fh):
                vals[short(row["Kernel_Name"])][row["Counter_Name"]].append(float(row["Counter_Value"]))
    for k in sorted(vals):
        if not k.startswith("k_"):
            continue
        cs = vals[k]
        print(k, " ".join("%s=%.4g" % (c, sum(v) / len(v)) for c, v in sorted(cs.items())))


if __name__ == "__main__":
    main()
