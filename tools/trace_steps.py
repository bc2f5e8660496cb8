#!/usr/bin/env python3
"""Per-step kernel timeline from a rocprofv3 --kernel-trace CSV (diagnostic): for the last K steps of
a bench run, each kernel's start / end relative to the step's first kernel, and the mean over steps.
    python tools/trace_steps.py <dir with *kernel_trace.csv> [first_kernel_name] [K]"""
import csv
import glob
import os
import sys
from collections import defaultdict


def short(n):
    return n.split("(")[0].replace("void ", "").split("<")[0].strip()


def main():
    src = sys.argv[1]
    first = sys.argv[2] if len(sys.argv) > 2 else "k_gen_actions_ctr"
    K = int(sys.argv[3]) if len(sys.argv) > 3 else 20
    rows = []
    for f in glob.glob(os.path.join(src, "**", "*kernel_trace.csv"), recursive=True):
        with open(f) as fh:
            for r in csv.DictReader(fh):
                rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), short(r["Kernel_Name"])))
    rows.sort()
    steps, cur = [], None
    for st, en, nm in rows:
        if nm == first:
            cur = []
            steps.append(cur)
        if cur is not None:
            cur.append((st, en, nm))
    steps = [s for s in steps if len(s) > 1][-K - 1:-1]
    acc = defaultdict(list)
    spans = []
    for s in steps:
        t0 = s[0][0]
        seen = defaultdict(int)
        for st, en, nm in s:
            k = "%s#%d" % (nm, seen[nm])
            seen[nm] += 1
            acc[k].append(((st - t0) / 1e3, (en - t0) / 1e3))
        spans.append((max(e for _, e, _ in s) - t0) / 1e3)
    for k, v in sorted(acc.items(), key=lambda kv: sum(a for a, _ in kv[1]) / len(kv[1])):
        a = sum(x for x, _ in v) / len(v)
        b = sum(y for _, y in v) / len(v)
        print("%-28s start %8.1f  end %8.1f  dur %7.1f us" % (k, a, b, b - a))
    if spans:
        print("step span (first start -> last end) mean %.1f us over %d steps" % (sum(spans) / len(spans), len(spans)))
        starts = [s[0][0] for s in steps]
        if len(starts) > 1:
            print("step period mean %.1f us" % ((starts[-1] - starts[0]) / 1e3 / (len(starts) - 1)))


if __name__ == "__main__":
    main()
