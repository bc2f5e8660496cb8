#!/usr/bin/env python3
"""Reduce tools/profile.sh output to the files committed under profiles/.

    python3 tools/pmc_summary.py gpurun_out/prof r01 [PRESET ENVS]

Writes
  profiles/<tag>_kernel_stats.csv   rocprofv3 --kernel-trace --stats summary (as produced)
  profiles/<tag>_pmc_per_kernel.csv per-kernel mean FETCH_SIZE / WRITE_SIZE per dispatch
  profiles/pmc_traffic.json         HBM bytes per launch per kernel for bench.py preset PRESET
                                    (default c3) profiled at ENVS envs per GPU (default 65536);
                                    bench.py scales them to its own envs per GPU

Units and corrections (MI355X_MICROARCH.md, HBM section): rocprofv3 reports FETCH_SIZE and
WRITE_SIZE in KiB; on gfx950 FETCH_SIZE counts 64 B per 128-B request, i.e. half the bytes
of wide coalesced reads, so it is doubled.  WRITE_SIZE is taken as is.  Other access widths
are uncalibrated: the raw values are kept next to the corrected ones.
"""
import csv
import glob
import json
import os
import shutil
import sys
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def short(name):
    n = name.split("(")[0]
    n = n.replace("void ", "")
    return n.split("<")[0].strip()


def counters(d, counter):
    vals = defaultdict(list)
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        with open(f) as fh:
            for row in csv.DictReader(fh):
                if row.get("Counter_Name") != counter:
                    continue
                vals[short(row["Kernel_Name"])].append(float(row["Counter_Value"]))
    return vals


def main():
    src, tag = sys.argv[1], sys.argv[2]
    preset = sys.argv[3] if len(sys.argv) > 3 else "c3"
    envs = int(sys.argv[4]) if len(sys.argv) > 4 else 65536
    prof = os.path.join(ROOT, "profiles")
    os.makedirs(prof, exist_ok=True)
    stats = glob.glob(os.path.join(src, "kt", "**", "*kernel_stats.csv"), recursive=True)
    if stats:
        shutil.copy(stats[0], os.path.join(prof, "%s_kernel_stats.csv" % tag))
    fetch = counters(os.path.join(src, "FETCH_SIZE"), "FETCH_SIZE")
    write = counters(os.path.join(src, "WRITE_SIZE"), "WRITE_SIZE")
    out = {}
    rows = []
    for k in sorted(set(fetch) | set(write)):
        f = fetch.get(k, [])
        w = write.get(k, [])
        fr = 1024.0 * sum(f) / len(f) if f else None
        wr = 1024.0 * sum(w) / len(w) if w else None
        fc = 2 * fr if fr is not None else None
        hbm = (fc or 0.0) + (wr or 0.0) if (fc is not None or wr is not None) else None
        out[k] = {"launches": max(len(f), len(w)), "fetch_bytes_raw": fr, "fetch_bytes_corrected": fc,
                  "write_bytes": wr, "hbm_bytes_per_launch": hbm}
        rows.append([k, max(len(f), len(w)), fr, fc, wr, hbm])
    with open(os.path.join(prof, "%s_pmc_per_kernel.csv" % tag), "w", newline="") as fh:
        wtr = csv.writer(fh)
        wtr.writerow(["kernel", "launches", "fetch_bytes_raw", "fetch_bytes_x2", "write_bytes", "hbm_bytes"])
        wtr.writerows(rows)
    path = os.path.join(prof, "pmc_traffic.json")
    doc = {}
    if os.path.exists(path):
        with open(path) as fh:
            doc = json.load(fh)
    if "workloads" not in doc:
        doc = {"workloads": {}}
    doc["_units"] = "bytes per launch; fetch_corrected = 2 x FETCH_SIZE (gfx950), hbm = fetch_corrected + write"
    doc["_source"] = "rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE, separate passes, tools/profile.sh"
    doc["workloads"][preset] = {"envs_per_gpu": envs, "profile": tag, "kernels": out}
    with open(path, "w") as fh:
        json.dump(doc, fh, indent=1, sort_keys=True)
    for r in rows:
        print("%-16s n=%4d fetch %12.0f (x2 %12.0f) write %12.0f" % (r[0], r[1], r[2] or 0, r[3] or 0, r[4] or 0))


if __name__ == "__main__":
    main()
