#!/usr/bin/env python3
"""Per-kernel SQ / GRBM counters collected by tools/pmc_sq.sh, raw means and derived issue figures.

    python3 tools/pmc_sq.py gpurun_out/pmcsq/<TAG> [WORKLOAD]

Prints one line per kernel.  With WORKLOAD (c3, c4, c5, n8, ...) also writes
profiles/<TAG>_sq.csv and the workload's entry of profiles/pmc_sq.json, which bench.py reads into
its roofline block.  Derived figures (MI355X_MICROARCH.md: SQ_* wave counters count quad-cycles,
GRBM_GUI_ACTIVE is summed over the 8 XCDs; 256 CUs, 1 024 SIMDs):
  kernel_cycles  = GRBM_GUI_ACTIVE / 8
  valu_busy      = 4 * SQ_ACTIVE_INST_VALU / (1024 * kernel_cycles)   (share of SIMD cycles issuing VALU)
  waves_per_cu   = 4 * SQ_WAVE_CYCLES / (256 * kernel_cycles)         (mean resident waves per CU)
  wait_frac      = SQ_WAIT_ANY / SQ_WAVE_CYCLES         (waves parked on s_waitcnt / barriers)
  stall_frac     = SQ_WAIT_INST_ANY / SQ_WAVE_CYCLES    (waves ready but not issued)
  active_frac    = SQ_ACTIVE_INST_ANY / SQ_WAVE_CYCLES  (waves issuing)
  *_per_wave     = SQ_INSTS_* / SQ_WAVES
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def short(name):
    return name.split("(")[0].replace("void ", "").split("<")[0].strip()


def derived(c):
    g = c.get("GRBM_GUI_ACTIVE")
    out = {}
    if g:
        cyc = g / 8.0
        out["kernel_cycles"] = cyc
        if "SQ_ACTIVE_INST_VALU" in c:
            out["valu_busy"] = 4.0 * c["SQ_ACTIVE_INST_VALU"] / (1024.0 * cyc)
        if "SQ_WAVE_CYCLES" in c:
            out["waves_per_cu"] = 4.0 * c["SQ_WAVE_CYCLES"] / (256.0 * cyc)
    wc = c.get("SQ_WAVE_CYCLES")
    if wc:
        for k, src in (("wait_frac", "SQ_WAIT_ANY"), ("stall_frac", "SQ_WAIT_INST_ANY"),
                       ("active_frac", "SQ_ACTIVE_INST_ANY")):
            if src in c:
                out[k] = c[src] / wc
    w = c.get("SQ_WAVES")
    if w:
        for k in ("VALU", "SALU", "LDS", "VMEM_RD", "VMEM_WR"):
            if "SQ_INSTS_" + k in c:
                out[k.lower() + "_per_wave"] = c["SQ_INSTS_" + k] / w
    return out


def main():
    src = sys.argv[1]
    workload = sys.argv[2] if len(sys.argv) > 2 else None
    vals = defaultdict(lambda: defaultdict(list))
    for f in glob.glob(os.path.join(src, "**", "*counter_collection.csv"), recursive=True):
        with open(f) as fh:
            for row in csv.DictReader(fh):
                vals[short(row["Kernel_Name"])][row["Counter_Name"]].append(float(row["Counter_Value"]))
    table = {}
    for k in sorted(vals):
        if not k.startswith("k_"):
            continue
        c = {n: sum(v) / len(v) for n, v in vals[k].items()}
        dv = derived(c)
        table[k] = {"counters": c, "derived": dv}
        print(k, " ".join("%s=%.3g" % kv for kv in sorted(dv.items())))
    if not workload:
        return
    tag = os.path.basename(os.path.normpath(src))
    prof = os.path.join(ROOT, "profiles")
    names = sorted({n for t in table.values() for n in t["counters"]})
    dnames = sorted({n for t in table.values() for n in t["derived"]})
    with open(os.path.join(prof, "%s_sq.csv" % tag), "w", newline="") as fh:
        w = csv.writer(fh)
        w.writerow(["kernel"] + names + dnames)
        for k, t in sorted(table.items()):
            w.writerow([k] + [t["counters"].get(n, "") for n in names] + [t["derived"].get(n, "") for n in dnames])
    path = os.path.join(prof, "pmc_sq.json")
    doc = {"workloads": {}}
    if os.path.exists(path):
        with open(path) as fh:
            doc = json.load(fh)
    doc["_source"] = "rocprofv3 --pmc, one SQ/GRBM group per pass (tools/pmc_sq.sh), bench.py --no-graph"
    doc["_derived"] = __doc__.split("Derived figures")[1].strip()
    doc["workloads"][workload] = {"profile": tag, "kernels": {k: t["derived"] for k, t in table.items()}}
    with open(path, "w") as fh:
        json.dump(doc, fh, indent=1, sort_keys=True)


if __name__ == "__main__":
    main()
