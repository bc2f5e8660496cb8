#!/bin/bash
# Instruction-cache counters per kernel of one bench command (one rocprofv3 pass, under its own time
# limit).  Usage: tools/pmc_icache.sh TAG [bench args...]; per-kernel sums in gpurun_out/pmcic/TAG/summary.txt
cd "$(dirname "$0")/.." || exit 2
ROOT=$PWD
cd /tmp && export TMPDIR=/tmp && cd "$ROOT" || exit 2
TAG=$1; shift
OUT=$ROOT/gpurun_out/pmcic/$TAG
mkdir -p "$OUT"
timeout -s KILL 120 rocprofv3 --pmc SQC_ICACHE_REQ SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQ_IFETCH SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU \
    -T --output-format csv -d "$OUT/p" -o run -- python3 bench.py "$@" > "$OUT/p.log" 2>&1 || { echo "pmc pass failed"; tail -5 "$OUT/p.log"; exit 1; }
python3 - "$OUT" <<'PY' > "$OUT/summary.txt"
import csv, glob, os, sys
from collections import defaultdict
acc = defaultdict(lambda: defaultdict(float)); n = defaultdict(set)
for f in glob.glob(os.path.join(sys.argv[1], "p", "**", "*counter_collection.csv"), recursive=True):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].split("(")[0].replace("void ", "").split("<")[0].strip()
        acc[k][r["Counter_Name"]] += float(r["Counter_Value"])
        n[k].add(r.get("Dispatch_Id", r.get("Correlation_Id", "")))
for k in sorted(acc, key=lambda k: -acc[k].get("SQ_INSTS_VALU", 0)):
    a = acc[k]; req = a.get("SQC_ICACHE_REQ", 0) or 1
    print("%-22s launches %4d  icache req %12.0f hits %12.0f misses %10.0f (%.4f of req) dup %10.0f  ifetch %12.0f  waves %9.0f  valu %13.0f salu %12.0f" % (
        k, len(n[k]), a.get("SQC_ICACHE_REQ", 0), a.get("SQC_ICACHE_HITS", 0), a.get("SQC_ICACHE_MISSES", 0),
        a.get("SQC_ICACHE_MISSES", 0) / req, a.get("SQC_ICACHE_MISSES_DUPLICATE", 0), a.get("SQ_IFETCH", 0),
        a.get("SQ_WAVES", 0), a.get("SQ_INSTS_VALU", 0), a.get("SQ_INSTS_SALU", 0)))
PY
cat "$OUT/summary.txt"
