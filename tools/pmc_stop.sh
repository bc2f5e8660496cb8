#!/bin/bash
# Diagnostic: k_tick's instruction counts per wave with the tick ended after phase k (the ZS_DIAG_STOP builds
# of tools/diag_stop.sh) against the product, one rocprofv3 counter pass per build (own time limit).
# Usage: CFG=c5 tools/pmc_stop.sh TAG; per-wave counts in gpurun_out/pmcstop/TAG/summary.txt
cd "$(dirname "$0")/.." || exit 2
ROOT=$PWD
cd /tmp && export TMPDIR=/tmp && cd "$ROOT" || exit 2
TAG=$1
OUT=$ROOT/gpurun_out/pmcstop/$TAG
mkdir -p "$OUT"
for v in ${VARIANTS:-product stop1 stop2 stop3 stop5}; do
  lib=libzombsole_amd/_build/libzombsole_mi355x.so
  [ "$v" != product ] && lib=libzombsole_amd/_build/libzombsole_mi355x_$v.so
  timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR \
      -T --output-format csv -d "$OUT/$v" -o run -- python3 bench.py --config "${CFG:-c5}" --engine-lib "$lib" --no-graph \
      --steps 20 --warmup 5 --no-cpu-baseline > "$OUT/$v.log" 2>&1 || { echo "pmc pass $v failed"; tail -5 "$OUT/$v.log"; exit 1; }
done
python3 - "$OUT" ${VARIANTS:-product stop1 stop2 stop3 stop5} <<'PY' | tee "$OUT/summary.txt"
import csv, glob, os, sys
from collections import defaultdict
for v in sys.argv[2:]:
    acc = defaultdict(float)
    for f in glob.glob(os.path.join(sys.argv[1], v, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if r["Kernel_Name"].split("(")[0].replace("void ", "").split("<")[0].strip() == "k_tick":
                acc[r["Counter_Name"]] += float(r["Counter_Value"])
    w = acc.get("SQ_WAVES", 0) or 1
    print("%-8s waves %9.0f  per wave: valu %7.1f salu %7.1f lds %6.1f vmem_rd %6.1f vmem_wr %6.1f" % (
        v, acc.get("SQ_WAVES", 0), acc.get("SQ_INSTS_VALU", 0) / w, acc.get("SQ_INSTS_SALU", 0) / w,
        acc.get("SQ_INSTS_LDS", 0) / w, acc.get("SQ_INSTS_VMEM_RD", 0) / w, acc.get("SQ_INSTS_VMEM_WR", 0) / w))
PY
