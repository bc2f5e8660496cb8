#!/bin/bash
# HBM traffic and issue counters of one bench command's kernels: FETCH_SIZE / WRITE_SIZE passes and the
# SQ / GRBM passes of tools/pmc_sq.sh, each rocprofv3 pass under its own time limit (counter passes
# only: no trace domains).  Usage: tools/pmc_obs.sh TAG [bench args...]; outputs gpurun_out/pmcobs/TAG.
cd "$(dirname "$0")/.." || exit 2
ROOT=$PWD
cd /tmp && export TMPDIR=/tmp && cd "$ROOT" || exit 2
TAG=$1; shift
OUT=$ROOT/gpurun_out/pmcobs/$TAG
mkdir -p "$OUT"
B="bench.py $* --steps 20 --warmup 5 --no-cpu-baseline"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T --output-format csv -d "$OUT/kt" -o run -- python3 $B > "$OUT/kt.log" 2>&1 \
    || { echo "kernel-trace failed"; tail -5 "$OUT/kt.log"; exit 1; }
for c in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 300 rocprofv3 --pmc $c -T --output-format csv -d "$OUT/$c" -o run -- python3 $B > "$OUT/$c.log" 2>&1 \
        || { echo "pmc $c failed"; tail -5 "$OUT/$c.log"; exit 1; }
done
bash tools/pmc_sq.sh "obs_$TAG" "$@" --steps 20 --warmup 5 --no-cpu-baseline --no-graph > "$OUT/sq.log" 2>&1 \
    || { echo "pmc sq failed"; tail -5 "$OUT/sq.log"; exit 1; }
echo "profiled $TAG"
