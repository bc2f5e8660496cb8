#!/bin/bash
# rocprofv3 evidence for profiles/: one kernel-trace/stats pass, then one PMC pass per
# counter (FETCH_SIZE and WRITE_SIZE do not fit one TCC pass on gfx950), each on the same
# bench command.  Outputs under gpurun_out/prof/<tag>; tools/pmc_summary.py reduces them.
cd "$(dirname "$0")/.." || exit 2
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null || exit 2
ROOT=$PWD
OUT=$ROOT/gpurun_out/prof
mkdir -p "$OUT"
BENCH="bench.py --steps ${STEPS:-50} --warmup 10 --no-cpu-baseline ${BENCH_ARGS}"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T --output-format csv -d "$OUT/kt" -o run -- python3 $BENCH \
    > "$OUT/kt.log" 2>&1 || { echo "kernel-trace pass failed"; tail -5 "$OUT/kt.log"; exit 1; }
echo "kernel-trace ok"
for c in FETCH_SIZE WRITE_SIZE; do
    timeout -k 10 300 rocprofv3 --pmc $c -T --output-format csv -d "$OUT/$c" -o run -- python3 $BENCH \
        > "$OUT/$c.log" 2>&1 || { echo "pmc $c pass failed"; tail -5 "$OUT/$c.log"; exit 1; }
    echo "pmc $c ok"
done
# profiles/ written on the box is not merged back: run tools/pmc_summary.py locally on gpurun_out/prof
python3 tools/pmc_summary.py "$OUT" ${TAG:-r01} ${PRESET:-c3} ${ENVS:-65536}
