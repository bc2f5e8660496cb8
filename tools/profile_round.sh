#!/bin/bash
# Round evidence in one GPU call: the -m gpu suite, the default bench line (with the CPU baseline),
# one bench line per config, and rocprofv3 kernel-trace + FETCH/WRITE passes per config.  Outputs
# under gpurun_out/round/<TAG>; tools/pmc_summary.py turns gpurun_out/round/<TAG>/prof_<cfg> into
# profiles/<TAG>_<cfg>_* here.  Stops at the first failing step.
cd "$(dirname "$0")/.." || exit 2
TAG=${TAG:-r02}
OUT=gpurun_out/round/$TAG
mkdir -p "$OUT"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1 \
    || { tail -30 "$OUT/pytest_gpu.log"; exit 1; }
tail -1 "$OUT/pytest_gpu.log"
timeout -k 10 300 python bench.py > "$OUT/bench_default.log" 2>&1 || { tail -5 "$OUT/bench_default.log"; exit 1; }
tail -1 "$OUT/bench_default.log" | cut -c1-200
for cfg in ${CFGS:-c3 c2 c4 c5}; do
    timeout -k 10 180 python bench.py --config $cfg --steps 200 --warmup 20 --no-cpu-baseline > "$OUT/bench_$cfg.log" 2>&1 \
        || { tail -5 "$OUT/bench_$cfg.log"; exit 1; }
done
timeout -k 10 180 python bench.py --envs 8192 --steps 300 --warmup 20 --no-cpu-baseline > "$OUT/bench_n8.log" 2>&1 \
    || { tail -5 "$OUT/bench_n8.log"; exit 1; }
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null || exit 2
for cfg in ${PCFGS:-c3 c4 c5}; do
    P=$PWD/$OUT/prof_$cfg
    mkdir -p "$P"
    B="bench.py --config $cfg --steps 50 --warmup 10 --no-cpu-baseline"
    timeout -k 10 300 rocprofv3 --kernel-trace --stats -T --output-format csv -d "$P/kt" -o run -- python3 $B > "$P/kt.log" 2>&1 \
        || { echo "kernel-trace $cfg failed"; tail -5 "$P/kt.log"; exit 1; }
    for c in FETCH_SIZE WRITE_SIZE; do
        timeout -s KILL 300 rocprofv3 --pmc $c -T --output-format csv -d "$P/$c" -o run -- python3 $B > "$P/$c.log" 2>&1 \
            || { echo "pmc $c $cfg failed"; tail -5 "$P/$c.log"; exit 1; }
    done
    echo "profiled $cfg"
done
