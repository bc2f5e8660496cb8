#!/bin/bash
# Round evidence in one GPU call: the -m gpu suite, the default bench line (with the CPU baseline),
# one bench line per config, and per profiled config a rocprofv3 kernel-trace pass, FETCH/WRITE passes
# and the SQ/GRBM counter passes (tools/pmc_sq.sh).  Outputs under gpurun_out/round/<TAG>;
# tools/pmc_summary.py and tools/pmc_sq.py turn them into profiles/<TAG>_<cfg>_* here.  Stops at the
# first failing step.  Configs: c2 c3 c4 c5 (bench.py presets) and n8 (the C3 shard of an 8-GPU run).
cd "$(dirname "$0")/.." || exit 2
TAG=${TAG:-r03}
OUT=gpurun_out/round/$TAG
mkdir -p "$OUT"
args() { case $1 in n8) echo "--config c3 --envs 8192";; c5n8) echo "--config c5 --envs 8192";; *) echo "--config $1";; esac; }
if [ -z "$NO_TESTS" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1 \
      || { tail -30 "$OUT/pytest_gpu.log"; exit 1; }
  tail -1 "$OUT/pytest_gpu.log"
fi
if [ -z "$NO_BENCH" ]; then
  timeout -k 10 300 python bench.py > "$OUT/bench_default.log" 2>&1 || { tail -5 "$OUT/bench_default.log"; exit 1; }
  tail -1 "$OUT/bench_default.log" | cut -c1-200
  for cfg in ${CFGS:-c3 c2 c4 c5 n8}; do
      timeout -k 10 180 python bench.py $(args $cfg) --steps 200 --warmup 20 --no-cpu-baseline > "$OUT/bench_$cfg.log" 2>&1 \
          || { tail -5 "$OUT/bench_$cfg.log"; exit 1; }
  done
fi
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null || exit 2
for cfg in ${PCFGS:-c3 c4 c5 n8}; do
    P=$PWD/$OUT/prof_$cfg
    mkdir -p "$P"
    B="bench.py $(args $cfg) --steps 50 --warmup 10 --no-cpu-baseline"
    timeout -k 10 300 rocprofv3 --kernel-trace --stats -T --output-format csv -d "$P/kt" -o run -- python3 $B > "$P/kt.log" 2>&1 \
        || { echo "kernel-trace $cfg failed"; tail -5 "$P/kt.log"; exit 1; }
    for c in FETCH_SIZE WRITE_SIZE; do
        timeout -s KILL 300 rocprofv3 --pmc $c -T --output-format csv -d "$P/$c" -o run -- python3 $B > "$P/$c.log" 2>&1 \
            || { echo "pmc $c $cfg failed"; tail -5 "$P/$c.log"; exit 1; }
    done
    bash tools/pmc_sq.sh "${TAG}_$cfg" $(args $cfg) --steps 20 --warmup 5 --no-cpu-baseline --no-graph > "$P/sq.log" 2>&1 \
        || { echo "pmc sq $cfg failed"; tail -5 "$P/sq.log"; exit 1; }
    echo "profiled $cfg"
done
