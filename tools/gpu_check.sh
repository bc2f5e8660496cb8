#!/bin/bash
# GPU regression pass: every -m gpu test (optionally -k filtered), then one bench line per config.
# Each GPU step has its own time limit; the script stops at the first failure.
cd "$(dirname "$0")/.." || exit 2
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} \
    > gpurun_out/pytest_gpu.log 2>&1 || { tail -40 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
for cfg in ${CFGS:-c3}; do
    timeout -k 10 180 python bench.py --config $cfg --steps 100 --warmup 10 --no-cpu-baseline > gpurun_out/bench_$cfg.json 2> gpurun_out/bench_$cfg.err || { tail -5 gpurun_out/bench_$cfg.err; exit 1; }
    python -c "import json,sys;d=json.load(open('gpurun_out/bench_$cfg.json'));r=d['roofline'];print('$cfg', round(d['value']/1e6,1), 'M/s ms', round(d['ms_per_step'],4), 'tick', round(r['step_launch_ms'],4), 'obs', round(r['k_obs_ms'],4), 'reset', round(r['k_reset_ms'],4), 'respawn', round(r['k_respawn_ms'],4))"
done
