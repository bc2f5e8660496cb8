#!/bin/bash
# launch-path sweep at a given env count (diagnostic).  LIST lines: tag, then env assignments.
cd "$(dirname "$0")/.." || exit 2
mkdir -p gpurun_out
N=${N:-65536}
LIST=${LIST:-"fobs0 ZS_FOBS=0
fobs1 ZS_FOBS=1"}
while read -r tag envs; do
    env ZS_VERBOSE=1 $envs timeout -k 10 120 python bench.py --steps 50 --warmup 10 --no-cpu-baseline --envs-per-gpu $N ${BENCH_ARGS} > gpurun_out/sg.log 2>&1 || { tail -5 gpurun_out/sg.log; exit 1; }
    grep zs_create gpurun_out/sg.log | head -1
    python -c "
import json; d=json.loads(open('gpurun_out/sg.log').read().strip().splitlines()[-1]); r=d['roofline']
print('$tag N=$N', round(d['value']/1e6,1), 'M/s', 'ms', round(d['ms_per_step'],4), 'step', round(r['step_launch_ms']*1e3,1), 'obs', round(r['k_obs_ms']*1e3,1), 'reset', round(r['k_reset_ms']*1e3,1))"
done <<< "$LIST"
