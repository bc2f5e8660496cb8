#!/bin/bash
# Diagnostic session: per-phase stamps of the step launch, then bench at several env counts and
# launch paths.  Never part of the product; outputs under gpurun_out/.
cd "$(dirname "$0")/.." || exit 2
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
GS=${GS:-8,16,32} timeout -k 10 300 python tools/stamps.py > gpurun_out/stamps.log 2>&1 || { echo "stamps failed"; tail -20 gpurun_out/stamps.log; exit 1; }
cat gpurun_out/stamps.log
for cfg in "8192" "16384" "32768" "65536" "8192 ZS_FOBS=0" "8192 ZS_FUSED=0"; do
    set -- $cfg
    N=$1; shift
    env $@ timeout -k 10 120 python bench.py --steps 100 --warmup 20 --no-cpu-baseline --envs-per-gpu $N > gpurun_out/diag_b.log 2>&1 || { echo "bench $cfg failed"; tail -5 gpurun_out/diag_b.log; exit 1; }
    python -c "
import json; d=json.loads(open('gpurun_out/diag_b.log').read().strip().splitlines()[-1]); r=d['roofline']
print('$cfg', round(d['value']/1e6,1), 'M/s', 'ms', round(d['ms_per_step'],4), 'tick', round(r['step_launch_ms']*1e3,1), 'obs', round(r['k_obs_ms']*1e3,1), 'reset', round(r['k_reset_ms']*1e3,1))"
done
