#!/bin/bash
# k_obs_pipe register budget variants (diagnostic builds -DZS_OBS_PIPE_WAVES=W), observations by k_obs
cd "$(dirname "$0")/.." || exit 2
for rep in 1 2; do
for W in 4 5 6; do
  lib=""; [ $W -ne 4 ] && lib="ZS_ENGINE_LIB=$PWD/libzombsole_amd/_build/libzombsole_mi355x_pw$W.so"
  for N in 65536 8192; do
    env $lib ZS_FOBS=0 timeout -k 10 120 python bench.py --steps 30 --warmup 5 --no-cpu-baseline --envs $N > gpurun_out/pw.log 2>&1 || { tail -5 gpurun_out/pw.log; exit 1; }
    python -c "
import json; d=json.loads(open('gpurun_out/pw.log').read().strip().splitlines()[-1]); r=d['roofline']
print('W=$W N=$N', round(d['value']/1e6,1), 'M/s step', round(r['step_launch_ms']*1e3,1), 'obs', round(r['k_obs_ms']*1e3,1), 'reset', round(r['k_reset_ms']*1e3,1))"
  done
done
done
