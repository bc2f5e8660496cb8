#!/bin/bash
# register-budget variants (diagnostic builds compiled with -DZS_STEP_WAVES=W) x launch paths
cd "$(dirname "$0")/.." || exit 2
for W in 1 4 6 8; do
  lib=""; [ $W -ne 1 ] && lib="ZS_ENGINE_LIB=$PWD/libzombsole_amd/_build/libzombsole_mi355x_w$W.so"
  for N in 65536 8192; do
    for v in "default ZS_DUMMY=1" "fobs0 ZS_FOBS=0" "unfused ZS_FUSED=0"; do
      set -- $v
      env $lib $2 timeout -k 10 120 python bench.py --steps 30 --warmup 5 --no-cpu-baseline --envs-per-gpu $N > gpurun_out/w.log 2>&1 || { tail -5 gpurun_out/w.log; exit 1; }
      python -c "
import json; d=json.loads(open('gpurun_out/w.log').read().strip().splitlines()[-1]); r=d['roofline']
print('W=$W N=$N $1', round(d['value']/1e6,1), 'M/s  ms', round(d['ms_per_step'],4), 'step', round(r['step_launch_ms']*1e3,1), 'obs', round(r['k_obs_ms']*1e3,1), 'reset', round(r['k_reset_ms']*1e3,1))"
    done
  done
done
