#!/bin/bash
# k_obs ablations (diagnostic builds): bit 1 = constant values, bit 2 = no staging, bit 4 = no static tables
cd "$(dirname "$0")/.." || exit 2
for x in ${EXPS:-0 1 2 3 7}; do
  lib=""; [ $x -ne 0 ] && lib="ZS_ENGINE_LIB=$PWD/libzombsole_amd/_build/libzombsole_mi355x_exp$x.so"
  env $lib ZS_FOBS=0 timeout -k 10 120 python bench.py --steps 30 --warmup 5 --no-cpu-baseline --envs-per-gpu 65536 > gpurun_out/exp.log 2>&1 || { tail -5 gpurun_out/exp.log; exit 1; }
  python -c "
import json; d=json.loads(open('gpurun_out/exp.log').read().strip().splitlines()[-1]); r=d['roofline']
print('exp$x', 'step', round(r['step_launch_ms']*1e3,1), 'obs', round(r['k_obs_ms']*1e3,1))"
done
timeout -k 10 120 ./tools/probe/storebw
