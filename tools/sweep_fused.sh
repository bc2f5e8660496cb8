cd "$(dirname "$0")/.." || exit 2
for F in 0 1; do
  for G in 16 32; do
    ZS_FUSED=$F timeout -k 10 120 python bench.py --steps 200 --warmup 20 --no-cpu-baseline --lanes-per-env $G > gpurun_out/sf_${F}_${G}.log 2>&1 || exit 1
    python -c "
import json; d=json.loads(open('gpurun_out/sf_${F}_${G}.log').read().strip().splitlines()[-1]); r=d['roofline']
print('fused=$F G=$G', round(d['value']/1e6,1), 'M/s', 'ms', round(d['ms_per_step'],4), 'tick', round(r['step_launch_ms']*1e3,1), 'obs', round(r['k_obs_ms']*1e3,1), 'reset', round(r['k_reset_ms']*1e3,1))"
  done
done
