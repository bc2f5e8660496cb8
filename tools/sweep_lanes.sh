cd /root/repo
for G in 8 16 32 64; do
  for N in 8192 32768; do
    timeout -k 10 120 python bench.py --steps 100 --warmup 20 --no-cpu-baseline --lanes-per-env $G --envs-per-gpu $N > gpurun_out/sw_${G}_${N}.log 2>&1 || exit 1
    python -c "
import json,sys; d=json.loads(open('gpurun_out/sw_${G}_${N}.log').read().strip().splitlines()[-1]); r=d['roofline']
print('G=$G N=$N', round(d['value']/1e6,1), 'M/s', 'ms', round(d['ms_per_step'],4), 'tick', round(r['step_launch_ms']*1e3,1), 'obs', round(r['k_obs_ms']*1e3,1), 'reset', round(r['k_reset_ms']*1e3,1))"
  done
done
