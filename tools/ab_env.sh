#!/bin/bash
# A/B of one engine switch on one box: bench line per (round, value of $VAR) for each config in CFGS.
cd "$(dirname "$0")/.." || exit 2
mkdir -p gpurun_out
args() { case $1 in n8) echo "--config c3 --envs 8192";; *) echo "--config $1";; esac; }
for r in 1 2; do
  for cfg in ${CFGS:-c3}; do
    for v in ${VALS:-0 1}; do
      out=gpurun_out/abenv_${cfg}_${VAR}_${v}_$r.json
      env $VAR=$v timeout -k 10 180 python bench.py $(args $cfg) --steps ${STEPS:-200} --warmup 20 --no-cpu-baseline > $out 2> $out.err || { tail -5 $out.err; exit 1; }
      python -c "import json;d=json.load(open('$out'));r=d['roofline'];print('$r $cfg $VAR=$v', round(d['value']/1e6,2), 'M/s ms', round(d['ms_per_step'],4), 'tick', round(r['step_launch_ms'],4), 'obs', round(r['k_obs_ms'],4), 'reset', round(r['k_reset_ms'],4))"
    done
  done
done
