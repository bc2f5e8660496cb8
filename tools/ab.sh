#!/bin/bash
# A/B of engine builds on one box: bench line per (round, lib) for each config in CFGS.
# LIBS: space-separated .so paths ("default" = the in-tree build), passed as bench.py --engine-lib.
cd "$(dirname "$0")/.." || exit 2
mkdir -p gpurun_out
args() { case $1 in n8) echo "--config c3 --envs 8192";; c5n8) echo "--config c5 --envs 8192";; *) echo "--config $1";; esac; }
for r in 1 2; do
  for cfg in ${CFGS:-c3}; do
    for lib in ${LIBS:-default}; do
      if [ "$lib" = default ]; then lflag=""; else lflag="--engine-lib $lib"; fi
      out=gpurun_out/ab_${cfg}_$(basename $lib .so)_$r.json
      timeout -k 10 180 python bench.py $(args $cfg) --steps ${STEPS:-200} --warmup 20 --no-cpu-baseline $lflag $BENCH_ARGS > $out 2> $out.err || { tail -5 $out.err; exit 1; }
      python -c "import json;d=json.load(open('$out'));r=d['roofline'];print('$r $cfg $(basename $lib)', round(d['value']/1e6,2), 'M/s ms', round(d['ms_per_step'],4), 'tick', round(r['step_launch_ms'],4), 'obs', round(r['k_obs_ms'],4), 'reset', round(r['k_reset_ms'],4))"
    done
  done
done
