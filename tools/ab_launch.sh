#!/bin/bash
# A/B of launch overrides on one box: bench line per (round, variant) for each config in CFGS.
# VARIANTS: space-separated bench.py --launch values ("auto" = no override), e.g.
#   CFGS="n8 c2" VARIANTS="auto fobs=1 lanes=32" bash tools/ab_launch.sh   (lanes=G: --lanes-per-env G)
cd "$(dirname "$0")/.." || exit 2
mkdir -p gpurun_out
args() { case $1 in n8) echo "--config c3 --envs 8192";; c5n8) echo "--config c5 --envs 8192";; *) echo "--config $1";; esac; }
for r in 1 2; do
  for cfg in ${CFGS:-c3}; do
    for v in ${VARIANTS:-auto}; do
      case $v in
        auto) lflag="";;
        lanes=*) lflag="--lanes-per-env ${v#lanes=}";;
        *) lflag="--launch $v";;
      esac
      tag=$(echo "$v" | tr ',=' '_-')
      out=gpurun_out/abl_${cfg}_${tag}_$r.json
      timeout -k 10 180 python bench.py $(args $cfg) --steps ${STEPS:-200} --warmup 20 --no-cpu-baseline $lflag > $out 2> $out.err || { tail -5 $out.err; exit 1; }
      python -c "import json;d=json.load(open('$out'));r=d['roofline'];print('$r $cfg $v', round(d['value']/1e6,2), 'M/s ms', round(d['ms_per_step'],4), 'step', round(r['step_launch_ms'],4), 'obs', round(r['k_obs_ms'],4), 'reset', round(r['k_reset_ms'],4), 'respawn', round(r['k_respawn_ms'],4))"
    done
  done
done
