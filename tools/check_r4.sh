#!/bin/bash
# Round-4 GPU pass: every -m gpu test (PYTEST_K filters), bench lines per config in CFGS, optional
# launch A/B (AB_CFGS x AB_VARIANTS) and step-launch phase stamps (STAMPS=1; build them on the CPU first
# with `python tools/stamps.py --build-only`).  Each GPU step has its own time limit; stops at the first failure.
cd "$(dirname "$0")/.." || exit 2
mkdir -p gpurun_out
if [ -z "$NO_TESTS" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} \
      > gpurun_out/pytest_gpu.log 2>&1 || { tail -40 gpurun_out/pytest_gpu.log; exit 1; }
  tail -2 gpurun_out/pytest_gpu.log
fi
args() { case $1 in n8) echo "--config c3 --envs 8192";; c5n8) echo "--config c5 --envs 8192";; *) echo "--config $1";; esac; }
for cfg in ${CFGS:-}; do
  timeout -k 10 180 python bench.py $(args $cfg) --steps 200 --warmup 20 --no-cpu-baseline > gpurun_out/bench_$cfg.json 2> gpurun_out/bench_$cfg.err || { tail -5 gpurun_out/bench_$cfg.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/bench_$cfg.json'));r=d['roofline'];print('$cfg', round(d['value']/1e6,1), 'M/s ms', round(d['ms_per_step'],4), 'step', round(r['step_launch_ms'],4), 'obs', round(r['k_obs_ms'],4), 'reset', round(r['k_reset_ms'],4), 'respawn', round(r['k_respawn_ms'],4))"
done
if [ -n "$AB_VARIANTS" ]; then
  CFGS="${AB_CFGS:-n8}" VARIANTS="$AB_VARIANTS" STEPS=${AB_STEPS:-200} bash tools/ab_launch.sh > gpurun_out/ab_launch.log 2>&1 || { tail -5 gpurun_out/ab_launch.log; exit 1; }
  cat gpurun_out/ab_launch.log
fi
if [ -n "$STAMPS" ]; then
  N_ENVS=8192 GS=16 timeout -k 10 120 python tools/stamps.py > gpurun_out/stamps_8192.log 2>&1 || { tail -5 gpurun_out/stamps_8192.log; exit 1; }
  cat gpurun_out/stamps_8192.log
  if [ -n "$STAMPS_LAUNCH" ]; then
    LAUNCH="$STAMPS_LAUNCH" N_ENVS=8192 GS=16 timeout -k 10 120 python tools/stamps.py > gpurun_out/stamps_8192_b.log 2>&1 || { tail -5 gpurun_out/stamps_8192_b.log; exit 1; }
    cat gpurun_out/stamps_8192_b.log
  fi
fi
