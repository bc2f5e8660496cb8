#!/bin/bash
# Round-3 GPU pass: the engine-shaped memset graph probe, every -m gpu test, bench lines for C3/C5/C4
# and the 8 192-env N=8 shard, and the k_tick / k_reset phase stamps at 8 192 and 65 536 envs.
cd "$(dirname "$0")/.." || exit 2
mkdir -p gpurun_out
(cd tools/probe && timeout -k 10 120 ./graphprobe memset fork > ../../gpurun_out/graphprobe_fork.log 2>&1)
echo "graphprobe rc=$?"
CFGS="${CFGS:-c3 c5 c4}" bash tools/gpu_check.sh || exit 1
timeout -k 10 120 python bench.py --envs 8192 --steps 200 --warmup 20 --no-cpu-baseline > gpurun_out/bench_n8.json 2> gpurun_out/bench_n8.err || exit 1
python -c "import json;d=json.load(open('gpurun_out/bench_n8.json'));r=d['roofline'];print('n8', round(d['value']/1e6,1), 'M/s ms', round(d['ms_per_step'],4), 'step', round(r['step_launch_ms'],4), 'obs', round(r['k_obs_ms'],4))"
if [ -n "$STAMPS" ]; then
  N_ENVS=8192 GS=16 timeout -k 10 120 python tools/stamps.py > gpurun_out/stamps_8192.log 2>&1 || exit 1
  N_ENVS=65536 GS=8 timeout -k 10 120 python tools/stamps.py > gpurun_out/stamps_65536.log 2>&1 || exit 1
fi
if [ -n "$AB_LIBS" ]; then
  CFGS="${AB_CFGS:-c5 c3}" LIBS="$AB_LIBS" STEPS=100 bash tools/ab.sh > gpurun_out/ab.log 2>&1 || { tail -5 gpurun_out/ab.log; exit 1; }
  cat gpurun_out/ab.log
fi
