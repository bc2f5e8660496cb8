#!/bin/bash
# C5's per-GPU shard at N=8 (8 192 envs, int16, 4 agents + 20 zombies) on one GPU: the bench line alone, then
# the same under torchrun (one rank, an RCCL group) with the per-step all-gather of observations, rewards,
# done and truncated (vector.StepGather: comm stream, double-buffered output sets).  The difference is the
# exchange's cost on the step at world size 1.
cd "$(dirname "$0")/.." || exit 2
mkdir -p gpurun_out
timeout -k 10 180 python bench.py --config c5 --envs 8192 --steps ${STEPS:-200} --warmup 20 --no-cpu-baseline --graph-steps 1 \
    > gpurun_out/bench_c5n8.json 2> gpurun_out/bench_c5n8.err || { tail -5 gpurun_out/bench_c5n8.err; exit 1; }
timeout -k 10 240 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 \
    --master-port ${PORT:-29533} bench.py --config c5 --envs 8192 --gather --steps ${STEPS:-200} --warmup 20 \
    --no-cpu-baseline > gpurun_out/bench_c5n8_gather.json 2> gpurun_out/bench_c5n8_gather.err \
    || { tail -5 gpurun_out/bench_c5n8_gather.err; exit 1; }
for f in bench_c5n8 bench_c5n8_gather; do
  python -c "import json;d=json.load(open('gpurun_out/$f.json'));r=d['roofline'];print('$f', round(d['value']/1e6,2), 'M/s ms', round(d['ms_per_step'],4), 'step', round(r['step_launch_ms'],4), 'obs', round(r['k_obs_ms'],4), d['config']['parallelism'])"
done
