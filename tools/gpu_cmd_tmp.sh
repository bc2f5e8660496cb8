#!/bin/bash
# scratch GPU command of the current session (not part of the product)
cd "$(dirname "$0")/.." || exit 2
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread \
    -k "obstacle_hp or store_stream or kernel_paths or ring or c5_65536 or c3_65536_graph or set_state or golden" > gpurun_out/pytest_patch.log 2>&1 || { tail -40 gpurun_out/pytest_patch.log; exit 1; }
tail -2 gpurun_out/pytest_patch.log
CFGS="c5" VAR=ZS_OBS_RING VALS="0 1" STEPS=100 bash tools/ab_env.sh 2>&1 | tee gpurun_out/ab_ring5b.log
TAG=r03b CFGS="c3 c2 c4 c5 n8" PCFGS="c3 c5" bash tools/profile_round.sh 2>&1 | tail -20
