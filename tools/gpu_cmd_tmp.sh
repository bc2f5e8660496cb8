#!/bin/bash
# scratch GPU command of the current session (not part of the product)
cd "$(dirname "$0")/.." || exit 2
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread \
    -k "gather or c4 or kernel_paths or respawn or city128 or golden" > gpurun_out/pytest_gather.log 2>&1 || { tail -40 gpurun_out/pytest_gather.log; exit 1; }
tail -2 gpurun_out/pytest_gather.log
CFGS="c4" VAR=ZS_OBS_GATHER_FLUSH VALS="0 1" STEPS=100 bash tools/ab_env.sh 2>&1 | tee gpurun_out/ab_gather.log
