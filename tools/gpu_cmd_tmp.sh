#!/bin/bash
# scratch GPU command of the current session (not part of the product)
cd "$(dirname "$0")/.." || exit 2
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_obstacle_hp.py -m gpu -x -v --timeout 240 --timeout-method thread > gpurun_out/pytest_hp.log 2>&1 || { tail -40 gpurun_out/pytest_hp.log; exit 1; }
tail -3 gpurun_out/pytest_hp.log
