#!/bin/bash
# scratch GPU command of the current session (not part of the product)
cd "$(dirname "$0")/.." || exit 2
mkdir -p gpurun_out
TAG=r03d CFGS="c5 c3" PCFGS="c5" bash tools/profile_round.sh 2>&1 | tail -20
