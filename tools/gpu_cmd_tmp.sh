#!/bin/bash
# scratch GPU command of the current session (not part of the product)
cd "$(dirname "$0")/.." || exit 2
mkdir -p gpurun_out
TAG=r03c CFGS="c3 c2 c4 c5 n8" PCFGS="c3" bash tools/profile_round.sh 2>&1 | tail -20
