#!/bin/bash
# scratch GPU command of the current session (not part of the product)
cd "$(dirname "$0")/.." || exit 2
mkdir -p gpurun_out
CFGS="c3 c5" LIBS="default $PWD/tools/probe/lib_t8.so $PWD/tools/probe/lib_t4.so" STEPS=200 bash tools/ab.sh 2>&1 | tee gpurun_out/ab_ringthr.log
