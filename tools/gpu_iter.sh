#!/bin/bash
# Iteration loop on the GPU box: parity tests first (stop on failure), then the launch-path sweep
# at the bench sizes.  Diagnostic; outputs under gpurun_out/.
cd "$(dirname "$0")/.." || exit 2
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests -m gpu -x -q ${PYTEST_ARGS} > gpurun_out/pytest_gpu.log 2>&1
rc=$?; tail -5 gpurun_out/pytest_gpu.log
[ $rc -ne 0 ] && exit $rc
export LIST=${LIST:-"default ZS_DUMMY=1
fobs0 ZS_FOBS=0
unfused ZS_FUSED=0"}
bash tools/sweep_g.sh && N=8192 bash tools/sweep_g.sh
