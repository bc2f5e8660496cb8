#!/bin/bash
# Parity of the engine's alternative launch paths: unfused (k_reset + k_tick + k_obs) and fused
# without in-launch observations (k_step + k_obs).  The default path is covered by gpu_check.sh.
cd "$(dirname "$0")/.." || exit 2
mkdir -p gpurun_out
for v in "ZS_FUSED=0" "ZS_FOBS=0"; do
    env $v timeout -k 10 600 python -m pytest -x -q tests/test_engine_oracle.py tests/test_engine_golden.py \
        > "gpurun_out/paths_${v%%=*}.log" 2>&1
    rc=$?; echo "$v pytest rc=$rc"; tail -3 "gpurun_out/paths_${v%%=*}.log"
    [ $rc -ne 0 ] && exit $rc
done
exit 0
