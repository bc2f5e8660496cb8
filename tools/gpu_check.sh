#!/bin/bash
# One GPU session: smoke -> gpu tests -> short bench.  Stops at the first crash /
# timeout (exit >= 2 from pytest, or any nonzero from the others); plain test
# failures (pytest exit 1) still let the bench run.
cd "$(dirname "$0")/.." || exit 2
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 300 python __graft_entry__.py smoke > gpurun_out/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -3 gpurun_out/smoke.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 ${PYTEST_TIMEOUT:-900} python -m pytest tests -m gpu -q ${PYTEST_ARGS} > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -15 gpurun_out/pytest_gpu.log
[ $rc -ge 2 ] && exit $rc
timeout -k 10 300 python bench.py ${BENCH_ARGS:---steps 100 --warmup 10} > gpurun_out/bench.log 2>&1
rc2=$?; echo "bench rc=$rc2"; tail -3 gpurun_out/bench.log
exit $(( rc > rc2 ? rc : rc2 ))
