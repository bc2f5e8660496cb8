#!/bin/bash
# observation-write diagnostics: store-shape probe, then PMC traffic of k_obs at 65536 envs
cd "$(dirname "$0")/.." || exit 2
mkdir -p gpurun_out
timeout -k 10 120 ./tools/probe/storebw > gpurun_out/storebw.log 2>&1; cat gpurun_out/storebw.log
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
for c in FETCH_SIZE WRITE_SIZE; do
  ZS_FOBS=0 timeout -k 10 300 rocprofv3 --pmc $c -T --output-format csv -d gpurun_out/pmc_$c -o run -- python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --envs-per-gpu 65536 > gpurun_out/pmc_$c.log 2>&1 || { tail -5 gpurun_out/pmc_$c.log; exit 1; }
done
echo pmc done
