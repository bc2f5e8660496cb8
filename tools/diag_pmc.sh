#!/bin/bash
# SQ counters of k_obs (product build and the EXP7 / EXP8 ablations), one counter group per pass
cd "$(dirname "$0")/.." || exit 2
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
mkdir -p gpurun_out/pmcsq
for x in 0 7 8; do
  lib=""; [ $x -ne 0 ] && lib="$PWD/libzombsole_amd/_build/libzombsole_mi355x_exp$x.so"
  for grp in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY" "SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM SQ_INSTS_VMEM_WR" "GRBM_GUI_ACTIVE GRBM_COUNT"; do
    tag=$(echo $grp | cut -d' ' -f1)
    env ${lib:+ZS_ENGINE_LIB=$lib} ZS_FOBS=0 timeout -k 10 200 rocprofv3 --pmc $grp -T --output-format csv -d gpurun_out/pmcsq/x${x}_$tag -o run -- python3 bench.py --steps 6 --warmup 2 --no-cpu-baseline --envs-per-gpu 65536 > gpurun_out/pmcsq/x${x}_$tag.log 2>&1 || { echo "fail $x $tag"; tail -3 gpurun_out/pmcsq/x${x}_$tag.log; }
  done
done
echo done
