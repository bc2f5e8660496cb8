#!/bin/bash
# SQ / GRBM counters per kernel of one bench command (one counter group per rocprofv3 pass, each pass
# under its own time limit).  Usage: tools/pmc_sq.sh TAG [bench args...]; summary: tools/pmc_sq.py
cd "$(dirname "$0")/.." || exit 2
ROOT=$PWD
cd /tmp && export TMPDIR=/tmp && cd "$ROOT" || exit 2
TAG=$1; shift
OUT=$ROOT/gpurun_out/pmcsq/$TAG
mkdir -p "$OUT"
i=0
for grp in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS" \
           "SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VMEM" \
           "GRBM_GUI_ACTIVE GRBM_COUNT"; do
    i=$((i + 1))
    timeout -s KILL 120 rocprofv3 --pmc $grp -T --output-format csv -d "$OUT/p$i" -o run -- python3 bench.py "$@" \
        > "$OUT/p$i.log" 2>&1 || { echo "pass $i failed"; tail -5 "$OUT/p$i.log"; exit 1; }
done
python3 tools/pmc_sq.py "$OUT"
