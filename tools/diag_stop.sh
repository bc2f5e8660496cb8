#!/bin/bash
# Diagnostic: k_tick's time with the tick ended after phase k (-DZS_DIAG_STOP=k builds, state frozen:
# nothing is stored back) against the product, per config: the throughput cost of each phase.
#   python -c "import __graft_entry__ as ge; ..."  builds libzombsole_mi355x_stop{1..5}.so first
cd "$(dirname "$0")/.." || exit 2
OUT=${OUT:-gpurun_out/diag_stop}
mkdir -p "$OUT"
for cfg in ${CFGS:-c3 c5 c4}; do
  for v in product stop1 stop2 stop3 stop4 stop5; do
    lib=libzombsole_amd/_build/libzombsole_mi355x.so
    [ "$v" != product ] && lib=libzombsole_amd/_build/libzombsole_mi355x_$v.so
    timeout -k 10 120 python bench.py --config "$cfg" --engine-lib "$lib" --no-graph --steps 100 --warmup 10 \
        --no-cpu-baseline > "$OUT/${cfg}_$v.json" 2> "$OUT/${cfg}_$v.err" || { echo "$cfg $v failed"; tail -5 "$OUT/${cfg}_$v.err"; exit 1; }
    python -c "import json,sys;d=json.load(open(sys.argv[1]));r=d['roofline'];print(sys.argv[2], sys.argv[3], 'tick', round(r['step_launch_ms']*1e3,1), 'us  obs', round(r['k_obs_ms']*1e3,1), 'us  respawn', round(r['k_respawn_ms']*1e3,1))" "$OUT/${cfg}_$v.json" "$cfg" "$v"
  done
done
