#!/bin/bash
# Run bench.py once per variant and print one summary line each.  Variants are arguments of the
# form 'label;ENV=v ENV2=v;bench args' (env and args may be empty), e.g.
#   bash tools/sweep.sh 'base;;' 'side0;;--launch reset_stream=-1' 'w2;;--engine-lib libzombsole_amd/_build/libzombsole_mi355x_w2.so'
# Stops at the first failing run (crash, timeout).
cd "$(dirname "$0")/.." || exit 2
mkdir -p gpurun_out/sweep
STEPS=${STEPS:-100}
for v in "$@"; do
    IFS=';' read -r label envs args <<< "$v"
    log=gpurun_out/sweep/$label.log
    env ZS_VERBOSE=1 $envs timeout -k 10 180 python bench.py --steps $STEPS --warmup 10 --no-cpu-baseline $args > "$log" 2>&1 || {
        echo "$label FAILED"; tail -5 "$log"; exit 1; }
    python3 - "$log" "$label" <<'EOF'
import json, sys
lines = open(sys.argv[1]).read().strip().splitlines()
d = json.loads(lines[-1]); r = d["roofline"]
cfg = [l for l in lines if l.startswith("zs_create")]
print("%-14s %7.1f M/s  %.4f ms/step  step %6.1f  obs %6.1f  reset %5.1f us  | %s" % (
    sys.argv[2], d["value"] / 1e6, d["ms_per_step"], r["step_launch_ms"] * 1e3, r["k_obs_ms"] * 1e3,
    r["k_reset_ms"] * 1e3, cfg[-1][10:] if cfg else ""))
EOF
done
