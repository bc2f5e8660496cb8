#!/bin/bash
# Round-6 GPU pass: TESTS (pytest paths / -k, default the whole -m gpu suite), then C1=1: the drop-in per-call
# timing (tools/c1_bench.py), then BENCHES = "name:args;..." bench lines.  Each GPU step has its own limit
# and the script stops at the first crash or time limit.
cd "$(dirname "$0")/.." || exit 2
TAG=${TAG:-r06}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
if [ -z "$NO_TESTS" ]; then
  timeout -k 10 900 python -u -m pytest ${TESTS:-tests} -m gpu -v --timeout 300 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} \
      > "$OUT/pytest_gpu.log" 2>&1
  rc=$?
  grep -E "^(FAILED|ERROR)" "$OUT/pytest_gpu.log" | head -20
  tail -2 "$OUT/pytest_gpu.log"
  [ $rc -le 1 ] || exit 1
fi
if [ -n "$C1" ]; then
  timeout -k 10 300 python -u tools/c1_bench.py --steps ${C1_STEPS:-3000} --out "$OUT/c1.json" > "$OUT/c1.log" 2>&1 \
      || { tail -20 "$OUT/c1.log"; exit 1; }
  head -2 "$OUT/c1.log"
  if [ -n "$C1_EVENTS" ]; then
    timeout -k 10 300 python -u tools/c1_bench.py --steps ${C1_STEPS:-3000} --events --out "$OUT/c1_events.json" \
        > "$OUT/c1_events.log" 2>&1 || { tail -20 "$OUT/c1_events.log"; exit 1; }
    head -2 "$OUT/c1_events.log"
  fi
fi
show() {
  python -c "import json,sys;d=json.load(open(sys.argv[1]));r=d['roofline'];m=d.get('multi_step_graph');print(sys.argv[2], round(d['value']/1e6,2), 'M/s ms', round(d['ms_per_step'],4), r['kernel'], 'step', round(r['step_launch_ms'],4), 'obs', round(r['k_obs_ms'],4), 'reset', round(r['k_reset_ms'],4), 'respawn', round(r['k_respawn_ms'],4), 'frac', round(r['frac'],3), ('multi %d: %.2f M' % (m['graph_steps'], m['value']/1e6)) if m else '')" "$1" "$2"
}
IFS=';' read -ra BL <<< "${BENCHES:-}"
for b in "${BL[@]}"; do
  name="${b%%:*}"; a="${b#*:}"
  [ -z "$name" ] && continue
  f="$OUT/bench_$name"
  timeout -k 10 180 python bench.py $a --steps ${STEPS:-200} --warmup 20 --no-cpu-baseline > "$f.json" 2> "$f.err" || { echo "bench $name failed"; tail -5 "$f.err"; exit 1; }
  show "$f.json" "$name"
done
