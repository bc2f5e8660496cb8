#!/bin/bash
# Round-5 GPU pass in stages (each GPU step under its own time limit, stop at the first failure):
#   1) the -m gpu suite without the k_fstep tests (PYTEST_K / NO_TESTS as check_r5.sh)
#   2) bench lines: BENCHES = "name:args;name:args;..." (bench.py arguments after the preset)
#   3) FSTEP_TESTS=1: the k_fstep parity tests on their own, under a short limit
#   4) EXCHANGE=1: as check_r5.sh
cd "$(dirname "$0")/.." || exit 2
TAG=${TAG:-r05}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
if [ -z "$NO_TESTS" ]; then
  # test failures (exit 1) are reported and the benches still run; a crash, abort or time limit stops here
  timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread -k "not fstep ${PYTEST_K:+and ($PYTEST_K)}" \
      > "$OUT/pytest_gpu.log" 2>&1
  rc=$?
  grep -E "^(FAILED|ERROR)" "$OUT/pytest_gpu.log" | head -20
  tail -2 "$OUT/pytest_gpu.log"
  [ $rc -le 1 ] || exit 1
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
if [ -n "$FSTEP_TESTS" ]; then
  timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 150 --timeout-method thread -k "fstep" \
      > "$OUT/pytest_fstep.log" 2>&1 || { tail -40 "$OUT/pytest_fstep.log"; exit 1; }
  tail -2 "$OUT/pytest_fstep.log"
  IFS=';' read -ra BL2 <<< "${BENCHES2:-}"
  for b in "${BL2[@]}"; do
    name="${b%%:*}"; a="${b#*:}"
    [ -z "$name" ] && continue
    f="$OUT/bench_$name"
    timeout -k 10 180 python bench.py $a --steps ${STEPS:-200} --warmup 20 --no-cpu-baseline > "$f.json" 2> "$f.err" || { echo "bench $name failed"; tail -5 "$f.err"; exit 1; }
    show "$f.json" "$name"
  done
fi
if [ -n "$EXCHANGE" ]; then
  export MASTER_ADDR=127.0.0.1 MASTER_PORT=${PORT:-29533} RANK=0 LOCAL_RANK=0 WORLD_SIZE=1 TORCHELASTIC_RUN_ID=$TAG
  B="bench.py --config c5 --envs 8192 --gather --steps ${STEPS:-200} --warmup 20 --no-cpu-baseline"
  timeout -k 10 180 python $B > "$OUT/bench_c5n8_gather.json" 2> "$OUT/bench_c5n8_gather.err" \
      || { tail -5 "$OUT/bench_c5n8_gather.err"; exit 1; }
  show "$OUT/bench_c5n8_gather.json" c5n8/gather-skipped
  timeout -k 10 180 python $B --gather-self > "$OUT/bench_c5n8_gather_self.json" 2> "$OUT/bench_c5n8_gather_self.err" \
      || { tail -5 "$OUT/bench_c5n8_gather_self.err"; exit 1; }
  show "$OUT/bench_c5n8_gather_self.json" c5n8/gather-self
  cd /tmp && export TMPDIR=/tmp && cd - > /dev/null || exit 2
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -T --output-format csv -d "$PWD/$OUT/prof_exchange" -o run -- \
      python3 bench.py --config c5 --envs 8192 --gather --gather-self --steps 50 --warmup 10 --no-cpu-baseline \
      > "$OUT/prof_exchange.log" 2>&1 || { tail -5 "$OUT/prof_exchange.log"; exit 1; }
  echo "exchange traced"
fi
