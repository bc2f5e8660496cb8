#!/bin/bash
# Round-5 GPU pass: the -m gpu tests (PYTEST_K filters, NO_TESTS skips), bench lines per config in CFGS for
# each policy in POLICIES (device: on-device uniform policy; external: torch policy on the previous step's
# observations + the caller-actions graph), and EXCHANGE=1: C5's 8 192-env shard with the per-step exchange at
# world size 1 (collectives skipped, then forced with --gather-self) plus a rocprofv3 kernel trace of the
# forced one.  Outputs under gpurun_out/$TAG.  Each GPU step has its own time limit; stops at the first failure.
cd "$(dirname "$0")/.." || exit 2
TAG=${TAG:-r05}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
if [ -z "$NO_TESTS" ]; then
  timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} \
      > "$OUT/pytest_gpu.log" 2>&1 || { tail -40 "$OUT/pytest_gpu.log"; exit 1; }
  tail -2 "$OUT/pytest_gpu.log"
fi
args() { case $1 in n8) echo "--config c3 --envs 8192";; c5n8) echo "--config c5 --envs 8192";; *) echo "--config $1";; esac; }
show() {
  python -c "import json,sys;d=json.load(open(sys.argv[1]));r=d['roofline'];m=d.get('multi_step_graph');print(sys.argv[2], round(d['value']/1e6,2), 'M/s ms', round(d['ms_per_step'],4), 'step', round(r['step_launch_ms'],4), 'obs', round(r['k_obs_ms'],4), 'reset', round(r['k_reset_ms'],4), 'respawn', round(r['k_respawn_ms'],4), ('multi %d: %.2f M' % (m['graph_steps'], m['value']/1e6)) if m else '')" "$1" "$2"
}
for cfg in ${CFGS:-}; do
  for pol in ${POLICIES:-device}; do
    f="$OUT/bench_${cfg}_$pol"
    timeout -k 10 180 python bench.py $(args $cfg) --policy $pol --steps ${STEPS:-200} --warmup 20 --no-cpu-baseline $BENCH_EXTRA \
        > "$f.json" 2> "$f.err" || { tail -5 "$f.err"; exit 1; }
    show "$f.json" "$cfg/$pol"
  done
done
if [ -n "$EXCHANGE" ]; then
  # one rank of an RCCL group without torchrun (the env:// rendezvous variables torchrun would set)
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
