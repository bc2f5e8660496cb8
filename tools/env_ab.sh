#!/bin/bash
# A/B of HIP runtime settings on bench lines (diagnostic): VARIANTS = "name:VAR=v VAR2=v;...",
# CASES = "name:bench.py arguments;..." (default: ARGS as one case).  Two passes over every case x variant,
# each run under its own time limit; stop at the first failure.
cd "$(dirname "$0")/.." || exit 2
OUT=gpurun_out/${TAG:-r05}/env_ab
mkdir -p "$OUT"
IFS=';' read -ra VL <<< "${VARIANTS:-base:}"
IFS=';' read -ra CL <<< "${CASES:-case:$ARGS}"
for rep in 1 2; do
  for c in "${CL[@]}"; do
    cname="${c%%:*}"; cargs="${c#*:}"
    for v in "${VL[@]}"; do
      name="${v%%:*}"; envs="${v#*:}"
      f="$OUT/${cname}_${name}_$rep"
      env $envs timeout -k 10 180 python bench.py $cargs --steps ${STEPS:-300} --warmup 30 --no-cpu-baseline > "$f.json" 2> "$f.err" \
          || { echo "variant $cname/$name failed"; tail -5 "$f.err"; exit 1; }
      python -c "import json,sys;d=json.load(open(sys.argv[1]));print('%-10s %-10s rep %s %8.2f M/s %.4f ms' % (sys.argv[2], sys.argv[3], sys.argv[4], d['value']/1e6, d['ms_per_step']))" "$f.json" "$cname" "$name" "$rep"
    done
  done
done
