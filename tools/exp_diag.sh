# bench with diagnostic engine builds (ZS_ENGINE_LIB=libzombsole_mi355x_diag<X>.so), one line each
for x in "" ${DIAGS:-1 2 4}; do
  lib=""; [ -n "$x" ] && lib="$PWD/libzombsole_amd/_build/libzombsole_mi355x_diag$x.so"
  echo "== diag '$x' ${CFG:-c3}"
  env ${lib:+ZS_ENGINE_LIB=$lib} timeout -k 10 120 python bench.py --config ${CFG:-c3} --steps 100 --warmup 10 --no-cpu-baseline > gpurun_out/e.json 2>/dev/null || exit 1
  python -c "import json;d=json.load(open('gpurun_out/e.json'));r=d['roofline'];print(d['ms_per_step'], r['step_launch_ms'], r['k_obs_ms'], r['k_reset_ms'])"
done
