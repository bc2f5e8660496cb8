# parity of the observation paths, then C3 / C5 bench lines at several k_obs_lds workgroup counts
set -o pipefail
timeout -k 10 400 python -u -m pytest tests/test_fullsize_parity.py tests/test_engine_oracle.py -k "c3_65536_graph or c5_65536 or one_obs_workgroup or store_stream or obs_lds or obs_pipe" -x -q --timeout 200 --timeout-method thread > gpurun_out/t3.log 2>&1 || { tail -30 gpurun_out/t3.log; exit 1; }
tail -2 gpurun_out/t3.log
for cfg in ${CFGS:-c3}; do
for v in ${WGSS:-2 3 4}; do
  echo "== $cfg ZS_OBS_WGS=$v"; ZS_OBS_WGS=$v timeout -k 10 120 python bench.py --config $cfg --steps 100 --warmup 10 --no-cpu-baseline > gpurun_out/e.json 2>/dev/null || exit 1
  python -c "import json;d=json.load(open('gpurun_out/e.json'));r=d['roofline'];print(d['ms_per_step'], r['step_launch_ms'], r['k_obs_ms'], r['k_reset_ms'])"
done
done
