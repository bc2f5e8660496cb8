cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
P=$PWD/gpurun_out/round/r02b/prof_c4
mkdir -p $P
B="bench.py --config c4 --steps 50 --warmup 10 --no-cpu-baseline"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T --output-format csv -d "$P/kt" -o run -- python3 $B > "$P/kt.log" 2>&1 || exit 1
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 300 rocprofv3 --pmc $c -T --output-format csv -d "$P/$c" -o run -- python3 $B > "$P/$c.log" 2>&1 || exit 1
done
timeout -k 10 180 python bench.py --config c4 --steps 200 --warmup 20 --no-cpu-baseline > gpurun_out/round/r02b/bench_c4.log 2>&1 || exit 1
echo done
