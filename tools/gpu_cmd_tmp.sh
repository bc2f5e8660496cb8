cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
for cfg in "c3:--config c3:k_gen_actions_ctr" "n8:--envs 8192:k_step" "c5:--config c5:k_gen_actions_ctr"; do n=${cfg%%:*}; r=${cfg#*:}; a=${r%%:*}; k=${r#*:}
timeout -k 10 300 rocprofv3 --kernel-trace -T --output-format csv -d $PWD/gpurun_out/trace_$n -o run -- python3 bench.py $a --steps 60 --warmup 10 --no-cpu-baseline > gpurun_out/trace_$n.log 2>&1 || exit 1
python3 tools/trace_steps.py gpurun_out/trace_$n $k 30 > gpurun_out/trace_$n.txt 2>&1
done
tail -12 gpurun_out/trace_*.txt
