cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
for c in FETCH_SIZE WRITE_SIZE; do
timeout -s KILL 120 rocprofv3 --pmc $c -T --output-format csv -d $PWD/gpurun_out/tickio_$c -o run -- ./tools/probe/tickio > gpurun_out/tickio_$c.log 2>&1 || exit 1
done
python3 - <<'PY'
import csv, glob
for c in ("FETCH_SIZE", "WRITE_SIZE"):
    vals = {}
    for f in glob.glob("gpurun_out/tickio_%s/**/*counter_collection.csv" % c, recursive=True):
        for row in csv.DictReader(open(f)):
            if "k_tick_io" in row["Kernel_Name"]:
                vals.setdefault(row["Dispatch_Id"], 0.0)
                vals[row["Dispatch_Id"]] += float(row["Counter_Value"])
    print(c, [round(v) for k, v in sorted(vals.items(), key=lambda kv: int(kv[0]))])
PY
head -3 gpurun_out/tickio_FETCH_SIZE.log | tail -1; grep "k_tick_io read" gpurun_out/tickio_*.log
