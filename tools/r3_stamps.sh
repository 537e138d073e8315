# in-step stamps vs rocprof on the same bench command
set -u
OUT=gpurun_out/r3_s7; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 300 python bench.py --steps 100 --no-cpu-baseline --fp32-steps 0 > $OUT/bench.log 2>&1 || { tail -30 $OUT/bench.log; exit 1; }
timeout -k 10 300 python bench.py --steps 100 --no-cpu-baseline --fp32-steps 0 --no-step-stamps --no-diagnostics > $OUT/bench_nostamp.log 2>&1 || { tail -30 $OUT/bench_nostamp.log; exit 1; }
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python bench.py --steps 100 --warmup 1 --no-cpu-baseline --fp32-steps 0 --no-diagnostics > $OUT/prof.log 2>&1 || { tail -30 $OUT/prof.log; exit 1; }
python - <<'PY'
import json, glob, csv
out = "gpurun_out/r3_s7"
for f in ("bench", "bench_nostamp"):
    d = json.loads([l for l in open(f"{out}/{f}.log") if l.startswith("{")][-1])
    r = d.get("roofline") or {}
    print(f, d["ms_per_step"], r.get("cls"), r.get("avg_launch_us"), r.get("frac"), r.get("avg_launch_us_b2b"))
    if f == "bench":
        print(json.dumps(d["encoder_trunk"]["classes"])[:1500])
        print(json.dumps(r["decoder_step_kernels"]))
st = glob.glob(f"{out}/prof/**/*kernel_stats.csv", recursive=True)
for row in csv.DictReader(open(st[0])):
    if any(k in row["Name"] for k in ("conv3x3_frag", "conv1x1_frag", "conv1x1_stream", "attn_", "lstm_")):
        print(row["Name"][:70], row["Calls"], row["AverageNs"])
PY
