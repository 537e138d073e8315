"""Print the headline figures of bench.py JSON lines (one log file per argument)."""
import json
import sys

for f in sys.argv[1:]:
    lines = [l for l in open(f) if l.startswith("{")]
    if not lines:
        print(f, "no JSON line")
        continue
    d = json.loads(lines[-1])
    r = d.get("roofline") or {}
    t = d.get("encoder_trunk") or {}
    print(f"{f}: {d['value']} img/s, {d['ms_per_step']} ms/step, B={d['config']['per_gpu_batch']}")
    print("  roofline", {k: r.get(k) for k in ("cls", "avg_launch_us", "frac", "avg_launch_us_overlapped",
                                                "frac_overlapped", "avg_launch_us_b2b")})
    print("  trunk", {k: t.get(k) for k in ("conv_us_per_forward", "conv_us_per_forward_overlapped", "frac_of_floor", "graph_ms_per_step")})
    for k, v in list((t.get("classes") or {}).items())[:6]:
        print("   ", k, v)
    ds = r.get("decoder_step_kernels")
    if ds:
        for g, v in ds["groups"].items():
            print("   ", g, v)
        print("  fused", ds["fused_attention_lstm"])
        print("  all", ds["all_step_kernels"])
        if ds.get("step_chain"):
            print("  chain", {k: v for k, v in ds["step_chain"].items() if k != "note"})
    if d.get("decoder_graphs_ms_per_step"):
        print("  decoder graphs ms/step", d["decoder_graphs_ms_per_step"])
