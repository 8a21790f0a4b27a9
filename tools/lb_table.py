"""Summarise loopback sweep JSONL files: one row per run (bin, shape, env) with
echoes/s, the pass timeline and per-loop fairness."""
import json
import sys

for path in sys.argv[1:]:
    for line in open(path):
        d = json.loads(line)
        t = d.get("pass_timeline_us") or {}
        shape = f"{d['connections']}c/{d['loops']}l/{d.get('mode')}"
        env = d.get("env", "")
        env = "" if env in ("", "GEVWS_NOP=1") else env.split("=")[-1]
        print(f"{d['bin'].split('/')[-1]:16s} {shape:18s} {env:5s} {d['echoes_per_s']:>10.0f}  conns/pass {d['mean_conns_per_pass']:6.1f}"
              f"  sel {t.get('select', 0):5.1f} stg {t.get('stage', 0):5.1f} lch {t.get('launch', 0):5.1f}"
              f" wait {t.get('wait', 0):6.1f} dlv {t.get('deliver', 0):5.1f} sig {t.get('signalled_share', 0):.3f}"
              f" gpu {t.get('gpu_decode', 0):5.1f}  fair {d.get("loop_min_over_max_per_conn", d.get("loop_min_over_max", 0)):.2f}")
