"""Print the headline and every sub-line of a bench.py JSON line (value, step, roofline frac, CPU baseline)."""
import json
import sys


def line(name, d):
    rf = d.get("roofline") or {}
    cpu = (d.get("cpu_baseline") or {}).get("value")
    extra = ""
    if "executed_gflop_per_step" in d:
        extra = f" e2e {d.get('e2e_frac_algorithmic')}/{d.get('e2e_frac_executed')}"
    print(f"{name:14s} {d['value']:>12} {d['unit']:9s} {d.get('ms_per_step')} ms  dtype {d.get('dtype')}  "
          f"roofline {rf.get('kernel', '')[:60]!r} frac {rf.get('frac')}  cpu {cpu}{extra}")


d = json.load(open(sys.argv[1]))
line("headline", d)
for k, v in d.items():
    if isinstance(v, dict) and "value" in v and "metric" in v:
        line(k, v)
