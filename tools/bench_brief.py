#!/usr/bin/env python3
"""One-line summary of a bench.py JSON line (headline, phases, deviation, secondary blocks)."""
import json
import sys

d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
e = d.get("extra", {})
out = [f"value {d['value']} {d['unit']} ms/step {d['ms_per_step']}",
       f"mcd {e.get('mcd_phase_ms')} de {e.get('de_phase_ms')}"]
dev = e.get("fp32_deviation", {})
if dev:
    out.append(f"dev mcd {dev.get('mcd_batch_bn', {}).get('max_abs_dp')} de {dev.get('de_member_max_abs_dp')}")
for k in ("bf16", "running_bn", "train"):
    if k in e:
        v = e[k]
        out.append(f"{k}: " + json.dumps({a: b for a, b in v.items() if not isinstance(b, (dict, list))})[:400])
print("\n".join(out))
