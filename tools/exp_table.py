#!/usr/bin/env python3
"""Table of a gpu_exp.sh / gpu_quick.sh JSONL: variant, config, env-steps/s, per-kernel ms."""
import json
import sys

var = "-"
for line in open(sys.argv[1]):
    d = json.loads(line)
    if "variant" in d:
        var = d["variant"] + ("" if "round" not in d else f"/{d['round']}")
        continue
    c = d["config"]
    k = d["roofline"]["kernel_avg_ms"]
    print(f"{var:8s} {c['envs_per_gpu']:7d}x{c['servers']:<3d} {c.get('dyn_mapping', '-'):6s} "
          f"{d['value'] / 1e6:8.2f} M/s  " + "  ".join(f"{a.replace('_kernel', '')} {b:.4f}" for a, b in k.items()))
