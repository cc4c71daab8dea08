#!/usr/bin/env python3
"""Table of a tools/gpu_ab.sh run: per (args, variant), the mean HIP-event kernel times and rate."""
import collections
import json
import sys

rows = collections.defaultdict(list)
cur = None
for line in open(sys.argv[1]):
    line = line.strip()
    if not line.startswith("{"):
        continue
    d = json.loads(line)
    if "variant" in d:
        cur = (d["args"], d["variant"])
        continue
    rows[cur].append(d)
for (args, var), ds in sorted(rows.items()):
    ks = collections.defaultdict(list)
    for d in ds:
        for k, v in d["roofline"]["kernel_avg_ms"].items():
            ks[k].append(v)
    rate = sum(d["value"] for d in ds) / len(ds) / 1e6
    kt = " ".join(f"{k.replace('_kernel', '')}={min(v):.4f}/{sum(v) / len(v):.4f}" for k, v in ks.items())
    print(f"{args:40s} {var:10s} {rate:8.1f}M  {kt}")
