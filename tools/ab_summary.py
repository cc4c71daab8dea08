"""Summarise an A/B jsonl written by tools/gpu_lib_ab.sh / gpu_obs_ab.sh: value and kernel times."""
import json
import sys

for line in open(sys.argv[1]):
    if line.startswith("=="):
        print(line.strip())
        continue
    try:
        d = json.loads(line)
    except ValueError:
        continue
    r = d["roofline"]
    ks = " ".join(f"{k}={v * 1e3:.1f}us" for k, v in r["kernel_avg_ms"].items())
    pol = d.get("policy_ms_per_step")
    ks += f" policy={pol * 1e3:.1f}us" if pol is not None else ""
    print(f"  {d['value'] / 1e6:.1f} M/s  {d['ms_per_step'] * 1e3:.1f} us/step  {ks}")
