"""Print a sweep.jsonl (bench lines) as a table: mapping, batch x servers, rate, kernel times."""
import json
import sys

for line in open(sys.argv[1]):
    if not line.startswith("{"):
        continue
    d = json.loads(line)
    c, k = d["config"], d["roofline"]["kernel_avg_ms"]
    print(f"{c.get('dyn_mapping', '?'):6s} {c['envs_per_gpu']:6d}x{c['servers']:<2d} "
          f"{d['value'] / 1e6:7.2f}M  step {d['ms_per_step']:.3f}  "
          f"dyn {k.get('dynamics_group_kernel', k.get('dynamics_kernel', 0)):.3f}  "
          f"obs {k.get('observe_pair_kernel', k.get('observe_kernel', 0)):.3f}  "
          f"one-launch {k.get('step_wave_kernel', 0):.3f}")
