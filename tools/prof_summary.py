#!/usr/bin/env python3
"""Summarise a rocprofv3 --kernel-trace CSV: per-kernel calls / avg / min / max (us), with lbsim
launches split into step vs reset by grid size and duration class.  Usage:
    python tools/prof_summary.py gpurun_out/prof/bench_kernel_trace.csv > profiles/<name>.md
"""
import csv
import statistics
import sys
from collections import defaultdict


def short(name: str) -> str:
    name = name.replace("(anonymous namespace)::", "")
    for key in ("dynamics_kernel", "dynamics_group_kernel", "observe_kernel", "features_kernel",
                "reward_kernel", "fused_step_kernel", "step_stats_kernel", "vpp_"):
        if key in name:
            return (name.split("(")[0].replace("void ", "").replace("lbk::", "")
                    .replace("(anonymous namespace)::", ""))
    return name[:60]


def main(path):
    rows = list(csv.DictReader(open(path)))
    d = defaultdict(list)
    for r in rows:
        dur = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
        d[(short(r["Kernel_Name"]), r["Grid_Size_X"], r["VGPR_Count"], r["LDS_Block_Size"])].append(dur)
    print(f"# kernel trace summary: {path}\n")
    print("| kernel | grid | VGPR | LDS B | calls | avg us | median us | min us | max us |")
    print("|---|---|---|---|---|---|---|---|---|")
    for (k, g, v, l), ds in sorted(d.items(), key=lambda kv: -sum(kv[1])):
        print(f"| {k} | {g} | {v} | {l} | {len(ds)} | {statistics.mean(ds):.1f} | "
              f"{statistics.median(ds):.1f} | {min(ds):.1f} | {max(ds):.1f} |")


if __name__ == "__main__":
    main(sys.argv[1])
