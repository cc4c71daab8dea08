#!/usr/bin/env python3
"""Summarise a rocprofv3 --kernel-trace CSV: per-kernel calls / avg / min / max (us), with lbsim
launches split into step vs reset by grid size and duration class.  Usage:
    python tools/prof_summary.py gpurun_out/prof/bench_kernel_trace.csv [--timed K W] > profiles/<name>.md

--timed K W: also the table of bench.py's timed region alone.  A bench run launches, in time order,
[the pre-warm scratch env's reset, its steps] [the measured env's reset, W warm-up + K timed steps]
[the accounting twin's reset, the same W + K steps]; the first run of exactly W + K step launches
of a kernel after a reset launch is the measured env's, and its last K are the timed ones -- the
launches bench.py's HIP events average (the whole-trace table mixes in the pre-warm's steps, which
run earlier in their episode).
"""
import csv
import statistics
import sys
from collections import defaultdict


def short(name: str) -> str:
    name = name.replace("(anonymous namespace)::", "")
    for key in ("dynamics_kernel", "dynamics_group_kernel", "dynamics_wave_kernel",
                "observe_kernel", "observe_pair_kernel", "features_kernel", "reward_kernel",
                "fused_step_kernel",
                "step_wave_kernel", "step_stats_kernel", "vpp_"):
        if key in name:
            return (name.split("(")[0].replace("void ", "").replace("lbk::", "")
                    .replace("(anonymous namespace)::", ""))
    return name[:60]


def is_reset(k: str) -> bool:
    """Reset launches: MODE (second template argument) 1 of the dynamics / observe kernels."""
    if "<" not in k:
        return False
    name, args = k.split("<", 1)
    a = [x.strip() for x in args.rstrip(">").split(",")]
    if name.startswith("observe_pair"):  # observe_pair*_kernel<MODE, ...>
        return a[0] == "1"
    return name.startswith(("dynamics", "observe_kernel")) and len(a) > 1 and a[1] == "1"


def is_step(k: str) -> bool:
    return (k.startswith(("dynamics", "observe_kernel", "observe_pair", "step_wave_kernel",
                          "fused_step_kernel"))
            and not is_reset(k))


def table(title, d):
    print(f"## {title}\n")
    print("| kernel | grid | VGPR | LDS B | calls | avg us | median us | min us | max us |")
    print("|---|---|---|---|---|---|---|---|---|")
    for (k, g, v, l), ds in sorted(d.items(), key=lambda kv: -sum(kv[1])):
        print(f"| {k} | {g} | {v} | {l} | {len(ds)} | {statistics.mean(ds):.1f} | "
              f"{statistics.median(ds):.1f} | {min(ds):.1f} | {max(ds):.1f} |")
    print()


def main(path, timed=None):
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    d = defaultdict(list)
    for r in rows:
        dur = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
        d[(short(r["Kernel_Name"]), r["Grid_Size_X"], r["VGPR_Count"], r["LDS_Block_Size"])].append(dur)
    print(f"# kernel trace summary: {path}\n")
    table("all launches", d)
    if timed is None:
        return
    K, W = timed
    # segments of step launches between reset launches, per kernel key
    segs, cur = [], defaultdict(list)
    for r in rows:
        k = short(r["Kernel_Name"])
        if is_reset(k):
            if cur:
                segs.append(cur)
            cur = defaultdict(list)
        elif is_step(k):
            dur = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
            cur[(k, r["Grid_Size_X"], r["VGPR_Count"], r["LDS_Block_Size"])].append(dur)
    if cur:
        segs.append(cur)
    for seg in segs:
        if seg and all(len(v) == K + W for v in seg.values()):
            table(f"timed region: the last {K} of the measured env's {W} + {K} step launches",
                  {key: v[W:] for key, v in seg.items()})
            return
    print(f"(no segment of exactly {W} + {K} step launches per kernel)\n")


if __name__ == "__main__":
    args = sys.argv[1:]
    t = None
    if "--timed" in args:
        i = args.index("--timed")
        t = (int(args[i + 1]), int(args[i + 2]))
        del args[i:i + 3]
    main(args[0], t)
