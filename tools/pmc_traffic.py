#!/usr/bin/env python3
"""Per-launch HBM traffic and SQ counters from a tools/gpu_pmc.sh run.

FETCH_SIZE / WRITE_SIZE are in KiB (MI355X_MICROARCH.md § HBM).  On gfx950 FETCH_SIZE reports
half the bytes of a coalesced streaming read; the calibration launch (tools/pmc_calib.py: known
read/write bytes, the same dword-per-lane access shape as observe_kernel) measures that factor
here and the traffic is corrected by it.  Writes are reported as counted.

    python tools/pmc_traffic.py gpurun_out/<tag> --batch 65536 --servers 4 [--out profiles/pmc_traffic.json]
"""
import argparse
import collections
import csv
import json
import os


def kernel_key(raw: str) -> str:
    """rocprofv3's Kernel_Name -> the template signature lbsim_launch_names reports
    ("observe_kernel<4, 0, false>"): bench.py matches counters to the kernels that ran by it."""
    k = raw
    depth = 0
    for i, ch in enumerate(k):  # cut the parameter list (the first '(' outside <>)
        if ch == "<":
            depth += 1
        elif ch == ">":
            depth -= 1
        elif ch == "(" and depth == 0 and not k.startswith("(anonymous namespace)", i):
            k = k[:i]
            break
    for pre in ("void ", "lbk::", "(anonymous namespace)::"):
        k = k.replace(pre, "")
    return k.strip()


def is_step_kernel(k: str) -> bool:
    """Launches of lbsim_step (reset launches carry the warm-up): MODE is the second template
    argument of dynamics_group_kernel / dynamics_kernel / dynamics_wave_kernel / observe_kernel;
    step_wave_kernel and fused_step_kernel are step launches."""
    name = k.split("<", 1)[0]
    if name in ("step_wave_kernel", "fused_step_kernel"):
        return True
    if name not in ("dynamics_group_kernel", "dynamics_kernel", "dynamics_wave_kernel",
                    "observe_kernel"):
        return False
    targs = [x.strip() for x in k.split("<", 1)[1].rstrip(">").split(",")]
    return len(targs) > 1 and targs[1] == "0"


def load(d, sub):
    agg = collections.defaultdict(list)
    path = os.path.join(d, sub, "run_counter_collection.csv")
    if not os.path.exists(path):
        return agg
    for r in csv.DictReader(open(path)):
        agg[(kernel_key(r["Kernel_Name"]), r["Counter_Name"])].append(float(r["Counter_Value"]))
    return agg


def mean(v):
    return sum(v) / len(v) if v else float("nan")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--batch", type=int, default=65536)
    ap.add_argument("--servers", type=int, default=4)
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    n = 1 << 21
    cal_read, cal_write = n * (2 * 512 + 4), n * 20
    cf, cw = load(a.dir, "calf"), load(a.dir, "calw")
    fetch_factor = mean(cf[("features_kernel", "FETCH_SIZE")]) * 1024 / cal_read
    write_factor = mean(cw[("features_kernel", "WRITE_SIZE")]) * 1024 / cal_write
    f, w = load(a.dir, "fetch"), load(a.dir, "write")
    sq = {**load(a.dir, "sq1"), **load(a.dir, "sq2")}
    S = a.servers
    # every step-mode launch of the run, keyed by its full template signature
    step = sorted({k for k, _ in f if is_step_kernel(k)})
    out = {"batch": a.batch, "servers": S, "fetch_calibration": fetch_factor,
           "write_calibration": write_factor, "keys": "full template signature "
           "(lbsim_launch_names / tools/pmc_traffic.py kernel_key)", "bytes_per_launch": {},
           "detail": {}}
    for kname in step:
        rd = mean(f[(kname, "FETCH_SIZE")]) * 1024 / fetch_factor
        wr = mean(w[(kname, "WRITE_SIZE")]) * 1024
        out["bytes_per_launch"][kname] = rd + wr
        det = {"read_bytes": rd, "write_bytes": wr,
               "read_bytes_per_env": rd / a.batch, "write_bytes_per_env": wr / a.batch}
        for (k, c), v in sq.items():
            if k == kname:
                det[c] = mean(v)
        out["detail"][kname] = det
    txt = json.dumps(out, indent=1)
    print(txt)
    if a.out:
        open(a.out, "w").write(txt + "\n")


if __name__ == "__main__":
    main()
