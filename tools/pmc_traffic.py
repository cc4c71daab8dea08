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


def load(d, sub):
    agg = collections.defaultdict(list)
    path = os.path.join(d, sub, "run_counter_collection.csv")
    if not os.path.exists(path):
        return agg
    for r in csv.DictReader(open(path)):
        k = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("lbk::", "")
        agg[(k, r["Counter_Name"])].append(float(r["Counter_Value"]))
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
    m = 4 if S <= 4 else 8 if S <= 8 else 16
    g = 2 if S <= 2 else m if S <= 16 else 32 if S <= 32 else 64
    # step-mode launches: dynamics_group_kernel<G, 0, POLICY, TRACE> (default mapping) or
    # dynamics_kernel<MAXS, 0, POLICY, TRACE> (env per lane), observe_kernel<MAXS, 0>
    prefixes = {"dynamics_group_kernel": f"dynamics_group_kernel<{g}, 0",
                "dynamics_kernel": f"dynamics_kernel<{m}, 0", "observe_kernel": f"observe_kernel<{m}, 0"}
    prefixes = {n: pfx for n, pfx in prefixes.items()
                if any(k.startswith(pfx) for k, _ in load(a.dir, "fetch"))}

    def match(agg, prefix):
        names = sorted({k for k, _ in agg if k.startswith(prefix)})
        return names[0] if names else prefix

    step = {n: match(load(a.dir, "fetch"), pfx) for n, pfx in prefixes.items()}
    out = {"batch": a.batch, "servers": S, "fetch_calibration": fetch_factor,
           "write_calibration": write_factor, "bytes_per_launch": {}, "detail": {}}
    for name, kname in step.items():
        rd = mean(f[(kname, "FETCH_SIZE")]) * 1024 / fetch_factor
        wr = mean(w[(kname, "WRITE_SIZE")]) * 1024
        out["bytes_per_launch"][name] = rd + wr
        det = {"read_bytes": rd, "write_bytes": wr,
               "read_bytes_per_env": rd / a.batch, "write_bytes_per_env": wr / a.batch}
        for (k, c), v in sq.items():
            if k == kname:
                det[c] = mean(v)
        out["detail"][name] = det
    txt = json.dumps(out, indent=1)
    print(txt)
    if a.out:
        open(a.out, "w").write(txt + "\n")


if __name__ == "__main__":
    main()
