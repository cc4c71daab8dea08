#!/usr/bin/env python3
"""Per-launch HBM traffic and SQ counters from a tools/gpu_pmc.sh run.

FETCH_SIZE / WRITE_SIZE are in KiB (MI355X_MICROARCH.md § HBM).  On gfx950 FETCH_SIZE reports
half the bytes of a coalesced streaming read; the calibration launch (tools/pmc_calib.py: known
read/write bytes, the same dword-per-lane access shape as observe_kernel) measures that factor
here and the traffic is corrected by it.  Writes are reported as counted.

    python tools/pmc_traffic.py gpurun_out/<tag> --batch 65536 --servers 4 --steps 20 --warmup 5
        [--out profiles/pmc_traffic.json]

Only the timed step launches are averaged (timed_positions), and the file records the workload
(steps, warm-up, pre-warm, the timed steps' reservoir slots per env-step): bench.py compares it
with its own run and marks the counters stale when the episode phase differs.
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
    if name.startswith("observe_pair"):  # observe_pair*_kernel<MODE, ...>
        return k.split("<", 1)[1].split(",")[0].rstrip(">").strip() == "0"
    if name not in ("dynamics_group_kernel", "dynamics_kernel", "dynamics_wave_kernel",
                    "observe_kernel"):
        return False
    targs = [x.strip() for x in k.split("<", 1)[1].rstrip(">").split(",")]
    return len(targs) > 1 and targs[1] == "0"


def timed_positions(n: int, steps: int, warmup: int):
    """Positions (in dispatch order) of the timed steps among the n step-mode dispatches of one
    kernel signature in a `bench.py --no-graph` run: the measured env runs W warm-up + K timed
    steps, then the accounting replay (bench.step_accounting: a twin env from the same seeds)
    runs the same W + K steps bit for bit, so the run ends with [W | K | W | K]; a pre-warm's
    scratch env (its own episode phase) comes before and is excluded.  The counters are then those
    of exactly the steps whose slots bench.py's accounting counts.  None if n < 2 (W + K)."""
    if not steps or n < 2 * (warmup + steps):
        return None
    base = n - 2 * (warmup + steps)
    first = range(base + warmup, base + warmup + steps)
    second = range(base + 2 * warmup + steps, base + 2 * (warmup + steps))
    return list(first) + list(second)


def load(d, sub, steps: int = 0, warmup: int = 0):
    """(kernel signature, counter) -> per-dispatch values.  With steps (K) and warmup (W), the
    step-mode kernels keep only the timed dispatches (timed_positions); other kernels keep all."""
    rows = collections.defaultdict(list)
    path = os.path.join(d, sub, "run_counter_collection.csv")
    if not os.path.exists(path):
        return collections.defaultdict(list)
    for r in csv.DictReader(open(path)):
        rows[(kernel_key(r["Kernel_Name"]), r["Counter_Name"])].append(
            (int(r["Dispatch_Id"]), float(r["Counter_Value"])))
    agg = collections.defaultdict(list)
    for key, v in rows.items():
        v.sort()
        vals = [x for _, x in v]
        pos = timed_positions(len(vals), steps, warmup) if is_step_kernel(key[0]) else None
        agg[key] = [vals[i] for i in pos] if pos is not None else vals
    return agg


def bench_workload(d, sub="fetch", steps: int = 0, warmup: int = 0):
    """The workload the counter passes ran: the bench JSON line of one pass's log (its timed
    steps' reservoir slots and flows per env-step -- the accounting the algorithmic bytes use),
    and which dispatches were kept."""
    out = {"steps": steps, "warmup": warmup,
           "dispatches": ("the K timed step launches and their exact replay (tools/pmc_traffic.py "
                          "timed_positions)" if steps else "every step-mode launch")}
    path = os.path.join(d, f"{sub}.log")
    if os.path.exists(path):
        for line in open(path):
            if line.startswith("{"):
                try:
                    j = json.loads(line)
                except ValueError:
                    continue
                acc = j.get("roofline", {}).get("accounting", {})
                out.update({"bench_steps": j.get("steps"), "bench_warmup": j.get("warmup"),
                            "prewarm": j.get("prewarm"),
                            "slots_per_env_step": acc.get("reservoir_slots_written_per_env_step"),
                            "flows_in_flight_per_env": acc.get("flows_in_flight_per_env")})
    return out


def mean(v):
    return sum(v) / len(v) if v else float("nan")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--batch", type=int, default=65536)
    ap.add_argument("--servers", type=int, default=4)
    ap.add_argument("--steps", type=int, default=20, help="bench --steps of the passes (K)")
    ap.add_argument("--warmup", type=int, default=5, help="bench --warmup of the passes (W)")
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    n = 1 << 21
    cal_read, cal_write = n * (2 * 512 + 4), n * 20
    cf, cw = load(a.dir, "calf"), load(a.dir, "calw")
    fetch_factor = mean(cf[("features_kernel", "FETCH_SIZE")]) * 1024 / cal_read
    write_factor = mean(cw[("features_kernel", "WRITE_SIZE")]) * 1024 / cal_write
    f, w = load(a.dir, "fetch", a.steps, a.warmup), load(a.dir, "write", a.steps, a.warmup)
    sq = {**load(a.dir, "sq1", a.steps, a.warmup), **load(a.dir, "sq2", a.steps, a.warmup)}
    S = a.servers
    # every step-mode launch of the run, keyed by its full template signature
    step = sorted({k for k, _ in f if is_step_kernel(k)})
    out = {"batch": a.batch, "servers": S, "fetch_calibration": fetch_factor,
           "write_calibration": write_factor,
           "workload": bench_workload(a.dir, "fetch", a.steps, a.warmup),
           "keys": "full template signature "
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
