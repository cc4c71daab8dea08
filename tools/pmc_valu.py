#!/usr/bin/env python3
"""Per-launch VALU accounting of the simulator kernels from a tools/gpu_pmc.sh run.

SQ counters (sq1, sq2: totals, wave cycles, waits; vc1, vc2: VALU instructions per op class) and
the VALU issue micro-benchmark (ubench_valu.jsonl: SIMD cycles per instruction of each class with
4 waves per SIMD, independent chains) give, per kernel launch:

  valu_per_env_step       SQ_INSTS_VALU / envs
  classes                 per-class instruction counts (INT32, INT64, F32 add/mul/fma, F64
                          add/mul/fma, TRANS_F32, CVT, other = total - classes)
  issue_cycles            sum over classes of count x measured SIMD cycles per instruction
  issue_bound_ms          issue_cycles / (SIMDs x clock): the kernel's time if the SIMDs issued
                          VALU back to back at the measured rates
  wait_any_share          SQ_WAIT_ANY / SQ_WAVE_CYCLES (waves parked on s_waitcnt / barriers)
  active_valu_per_simd_quad  SQ_ACTIVE_INST_VALU / (GRBM_GUI_ACTIVE / 8 XCDs / 4 x SIMDs):
                          VALU quad-cycles per SIMD quad-cycle (the 'VALUBusy' basis per SIMD;
                          a SIMD dual-issues VALU from two waves, so the ceiling is 2, not 1).
                          GRBM_GUI_ACTIVE comes summed over the 8 XCDs (8 x the kernel's cycles)

    python tools/pmc_valu.py gpurun_out/<tag> --batch 65536 --servers 4 [--out profiles/pmc_valu.json]
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from pmc_traffic import bench_workload, is_step_kernel, load  # noqa: E402

CLOCK_HZ = 2.4e9  # MI355X peak engine clock (MI355X_MICROARCH.md)
SIMDS = 1024      # 256 CUs x 4
XCDS = 8

# counter -> ubench_valu op whose measured throughput prices it
PRICE = {"SQ_INSTS_VALU_INT32": "v_add_u32", "SQ_INSTS_VALU_ADD_F32": "v_fma_f32",
         "SQ_INSTS_VALU_MUL_F32": "v_fma_f32", "SQ_INSTS_VALU_FMA_F32": "v_fma_f32",
         "SQ_INSTS_VALU_ADD_F64": "v_add_f64", "SQ_INSTS_VALU_MUL_F64": "v_mul_f64",
         "SQ_INSTS_VALU_FMA_F64": "v_fma_f64", "SQ_INSTS_VALU_TRANS_F32": "v_exp_f32",
         "SQ_INSTS_VALU_INT64": "v_lshlrev_b64+pack", "SQ_INSTS_VALU_CVT": None,
         "other": "v_add_u32"}
# ops of the micro-benchmark that issue two VALU instructions per counted step
PAIRS = {"v_mad_u64_u32+xor", "v_mov_dpp+add", "v_cvt_f64_f32+v_cvt_f32_f64", "v_lshlrev_b64+pack"}


def mean(v):
    return sum(v) / len(v) if v else float("nan")


def ubench_costs(d, waves=4):
    """SIMD cycles per instruction at `waves` waves per SIMD, 8 independent chains."""
    cost = {}
    path = os.path.join(d, "ubench_valu.jsonl")
    for line in open(path):
        r = json.loads(line)
        if r["waves_per_simd"] == waves and r["chains"] == 8:
            c = r["simd_cyc_per_inst"]
            cost[r["op"]] = c / 2 if r["op"] in PAIRS else c
    return cost


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--batch", type=int, default=65536)
    ap.add_argument("--servers", type=int, default=4)
    ap.add_argument("--waves", type=int, default=4, help="ubench occupancy used for the prices")
    ap.add_argument("--steps", type=int, default=20, help="bench --steps of the passes (K)")
    ap.add_argument("--warmup", type=int, default=5, help="bench --warmup of the passes (W)")
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    cost = ubench_costs(a.dir, a.waves)
    cost["v_cvt"] = cost.get("v_cvt_f64_f32+v_cvt_f32_f64")
    agg = {}
    for sub in ("sq1", "sq2", "vc1", "vc2"):
        agg.update(load(a.dir, sub, a.steps, a.warmup))
    kernels = sorted({k for k, _ in agg if is_step_kernel(k)})
    out = {"batch": a.batch, "servers": a.servers,
           "workload": bench_workload(a.dir, "sq1", a.steps, a.warmup),
           "clock_hz": CLOCK_HZ, "simds": SIMDS,
           "ubench_waves_per_simd": a.waves, "ubench_simd_cyc_per_inst": cost, "kernels": {}}
    for k in kernels:  # keyed by the full template signature (lbsim_launch_names)
        c = {cn: mean(v) for (kn, cn), v in agg.items() if kn == k}
        if "SQ_INSTS_VALU" not in c:
            continue
        cls = {n: c.get(n, 0.0) for n in PRICE if n != "other"}
        cls["other"] = max(0.0, c["SQ_INSTS_VALU"] - sum(cls.values()))
        cyc = 0.0
        for n, v in cls.items():
            op = PRICE[n] if PRICE[n] is not None else "v_cvt"
            cyc += v * cost.get(op, cost["v_add_u32"])
        gui = c.get("GRBM_GUI_ACTIVE", float("nan"))
        rec = {
            "valu_per_launch": c["SQ_INSTS_VALU"],
            "valu_per_env_step": c["SQ_INSTS_VALU"] / a.batch,
            "classes_per_env_step": {n: v / a.batch for n, v in cls.items()},
            "issue_cycles_per_launch": cyc,
            "issue_bound_ms": cyc / (SIMDS * CLOCK_HZ) * 1e3,
            "wait_any_share": c.get("SQ_WAIT_ANY", float("nan")) / c.get("SQ_WAVE_CYCLES", float("nan")),
            "wait_inst_any_share": c.get("SQ_WAIT_INST_ANY", float("nan")) / c.get("SQ_WAVE_CYCLES", float("nan")),
            "active_valu_per_simd_quad": c.get("SQ_ACTIVE_INST_VALU", float("nan")) / (gui / XCDS / 4 * SIMDS),
            "valu2_quads_share": c.get("SQ_ACTIVE_INST_VALU2", float("nan")) / c.get("SQ_ACTIVE_INST_VALU", float("nan")),
            "gui_active_ms": gui / XCDS / CLOCK_HZ * 1e3,
            "issue_frac_of_gui": cyc / (SIMDS * gui / XCDS),
            "counters": c,
        }
        out["kernels"][k] = rec
    txt = json.dumps(out, indent=1)
    print(txt)
    if a.out:
        open(a.out, "w").write(txt + "\n")


if __name__ == "__main__":
    main()
