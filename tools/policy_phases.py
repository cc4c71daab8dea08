#!/usr/bin/env python3
"""Phase timeline of the policy kernels (timing diagnostic): with the LBSIM_EXP_PHASES=1 build
(`python -m marllb_amd.build --variant phases --only pol.o -DLBSIM_EXP_PHASES=1`, loaded through
LBSIM_LIBRARY) every gridDim/64-th workgroup of a policy launch stamps the 100 MHz clock at its
phase boundaries (lbsim_fused.h LB_PHASE).  Steps the SAC-GRU (65536 x 8) or QMIX (8192 x 4x4)
rollout as bench.py does, then prints one JSON line: per phase the median over the sampled
workgroups of the time since the previous phase (us), the median workgroup span, and the launch's
first-start-to-last-end span.

    LBSIM_LIBRARY=marllb_amd/exp/liblbsim_phases.so python tools/policy_phases.py --workload qmix
"""
import argparse
import ctypes
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

NAMES = {"sac-gru": ["start", "staged_local", "staged", "gru_mma", "gru_stored", "fc1_mma",
                     "fc1_stored", "heads", "sample"],
         "qmix": ["start", "staged_local", "staged", "gru", "gru_stored", "fc1", "fc2", "fc3",
                  "eps_greedy", "mix_l1", "mix_l2", "mix_tail"]}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", choices=["sac-gru", "qmix"], default="qmix")
    ap.add_argument("--steps", type=int, default=12)
    a = ap.parse_args()
    import numpy as np
    import torch

    from marllb_amd import _lib
    from marllb_amd.env import VecLoadBalanceEnv
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    if a.workload == "sac-gru":
        from marllb_amd.rollout import SACGRURollout
        env = VecLoadBalanceEnv(65536, 8, action_type="continuous", max_steps=10000, seed=1,
                                device=dev)
        ro = SACGRURollout(env, seed=1)
    else:
        from marllb_amd.multi_agent import VecMultiAgentLoadBalanceEnv
        from marllb_amd.rollout import QMIXRollout
        env = VecMultiAgentLoadBalanceEnv(8192, 4, 4, action_type="discrete", max_steps=100,
                                          seed=1, device=dev)
        ro = QMIXRollout(env, seed=1)
    out = {"workload": a.workload, "unit": "us", "steps": []}
    lib = _lib.load()
    buf = (ctypes.c_ulonglong * (64 * 16))()
    names = NAMES[a.workload]
    n = len(names)
    for k in range(a.steps):
        ro.step()
        torch.cuda.synchronize()
        if k < a.steps - 3:
            continue
        if lib.lbsim_exp_phase_read(buf) != 0:
            raise SystemExit("lbsim_exp_phase_read failed (not the LBSIM_EXP_PHASES build?)")
        ts = np.frombuffer(buf, dtype=np.uint64).reshape(64, 16)[:, :n].astype(np.int64)
        ok = (ts > 0).all(axis=1)
        ts = ts[ok]
        d = np.diff(ts, axis=1) / 100.0  # 100 MHz ticks -> us
        out["steps"].append({
            "phases_median_us": {names[i + 1]: float(np.median(d[:, i])) for i in range(n - 1)},
            "workgroup_span_median_us": float(np.median((ts[:, -1] - ts[:, 0]) / 100.0)),
            "launch_span_us": float((ts[:, -1].max() - ts[:, 0].min()) / 100.0),
            "start_spread_us": float((ts[:, 0].max() - ts[:, 0].min()) / 100.0),
            "samples": int(ok.sum())})
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
