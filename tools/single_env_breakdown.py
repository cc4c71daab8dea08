#!/usr/bin/env python3
"""Where the single-env drop-in step's time goes (LoadBalanceEnv.step, problem-04 Trainer path):
the facade step, the bare lbsim_step_ex + stream sync with device-resident actions, the same plus
the device->host copy, the sync floor of one tiny launch, and the per-kernel HIP-event times
(lbsim_profile).  One JSON line, us per step.

    python tools/single_env_breakdown.py [--steps 2000] [--servers 4]
"""
import argparse
import ctypes
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=2000)
    ap.add_argument("--servers", type=int, default=4)
    ap.add_argument("--arrival-rate", type=float, default=400.0)
    args = ap.parse_args()
    import numpy as np
    import torch

    from marllb_amd import LoadBalanceEnv, _lib
    S, K = args.servers, args.steps
    env = LoadBalanceEnv(num_servers=S, max_steps=10**9, seed=1, step_interval=0.0,
                         arrival_rate=args.arrival_rate)
    rng = np.random.default_rng(0)
    acts = [rng.integers(0, 3, S) for _ in range(256)]
    out = {"servers": S, "steps": K, "unit": "us/step", "arrival_rate": args.arrival_rate}

    def per_step(fn, k=K):
        for i in range(50):
            fn(i)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for i in range(k):
            fn(i)
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) / k * 1e6

    env.reset()
    out["facade_step"] = per_step(lambda i: env.step(acts[i % 256]))
    v = env._vec
    host, hview, act_h, aview, done_h, so, cur, sptr, dt, n = env._io_buffers()[:10]
    lib, h = v.handle.lib, v.handle.h
    act_d = torch.zeros(S, dtype=torch.int64, device=v.device)
    dev = torch.zeros(2 * n + 2, dtype=torch.float32, device=v.device)
    sd = _lib.StepOutputs()  # device-resident outputs
    base = dev.data_ptr()
    sd.obs, sd.raw_obs, sd.reward = base, base + 4 * n, base + 8 * n
    done_d = torch.zeros(8, dtype=torch.uint8, device=v.device)
    sd.done = done_d.data_ptr()
    stream = sptr

    def bare(i):  # device-resident action and outputs
        lib.lbsim_step_ex(h, act_d.data_ptr(), _lib.DTYPE_I64, ctypes.byref(sd), stream)
        cur.synchronize()
    out["step_ex_sync"] = per_step(bare)

    def bare_copy(i):
        lib.lbsim_step_ex(h, act_d.data_ptr(), _lib.DTYPE_I64, ctypes.byref(sd), stream)
        host.copy_(dev, non_blocking=True)
        cur.synchronize()
    out["step_ex_copy_sync"] = per_step(bare_copy)

    def zero_copy(i):  # the facade's form: pinned host action and outputs
        lib.lbsim_step_ex(h, act_h.data_ptr(), _lib.DTYPE_I64, ctypes.byref(so), stream)
        cur.synchronize()
    out["step_ex_zero_copy_sync"] = per_step(zero_copy)

    def launches_only(i):
        lib.lbsim_step_ex(h, act_d.data_ptr(), _lib.DTYPE_I64, ctypes.byref(sd), stream)
    out["step_ex_enqueue_only"] = per_step(launches_only)

    x = torch.zeros(1, device=v.device)

    def floor(i):
        x.add_(1.0)
        cur.synchronize()
    out["tiny_launch_sync"] = per_step(floor)

    # per-kernel HIP-event times of the bare step
    v.handle.check(lib.lbsim_profile_begin(h, 4 * 500 + 8))
    for i in range(500):
        lib.lbsim_step_ex(h, act_d.data_ptr(), _lib.DTYPE_I64, ctypes.byref(sd), stream)
    ms = (ctypes.c_double * 5)()
    cnt = (ctypes.c_int64 * 5)()
    v.handle.check(lib.lbsim_profile_end_ex(h, ms, cnt, 5))
    out["kernel_us"] = {name: (ms[i] / max(cnt[i], 1) * 1e3) for i, name in
                        enumerate(("dynamics", "observe", "dynamics_reset", "observe_reset",
                                   "one_launch_step")) if cnt[i] > 0}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
