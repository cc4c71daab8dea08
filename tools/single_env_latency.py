#!/usr/bin/env python3
"""Latency of the single-env drop-in step (problem-04 Trainer path, env.py:215-286 on the facade):
µs per LoadBalanceEnv.step on the GPU simulator (one launch pair + one device->host copy per step),
beside the reference-plumbing mode (host-only restatement of the reference's simulation step) and
the survey's recorded figure for the reference itself (122.5 µs/step, different host).

    python tools/single_env_latency.py [--steps 2000] [--servers 4]   -> one JSON line
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def timed(env, acts, steps):
    env.reset()
    for a in acts[:50]:
        env.step(a)
    t0 = time.perf_counter()
    for k in range(steps):
        env.step(acts[k % len(acts)])
    return (time.perf_counter() - t0) / steps * 1e6


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=2000)
    ap.add_argument("--servers", type=int, default=4)
    ap.add_argument("--dyn-mapping", default="auto", choices=["auto", "env", "server"])
    args = ap.parse_args()
    import numpy as np
    import torch

    from marllb_amd import LoadBalanceEnv
    S = args.servers
    rng = np.random.default_rng(0)
    disc = [rng.integers(0, 3, S) for _ in range(256)]
    cont = [rng.uniform(-1, 1, S).astype(np.float32) for _ in range(256)]
    out = {"servers": S, "steps": args.steps, "unit": "us/step", "dyn_mapping": args.dyn_mapping}
    dm = {"dyn_mapping": args.dyn_mapping}
    if torch.cuda.is_available():
        out["gpu_discrete"] = timed(LoadBalanceEnv(num_servers=S, max_steps=10**9, seed=1,
                                                   step_interval=0.0, **dm), disc, args.steps)
        out["gpu_continuous_normalized"] = timed(
            LoadBalanceEnv(num_servers=S, action_type="continuous", normalize_obs=True,
                           max_steps=10**9, seed=1, step_interval=0.0, **dm), cont, args.steps)
    out["reference_plumbing_host"] = timed(
        LoadBalanceEnv(num_servers=S, max_steps=10**9, seed=1, step_interval=0.0,
                       reference_plumbing=True), disc, args.steps)
    out["reference_recorded_different_host"] = 122.5  # SURVEY §6 (S=4, step_interval=0)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
