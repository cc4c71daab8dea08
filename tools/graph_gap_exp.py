#!/usr/bin/env python3
"""Does a captured step run slower than the eager one because of the launches, or because the
GPU runs the kernels back to back?  The random-policy rollout (65536 x 4, next-step auto-reset)
captured K steps per torch.cuda.CUDAGraph; each replay timed with HIP events (a) back to back,
(b) with the GPU idle for --idle-ms between replays, and (c) the same K steps eager with events
around them, both ways.  JSON line per mode: ms per step of the replays / eager groups.

    python tools/graph_gap_exp.py [--batch 65536] [--k 5] [--reps 40] [--idle-ms 2]
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch
    from marllb_amd.env import VecLoadBalanceEnv
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=65536)
    ap.add_argument("--servers", type=int, default=4)
    ap.add_argument("--k", type=int, default=5)
    ap.add_argument("--reps", type=int, default=40)
    ap.add_argument("--idle-ms", type=float, default=2.0)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    B, S, k = a.batch, a.servers, a.k
    out = {}
    for mode in ("graph", "eager"):
        env = VecLoadBalanceEnv(B, S, device=dev, seed=7, max_steps=10000, autoreset=True,
                                autoreset_mode="next_step", graph_mode=(mode == "graph"))
        env.reset()
        gen = torch.Generator(device=dev)
        gen.manual_seed(11)

        def step():
            env.step(torch.randint(0, 3, (B, S), device=dev, dtype=torch.int64, generator=gen))
        if mode == "graph":
            side = torch.cuda.Stream(dev)
            side.wait_stream(torch.cuda.current_stream(dev))
            with torch.cuda.stream(side):
                for _ in range(2):
                    env.step(torch.randint(0, 3, (B, S), device=dev, dtype=torch.int64))
            torch.cuda.current_stream(dev).wait_stream(side)
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g):
                for _ in range(k):
                    env.step(torch.randint(0, 3, (B, S), device=dev, dtype=torch.int64))
            group = g.replay
        else:
            def group():
                for _ in range(k):
                    step()
        for _ in range(4):
            group()
        torch.cuda.synchronize()
        for idle in (0.0, a.idle_ms):
            ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
                  for _ in range(a.reps)]
            t0 = time.perf_counter()
            for e0, e1 in ev:
                e0.record()
                group()
                e1.record()
                if idle > 0:
                    torch.cuda.synchronize()
                    time.sleep(idle * 1e-3)
            torch.cuda.synchronize()
            wall = time.perf_counter() - t0
            ms = sorted(e0.elapsed_time(e1) / k for e0, e1 in ev)
            out[f"{mode}_idle{idle:g}ms"] = {"median_ms_per_step": ms[len(ms) // 2],
                                            "min_ms_per_step": ms[0],
                                            "wall_ms_per_step": wall / (a.reps * k) * 1e3}
        env.close()
    print(json.dumps({"batch": B, "servers": S, "steps_per_group": k, "reps": a.reps,
                      "idle_ms": a.idle_ms, "modes": out}))


if __name__ == "__main__":
    main()
