#!/usr/bin/env python3
"""Captured vs eager steps of the random-policy rollout on the same GPU state.

Fresh envs (65536 x 4, same seed) are stepped, in the order given by --order, through W warm-up
steps and then K timed steps (groups of --k steps; a group is one graph replay in graph mode),
each group bracketed by HIP events, plus the wall time over the timed steps.  Repeating the
sequence (--rounds) shows whether a mode is slower by itself or by its place in the run (GPU
state after sustained load).  One JSON line per (round, mode).

    python tools/graph_gap_exp.py [--order eager_same,eager_next,graph_next] [--rounds 2]
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def run(mode, B, S, k, warmup, steps, seed):
    import torch
    from marllb_amd.env import VecLoadBalanceEnv
    dev = torch.device("cuda", 0)
    graph = mode.startswith("graph")
    ar = "next_step" if mode.endswith("next") else "same_step"
    env = VecLoadBalanceEnv(B, S, device=dev, seed=seed, max_steps=10000, autoreset=True,
                            autoreset_mode=ar, graph_mode=graph)
    env.reset()
    gen = torch.Generator(device=dev)
    gen.manual_seed(seed + 1)
    if graph:
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
                env.step(torch.randint(0, 3, (B, S), device=dev, dtype=torch.int64,
                                       generator=gen))
    for _ in range(max(1, warmup // k)):
        group()
    torch.cuda.synchronize()
    n = max(1, steps // k)
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
          for _ in range(n)]
    t0 = time.perf_counter()
    for e0, e1 in ev:
        e0.record()
        group()
        e1.record()
    torch.cuda.synchronize()
    wall = time.perf_counter() - t0
    ms = sorted(e0.elapsed_time(e1) / k for e0, e1 in ev)
    env.close()
    torch.cuda.synchronize()
    return {"mode": mode, "median_ms_per_step": ms[len(ms) // 2], "min_ms_per_step": ms[0],
            "wall_ms_per_step": wall / (n * k) * 1e3}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=65536)
    ap.add_argument("--servers", type=int, default=4)
    ap.add_argument("--k", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--steps", type=int, default=30)
    ap.add_argument("--rounds", type=int, default=2)
    ap.add_argument("--order", default="eager_same,eager_next,graph_next")
    a = ap.parse_args()
    for r in range(a.rounds):
        for mode in a.order.split(","):
            res = run(mode, a.batch, a.servers, a.k, a.warmup, a.steps, 20260109)
            print(json.dumps({"round": r, "batch": a.batch, "servers": a.servers, **res}),
                  flush=True)


if __name__ == "__main__":
    main()
