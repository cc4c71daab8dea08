"""Experiment: the headline batch (65536 x 4) as P handles of B/P envs stepped on P HIP streams
(global env ids kept: handle i owns [i B/P, (i+1) B/P)), so the latency-bound dynamics launch of
one part can overlap the VALU-bound observe launch of another.  Prints one JSON line per P.

usage: python tools/stream_split_exp.py [--batch 65536] [--servers 4] [--steps 50] [--parts 1,2,4]
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=65536)
    ap.add_argument("--servers", type=int, default=4)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--parts", default="1,2,4")
    args = ap.parse_args()
    import torch
    from marllb_amd.env import VecLoadBalanceEnv
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(0)
    for P in [int(x) for x in args.parts.split(",")]:
        b = args.batch // P
        S = args.servers
        streams = [torch.cuda.Stream(dev) for _ in range(P)]
        envs, gens = [], []
        for i in range(P):
            with torch.cuda.stream(streams[i]):
                e = VecLoadBalanceEnv(b, S, device=dev, seed=0, env_id_offset=i * b,
                                      autoreset=True, max_steps=10000)
                e.reset()
                g = torch.Generator(device=dev)
                g.manual_seed(i)
            envs.append(e)
            gens.append(g)
        torch.cuda.synchronize()

        def one_step():
            for i in range(P):
                with torch.cuda.stream(streams[i]):
                    a = torch.randint(0, 3, (b, S), device=dev, dtype=torch.int64,
                                      generator=gens[i])
                    envs[i].step(a)

        for _ in range(args.warmup):
            one_step()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(args.steps):
            one_step()
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        print(json.dumps({"parts": P, "batch": args.batch, "servers": S, "steps": args.steps,
                          "ms_per_step": dt / args.steps * 1e3,
                          "env_steps_per_s": args.batch * args.steps / dt}), flush=True)
        del envs
        torch.cuda.synchronize()


if __name__ == "__main__":
    main()
