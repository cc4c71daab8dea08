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
    ap.add_argument("--join", default="none,step",
                    help="none: the parts run free on their streams; step: one randint on the "
                         "main stream per step, every part waits for it and the main stream "
                         "waits for every part (the join a single batched step() would need)")
    args = ap.parse_args()
    import torch
    from marllb_amd.env import VecLoadBalanceEnv
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(0)
    main_s = torch.cuda.current_stream(dev)
    for join, P in [(j, int(x)) for j in args.join.split(",") for x in args.parts.split(",")]:
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

        def one_step_join():
            a = torch.randint(0, 3, (args.batch, S), device=dev, dtype=torch.int64,
                              generator=gens[0])
            ev = torch.cuda.Event()
            ev.record(main_s)
            done = []
            for i in range(P):
                streams[i].wait_event(ev)
                with torch.cuda.stream(streams[i]):
                    envs[i].step(a[i * b:(i + 1) * b])
                    e = torch.cuda.Event()
                    e.record(streams[i])
                    done.append(e)
            for e in done:
                main_s.wait_event(e)

        def one_step_free():
            for i in range(P):
                with torch.cuda.stream(streams[i]):
                    a = torch.randint(0, 3, (b, S), device=dev, dtype=torch.int64,
                                      generator=gens[i])
                    envs[i].step(a)

        one_step = one_step_join if join == "step" else one_step_free
        for _ in range(args.warmup):
            one_step()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(args.steps):
            one_step()
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        print(json.dumps({"parts": P, "join": join, "batch": args.batch, "servers": S, "steps": args.steps,
                          "ms_per_step": dt / args.steps * 1e3,
                          "env_steps_per_s": args.batch * args.steps / dt}), flush=True)
        del envs
        torch.cuda.synchronize()


if __name__ == "__main__":
    main()
