"""One rank of the sharded rollout used by tests/test_dist.py (not collected by pytest).

    RANK=r WORLD_SIZE=n python tests/dist_worker.py --mode oracle|gpu --port P --out F ...

Each rank steps only its own shard (global env ids [r*B, (r+1)*B) via env_id_offset, exactly as
bench.py does), with actions that are a function of (global env id, server, step) so the union of
the shards is comparable with one process stepping all n*B envs.  Collectives (gloo) only gather
the results to rank 0 and reduce the timing, mirroring the bench's measurement-only collectives.
"""
import argparse
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def actions(gids: np.ndarray, S: int, k: int) -> np.ndarray:
    """Deterministic discrete actions keyed by global env id (shared with the single-process run)."""
    s = np.arange(S)[None, :]
    return ((gids[:, None] * 7 + s * 5 + k * 3 + (gids[:, None] >> 3)) % 3).astype(np.int64)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--mode", choices=["oracle", "gpu"], required=True)
    ap.add_argument("--port", type=int, required=True)
    ap.add_argument("--out", required=True)
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--servers", type=int, default=4)
    ap.add_argument("--steps", type=int, default=4)
    ap.add_argument("--seed", type=int, default=1234)
    args = ap.parse_args()

    import torch.distributed as dist

    from marllb_amd import dist as lbdist
    from marllb_amd.env import make_config

    shard = lbdist.from_env(args.batch)
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{args.port}",
                            rank=shard.rank, world_size=shard.world)
    gids = np.arange(shard.env_id_offset, shard.env_id_offset + args.batch, dtype=np.int64)
    B, S = args.batch, args.servers
    kw = dict(seed=args.seed, env_id_offset=shard.env_id_offset, max_steps=1000)
    if args.mode == "oracle":
        import oracle
        env = oracle.OracleEnv(make_config(B, S, **kw), threads=1)
        obs = [env.reset()]
        rew = []
        for k in range(args.steps):
            o, r, _, _ = env.step(actions(gids, S, k))
            obs.append(o)
            rew.append(r)
    else:
        import torch
        from marllb_amd import VecLoadBalanceEnv
        env = VecLoadBalanceEnv(B, S, device="cuda:0", autoreset=False, **kw)
        obs = [env.reset().cpu().numpy()]
        rew = []
        for k in range(args.steps):
            o, r, _, _ = env.step(torch.from_numpy(actions(gids, S, k)).cuda())
            obs.append(o.cpu().numpy())
            rew.append(r.cpu().numpy())
        env.close()

    payload = (shard.env_id_offset, np.stack(obs), np.stack(rew))
    gathered = [None] * shard.world if shard.rank == 0 else None
    dist.gather_object(payload, gathered, dst=0)
    # the bench's timing reduction: slowest rank wins; whole-job rate over all ranks' envs
    slowest = lbdist.max_over_ranks(float(shard.rank + 1))
    per_rank = lbdist.gather_over_ranks(float(shard.rank + 1))
    rate = lbdist.throughput(shard, args.steps, slowest)
    if shard.rank == 0:
        gathered.sort(key=lambda p: p[0])
        np.savez(args.out, offsets=np.array([p[0] for p in gathered]),
                 obs=np.concatenate([p[1] for p in gathered], axis=1),
                 rew=np.concatenate([p[2] for p in gathered], axis=1),
                 slowest=slowest, rate=rate, per_rank=np.array(per_rank))
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
