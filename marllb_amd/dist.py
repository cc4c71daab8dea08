"""Multi-GPU sharding of the env batch.

The path shards perfectly: env b's trajectory depends only on (seed, global env id, episode), so
rank r owns global ids [r*B, (r+1)*B) through `env_id_offset` and ranks never exchange data.  The
only collectives are around measurement: a barrier before/after the timed region and max/sum
reductions of the per-rank results.  Weak scaling: per-rank B is fixed as world grows.
"""
import os
from dataclasses import dataclass


@dataclass(frozen=True)
class Shard:
    rank: int
    world: int
    envs_per_rank: int

    @property
    def env_id_offset(self) -> int:
        return self.rank * self.envs_per_rank

    @property
    def global_envs(self) -> int:
        return self.world * self.envs_per_rank

    def global_ids(self):
        return range(self.env_id_offset, self.env_id_offset + self.envs_per_rank)


def from_env(envs_per_rank: int) -> Shard:
    """Shard of this process from torch.distributed.run's RANK/WORLD_SIZE (1 process if unset)."""
    return Shard(int(os.environ.get("RANK", "0")), int(os.environ.get("WORLD_SIZE", "1")),
                 envs_per_rank)


def max_over_ranks(x: float, device=None) -> float:
    """Max of a per-rank scalar (the bench's elapsed time) over the default process group."""
    import torch
    import torch.distributed as dist
    if not (dist.is_available() and dist.is_initialized()):
        return float(x)
    t = torch.tensor([float(x)], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def gather_over_ranks(x: float, device=None) -> list:
    """Every rank's value of a per-rank scalar, in rank order (the bench reports the per-rank
    elapsed times beside their max, so an imbalanced rank shows in the line)."""
    import torch
    import torch.distributed as dist
    if not (dist.is_available() and dist.is_initialized()):
        return [float(x)]
    n = dist.get_world_size()
    t = torch.zeros(n, dtype=torch.float64, device=device)
    t[dist.get_rank()] = float(x)
    dist.all_reduce(t, op=dist.ReduceOp.SUM)  # one small collective, no all_gather list plumbing
    return [float(v) for v in t.tolist()]


def throughput(shard: Shard, steps: int, elapsed_max: float) -> float:
    """Whole-job env-steps/s: every rank's envs x steps over the slowest rank's time."""
    return shard.global_envs * steps / elapsed_max
