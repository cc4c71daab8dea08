"""Reference plumbing mode (BASELINE configs[0]): the reference env's own CPU step, host only.

`LoadBalanceEnv(..., reference_plumbing=True)` reproduces what
simulation-mode/problem-03-rl-environment/src/env.py returns in simulation mode, byte for byte, for
the same seed: random observations from numpy's MT19937 (`_simulate_observation`, env.py:425-448:
per server, server-major, randint(5, 20) then 6 uniforms, the decay columns as products), the
dict round trip (env.py:391-423), `RewardFunction.compute` (rewards.py:329-381) with the nine
metrics in the same numpy operation order (rewards.py:21-287), and the float64 running
normalisation (env.py:450-470).  There is no flow simulator and no GPU in this mode: it exists so
a caller of the reference's configs[0] gets the reference's numbers, and so the drop-in facade is
pinned against captured reference traces (tests/golden/gen_plumbing.py).  It is opt-in only;
nothing ever falls back to it, and the batched hot path (VecLoadBalanceEnv) never touches it.
"""
from __future__ import annotations

from typing import Callable, Dict, List

import numpy as np

FEATURE_NAMES = [
    "n_flow_on", "fct_mean", "fct_p90", "fct_std", "fct_mean_decay", "fct_p90_decay",
    "flow_duration_mean", "flow_duration_p90", "flow_duration_std",
    "flow_duration_mean_decay", "flow_duration_avg_decay",
]  # env.py:401-405


# ---- the nine metrics, same numpy operation order as rewards.py:21-287 (float64 inputs)
def _jain(v, eps=1e-10):  # rewards.py:21-61
    v = np.asarray(v, dtype=np.float64)
    if len(v) == 0:
        return 1.0
    if np.sum(v) < eps:
        return 1.0
    s, sq = np.sum(v), np.sum(v ** 2)
    if sq < eps:
        return 1.0
    n = len(v)
    return np.clip((s ** 2) / (n * sq), 1.0 / n, 1.0)


def _variance(v):  # rewards.py:64-86
    v = np.asarray(v, dtype=np.float64)
    return 0.0 if len(v) == 0 else -np.var(v)


def _std(v):  # rewards.py:89-105
    v = np.asarray(v, dtype=np.float64)
    return 0.0 if len(v) == 0 else -np.std(v)


def _cv(v, eps=1e-10):  # rewards.py:108-134
    v = np.asarray(v, dtype=np.float64)
    if len(v) == 0:
        return 0.0
    mean = np.mean(v)
    if mean < eps:
        return 0.0
    return -(np.std(v) / (mean + eps))


def _max(v):  # rewards.py:137-160
    v = np.asarray(v, dtype=np.float64)
    return 0.0 if len(v) == 0 else -np.max(v)


def _min(v):  # rewards.py:163-178
    v = np.asarray(v, dtype=np.float64)
    return 0.0 if len(v) == 0 else np.min(v)


def _product(v, eps=1e-10):  # rewards.py:181-208
    v = np.asarray(v, dtype=np.float64)
    return 0.0 if len(v) == 0 else np.sum(np.log(v + eps))


def _range(v):  # rewards.py:211-227
    v = np.asarray(v, dtype=np.float64)
    return 0.0 if len(v) == 0 else -(np.max(v) - np.min(v))


def _gini(v):  # rewards.py:230-262: the double loop, in order (its sum order fixes the bits)
    v = np.asarray(v, dtype=np.float64)
    if len(v) == 0:
        return 0.0
    n = len(v)
    mean = np.mean(v)
    if mean == 0:
        return 0.0
    d = 0.0
    for i in range(n):
        for j in range(n):
            d += abs(v[i] - v[j])
    return -(d / (2 * n * n * mean))


METRIC_FUNCS: Dict[str, Callable] = {
    "jain": _jain, "variance": _variance, "std": _std, "cv": _cv, "max": _max, "min": _min,
    "product": _product, "range": _range, "gini": _gini,
}  # rewards.py:297-307 SUPPORTED_METRICS


def reward_of(obs_dict: dict, metric: str, field: str):
    """RewardFunction.compute (rewards.py:329-381)."""
    active = obs_dict.get("active_servers", [])
    stats = obs_dict.get("server_stats", {})
    if not active:
        return 0.0
    vals: List[float] = []
    for sid in active:
        if sid in stats and field in stats[sid]:
            vals.append(stats[sid][field])
    if not vals:
        return 0.0
    return METRIC_FUNCS[metric](vals)


class ReferencePlumbing:
    """The state the reference env keeps in simulation mode: RandomState, normalisation stats."""

    def __init__(self, num_servers: int, seed, normalize_obs: bool, reward_metric: str,
                 reward_field: str):
        self.S = int(num_servers)
        self.rng = np.random.RandomState(seed)          # env.py:127
        self.normalize_obs = normalize_obs
        self.metric, self.field = reward_metric, reward_field
        self.obs_mean = np.zeros((self.S, 11))          # env.py:152-154
        self.obs_std = np.ones((self.S, 11))
        self.obs_count = 0

    def seed(self, seed) -> None:                        # env.py:327-330
        self.rng = np.random.RandomState(seed)

    def simulate(self) -> np.ndarray:
        """env.py:425-448: 7 MT19937 draws per server, server-major, float32 storage."""
        r = self.rng
        obs = np.zeros((self.S, 11), dtype=np.float32)
        for s in range(self.S):
            obs[s, 0] = r.randint(5, 20)
            obs[s, 1] = r.uniform(5, 15)
            obs[s, 2] = r.uniform(10, 25)
            obs[s, 3] = r.uniform(1, 5)
            obs[s, 4] = obs[s, 1] * 0.9
            obs[s, 5] = obs[s, 2] * 0.9
            obs[s, 6] = r.uniform(8, 18)
            obs[s, 7] = r.uniform(15, 30)
            obs[s, 8] = r.uniform(2, 8)
            obs[s, 9] = obs[s, 6] * 0.85
            obs[s, 10] = obs[s, 6] * 0.9
        return obs

    def normalize(self, obs: np.ndarray) -> np.ndarray:
        """env.py:450-470 (float64 statistics; the result is float64, as the reference's)."""
        self.obs_count += 1
        delta = obs - self.obs_mean
        self.obs_mean += delta / self.obs_count
        delta2 = obs - self.obs_mean
        self.obs_std = np.sqrt(np.maximum(
            (self.obs_std ** 2 * (self.obs_count - 1) + delta * delta2) / self.obs_count, 1e-8))
        return (obs - self.obs_mean) / (self.obs_std + 1e-8)

    def reward(self, obs_dict: dict):
        return reward_of(obs_dict, self.metric, self.field)
