#!/usr/bin/env python3
"""Generate the golden fixtures in tests/golden/ by running the MARLLB reference Python in place.

Runs ONLY in the build container (it needs /root/reference, which never travels to the GPU box).
Nothing from the reference is copied: the reference modules are imported from their own tree and
only their OUTPUTS (inputs + expected values) are written here as data.  The one piece of
scaffolding is tests/golden/gym_shim (our two-class stand-in for gym==0.17.2, which cannot be
installed offline and which env.py needs only for its space objects).

Reference entry points exercised (paths relative to the reference root):
  ReservoirSampler.get_features        simulation-mode/problem-01-reservoir-sampling/src/reservoir.py:105-196
  RewardFunction.compute + metrics     simulation-mode/problem-03-rl-environment/src/rewards.py:21-381
  LoadBalanceEnv._setup_spaces         simulation-mode/problem-03-rl-environment/src/env.py:156-184
  LoadBalanceEnv._action_to_weights    env.py:334-353
  LoadBalanceEnv._array_to_dict        env.py:391-423
  LoadBalanceEnv._normalize_observation env.py:450-470
  LoadBalanceEnv.reset/step bookkeeping env.py:186-286
  gen_alias                            src/lb/shm_proxy.py:127-146 (weights -> alias table)

Usage:  python tests/golden/gen_golden.py [--reference /root/reference] [--only alias]
"""
import argparse
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
FEATURE_NAMES = [
    "n_flow_on", "fct_mean", "fct_p90", "fct_std", "fct_mean_decay", "fct_p90_decay",
    "flow_duration_mean", "flow_duration_p90", "flow_duration_std",
    "flow_duration_mean_decay", "flow_duration_avg_decay",
]  # env.py:377-381 (column order of the observation)
METRICS = ["jain", "variance", "std", "cv", "max", "min", "product", "range", "gini"]
K = 128


def import_reference(root):
    p01 = os.path.join(root, "simulation-mode/problem-01-reservoir-sampling/src")
    p03 = os.path.join(root, "simulation-mode/problem-03-rl-environment/src")
    sys.path[:0] = [os.path.join(HERE, "gym_shim"), p01, p03]
    import reservoir  # noqa: E402
    import rewards  # noqa: E402
    import env as refenv  # noqa: E402
    return reservoir, rewards, refenv


# ------------------------------------------------------------------ reservoir features
def reservoir_cases(rng):
    cases = []  # (values[K] f32, ts_ms[K] u32, count, now_ms)

    def add(vals, ts, count, now):
        v = np.zeros(K, np.float32)
        t = np.zeros(K, np.uint32)
        v[: len(vals)] = vals
        t[: len(ts)] = ts
        cases.append((v, t, int(count), int(now)))

    # empty (test_reservoir.py:73-78)
    add([], [], 0, 1000)
    # known answers of test_reservoir.py:80-131
    add(np.arange(1, 6, dtype=np.float32), [5000] * 5, 5, 5000)
    add(np.arange(100, dtype=np.float32), [7000] * 100, 100, 7000)
    add([1.0] * 64 + [10.0] * 64, [0] * 64 + [100000] * 64, 128, 100000)
    add(np.arange(10, dtype=np.float32), np.arange(10) * 1000, 10, 10000)
    add([0.5], [1234], 1, 1234)
    add([3.0, 3.0, 3.0], [10, 20, 30], 3, 30)
    # random reservoirs: sizes, fills, value distributions, time spans
    sizes = [1, 2, 3, 7, 8, 9, 15, 16, 17, 31, 63, 64, 65, 100, 127, 128]
    spans = [0, 1, 250, 5000, 60000, 600000]
    for i in range(360):
        n = sizes[i % len(sizes)] if i < 2 * len(sizes) else int(rng.integers(1, K + 1))
        count = n if n < K else int(rng.choice([K, K + 1, 1000, 123456]))
        kind = i % 4
        if kind == 0:  # FCT-like: integer microseconds * 1e-6 (what the simulator emits)
            us = rng.exponential(rng.choice([2e3, 8e3, 4e4]), n).astype(np.int64) + 1
            vals = (us.astype(np.float32) * np.float32(1e-6)).astype(np.float32)
        elif kind == 1:  # heavy duplicates
            vals = rng.choice(np.float32([0.001, 0.002, 0.005, 0.5]), n)
        elif kind == 2:  # wide dynamic range, zeros
            vals = (rng.exponential(1.0, n) * 10.0 ** rng.integers(-4, 3, n)).astype(np.float32)
            vals[rng.random(n) < 0.1] = 0.0
        else:
            vals = rng.uniform(0, 100, n).astype(np.float32)
        span = int(spans[i % len(spans)])
        now = int(rng.integers(span, span + 10_000_000))
        ts = now - rng.integers(0, span + 1, n)
        add(vals, ts, count, now)
    return cases


def reference_features(reservoir, case):
    v, t, count, now = case
    r = reservoir.ReservoirSampler(capacity=K, seed=0)
    r.values[:] = v
    r.timestamps[:] = t.astype(np.float64) / 1000.0
    r.count = count
    r._is_full = count >= K
    f = r.get_features(decay_factor=0.9, current_time=now / 1000.0)
    out = [f["mean"], f["p90"], f["std"], f["mean_decay"], f["p90_decay"]]
    # margin of the weighted-p90 searchsorted decision (reservoir.py:180-196)
    n = min(count, K)
    margin = 1.0
    if n > 0:
        vals = v[:n]
        w = np.power(0.9, now / 1000.0 - t[:n].astype(np.float64) / 1000.0)
        order = np.argsort(vals, kind="stable")
        cs = np.cumsum(w[order])
        cut = 0.9 * cs[-1]
        rel = np.abs(cs - cut) / cs[-1]
        margin = float(rel.min())
    return out, margin


# ------------------------------------------------------------------ rewards
def reward_cases(rng):
    groups = {}
    for S in (1, 2, 3, 4, 8, 16):
        obs = []
        for i in range(40):
            o = rng.exponential(5.0, (S, 11)).astype(np.float32)
            mode = i % 6
            if mode == 1:  # some inactive servers (all-zero rows)
                o[rng.random(S) < 0.4] = 0.0
            elif mode == 2:  # active but the reward column is 0
                o[rng.random(S) < 0.5, 10] = 0.0
            elif mode == 3:  # everything inactive
                o[:] = 0.0
            elif mode == 4:  # integer-valued, equal loads
                o[:, :] = np.float32(rng.integers(1, 20))
            elif mode == 5:  # tiny values (epsilon branches)
                o *= np.float32(1e-12)
            obs.append(o)
        if S == 4:  # test_rewards.py known answers
            for vals in ([10, 10, 10, 10], [15, 10, 10, 5], [25, 10, 10, 5], [40, 5, 5, 0],
                         [40, 0, 0, 0], [20, 10, 0, 0]):
                o = np.ones((S, 11), np.float32)
                o[:, 10] = vals
                obs.append(o)
        groups[S] = np.stack(obs)
    return groups


# ------------------------------------------------------------------ alias tables
def alias_cases(rng):
    """Weight vectors as the env produces them (float32 action weights, all > 0): random, the
    discrete levels, ties with the mean, one dominant server, n = 1..16."""
    cases = []
    for n in range(1, 17):
        for _ in range(6):
            cases.append(rng.uniform(0.1, 10.0, n).astype(np.float32))
        cases.append(rng.choice(np.array([1.0, 1.5, 2.0], np.float32), n))
        cases.append(np.full(n, 1.5, np.float32))
    cases += [np.array(w, np.float32) for w in (
        [1, 1, 1, 1, 2, 2, 2],            # SURVEY §8a a13 worked example
        [0.1] * 15 + [10.0], [10.0] + [0.1] * 15, [1, 2, 3, 4], [4, 3, 2, 1],
        [1, 1, 1, 5], [0.1, 0.1, 10, 10], [2, 2, 2, 6], [1.5, 1.0, 2.0, 1.5])]
    return cases


def alias_goldens(root, rng):
    """gen_alias (src/lb/shm_proxy.py:127-146) imported in place; the module reads
    ./shm_layout.json at import time, hence the chdir."""
    import importlib
    lb = os.path.join(root, "src/lb")
    cwd = os.getcwd()
    sys.path.insert(0, lb)
    os.chdir(lb)
    try:
        shm_proxy = importlib.import_module("shm_proxy")
    finally:
        os.chdir(cwd)
    out = []
    for w in alias_cases(rng):
        weights = [float(x) for x in w]  # python floats of the float32 weights
        tab = shm_proxy.gen_alias(weights)
        out.append({"weights": weights, "odd": [float(a[0]) for a in tab],
                    "alias": [int(a[1]) for a in tab]})
    with open(os.path.join(HERE, "alias.json"), "w") as fh:
        json.dump({"source": "src/lb/shm_proxy.py:127-146 gen_alias", "cases": out}, fh)
    print(f"wrote alias.json ({len(out)} tables)")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reference", default="/root/reference")
    ap.add_argument("--only", choices=["alias"], default=None)
    args = ap.parse_args()
    if args.only == "alias":
        alias_goldens(args.reference, np.random.default_rng(20260110))
        return
    reservoir, rewards, refenv = import_reference(args.reference)
    rng = np.random.default_rng(20260109)

    # ---- reservoir features
    cases = reservoir_cases(rng)
    feats, margins = [], []
    for c in cases:
        f, m = reference_features(reservoir, c)
        feats.append(f)
        margins.append(m)
    np.savez_compressed(
        os.path.join(HERE, "reservoir_features.npz"),
        values=np.stack([c[0] for c in cases]),
        ts_ms=np.stack([c[1] for c in cases]),
        counts=np.array([c[2] for c in cases], np.uint32),
        now_ms=np.array([c[3] for c in cases], np.int64),
        expected=np.array(feats, np.float64),
        p90d_margin=np.array(margins, np.float64),
        decay=np.float64(0.9),
    )

    # ---- rewards: RewardFunction.compute(_array_to_dict(obs)) for every metric and 4 fields
    fields = ["flow_duration_avg_decay", "n_flow_on", "fct_mean", "no_such_field"]
    out = {}
    for S, obs in reward_cases(rng).items():
        e = refenv.LoadBalanceEnv(num_servers=S, step_interval=0.0, seed=0)
        exp = np.zeros((len(obs), len(METRICS), len(fields)), np.float64)
        for i, o in enumerate(obs):
            d = e._array_to_dict(o)
            for m, metric in enumerate(METRICS):
                for f, field in enumerate(fields):
                    exp[i, m, f] = float(rewards.RewardFunction(metric, field).compute(d))
        out[f"obs_S{S}"] = obs
        out[f"expected_S{S}"] = exp
    np.savez_compressed(os.path.join(HERE, "rewards.npz"), metrics=np.array(METRICS),
                        fields=np.array(fields), **out)

    # ---- env plumbing
    plumb = {"feature_names": FEATURE_NAMES, "spaces": [], "action_to_weights": [],
             "array_to_dict": [], "normalize": [], "episode": [], "metric_kat": []}
    for S, at, gt in ((4, "discrete", False), (4, "continuous", False), (8, "discrete", True),
                      (16, "continuous", True), (1, "discrete", False)):
        e = refenv.LoadBalanceEnv(num_servers=S, action_type=at, use_ground_truth=gt,
                                  step_interval=0.0)
        sp = {"S": S, "action_type": at, "use_ground_truth": gt,
              "obs_shape": list(e.observation_space.shape),
              "obs_low": float(np.min(e.observation_space.low)),
              "obs_high": float(np.max(e.observation_space.high))}
        if at == "discrete":
            sp["nvec"] = [int(x) for x in e.action_space.nvec]
        else:
            sp["act_shape"] = list(e.action_space.shape)
            sp["act_low"] = float(np.min(e.action_space.low))
            sp["act_high"] = float(np.max(e.action_space.high))
        plumb["spaces"].append(sp)
    for kw, action in (
        ({"action_type": "discrete"}, [0, 1, 2, 1]),
        ({"action_type": "discrete"}, [2, 2, 0, -1]),
        ({"action_type": "discrete", "discrete_weights": [0.5, 1.0, 4.0, 8.0]}, [3, 0, 1, 2]),
        ({"action_type": "continuous", "min_weight": 0.5, "max_weight": 5.0}, [1.0, 2.0, 3.0, 4.0]),
        ({"action_type": "continuous", "min_weight": 0.5, "max_weight": 5.0}, [0.1, 2.0, 6.0, 3.0]),
        ({"action_type": "continuous"}, [-1.0, -0.5, 0.5, 1.0]),
        ({"action_type": "continuous"}, [11.0, 0.05, 9.99, 0.1000001]),
    ):
        e = refenv.LoadBalanceEnv(num_servers=4, step_interval=0.0, **kw)
        w = e._action_to_weights(np.array(action))
        plumb["action_to_weights"].append({"kwargs": kw, "action": action,
                                           "weights": [float(x) for x in w],
                                           "dtype": str(w.dtype)})
    e = refenv.LoadBalanceEnv(num_servers=4, step_interval=0.0)
    for o in (np.ones((4, 11), np.float32),
              np.array([[0] * 11, [1] + [0] * 10, [0] * 10 + [2.5], [0] * 11], np.float32),
              np.zeros((4, 11), np.float32),
              -np.ones((4, 11), np.float32)):
        d = e._array_to_dict(o)
        plumb["array_to_dict"].append({"obs": o.tolist(), "active": d["active_servers"]})
    e = refenv.LoadBalanceEnv(num_servers=4, step_interval=0.0, normalize_obs=True, seed=3)
    seq = [rng.exponential(5.0, (4, 11)).astype(np.float32) for _ in range(6)]
    normed = [e._normalize_observation(o) for o in seq]
    plumb["normalize"] = {"inputs": [o.tolist() for o in seq],
                          "outputs": [n.tolist() for n in normed]}
    e = refenv.LoadBalanceEnv(num_servers=4, max_steps=5, step_interval=0.0, seed=42)
    e.reset()
    total = 0.0
    for k in range(7):
        _, r, done, info = e.step(np.array([0, 1, 2, 1]))
        total += r
        plumb["episode"].append({"step": k + 1, "done": bool(done), "info_keys": sorted(info),
                                 "info_step": info["step"],
                                 "has_episode": "episode" in info,
                                 "episode_l": info.get("episode", {}).get("l")})
    for vals in ([10, 10, 10, 10], [15, 10, 10, 5], [40, 0, 0, 0], [20, 10], [40, 5, 5, 0]):
        plumb["metric_kat"].append({"values": vals, **{m: float(
            rewards.RewardFunction.SUPPORTED_METRICS[m](vals)) for m in METRICS}})
    with open(os.path.join(HERE, "env_plumbing.json"), "w") as fh:
        json.dump(plumb, fh, indent=1)
    print("wrote reservoir_features.npz, rewards.npz, env_plumbing.json")
    alias_goldens(args.reference, np.random.default_rng(20260110))


if __name__ == "__main__":
    main()
