#!/usr/bin/env python3
"""Capture reference reset()/step() traces, problem-05 wrapper I/O and a problem-04 trainer-driven
episode into tests/golden/plumbing.npz (+ plumbing.json), by running the reference in place.

Runs ONLY in the build container (it needs /root/reference, which never travels to the GPU box).
Nothing from the reference is copied: its modules are imported from their own tree and only their
outputs (inputs + expected values) are written here as data.  Scaffolding of our own: the gym
shim (tests/golden/gym_shim) and `Recorder`, a proxy that logs the calls a caller makes on an env.

Reference entry points exercised (paths relative to the reference root):
  LoadBalanceEnv.reset/step/seed (simulation mode)  simulation-mode/problem-03-rl-environment/src/env.py:186-330
    _simulate_observation (MT19937 stream)          env.py:425-448
    _normalize_observation                          env.py:450-470
    RewardFunction.compute                          src/rewards.py:329-381
  MultiAgentLoadBalanceEnv                          simulation-mode/problem-05-qmix/src/multi_agent_env.py:44-282
    _get_agent_observation / _combine_actions       :152-208
    _compute_local_rewards / get_state              :210-282
  Trainer.train / evaluate (SAC_GRU_Agent)          simulation-mode/problem-04-sac-gru/src/trainer.py:78-198

Also checks, at generation time, that marllb_amd.LoadBalanceEnv(reference_plumbing=True) driven by
the reference Trainer produces the identical stream (the drop-in claim for configs[0]).

Usage:  python tests/golden/gen_plumbing.py [--reference /root/reference]
"""
import argparse
import json
import os
import random
import sys
import tempfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))


class Recorder:
    """Proxy env: forwards reset/step and the attributes callers read; logs every call."""

    def __init__(self, env):
        self._env = env
        self.log = []

    def __getattr__(self, name):
        return getattr(self._env, name)

    def reset(self):
        o = self._env.reset()
        self.log.append(("reset", None, np.array(o), None, None, None))
        return o

    def step(self, a):
        o, r, d, info = self._env.step(a)
        self.log.append(("step", np.array(a), np.array(o), r, d, info))
        return o, r, d, info


def _info_json(info):
    if info is None:
        return None
    out = {}
    for k, v in info.items():
        if isinstance(v, np.ndarray):
            v = v.tolist()
        out[k] = v
    return out


def _reward_json(r):
    return None if r is None else {"value": float(r), "type": type(r).__name__}


def env_traces(refenv):
    """Per config: reset, 12 steps (max_steps 10: done at 10, stepping past it), seed(123),
    reset, 3 steps."""
    rng = np.random.default_rng(20260110)
    configs = []
    for S, at, norm, seed in ((4, "discrete", False, 0), (4, "discrete", False, 42),
                              (4, "continuous", False, 0), (4, "continuous", True, 42),
                              (4, "discrete", True, 0), (8, "continuous", False, 7),
                              (16, "discrete", True, 3), (1, "continuous", False, 5)):
        for metric in (("jain", "gini") if (S, seed) == (4, 0) and at == "discrete" and not norm
                       else ("jain",)):
            kw = dict(num_servers=S, action_type=at, normalize_obs=norm, seed=seed, max_steps=10,
                      step_interval=0.0, reward_metric=metric)
            e = Recorder(refenv.LoadBalanceEnv(**kw))
            e.reset()
            for _ in range(12):
                if at == "discrete":
                    a = rng.integers(-3, 3, S)  # negative indices: python list indexing
                else:
                    a = rng.uniform(-1.5, 12.0, S).astype(np.float32)
                e.step(a)
            e.seed(123)
            e.reset()
            for _ in range(3):
                e.step(rng.integers(0, 3, S) if at == "discrete"
                       else rng.uniform(-1.0, 1.0, S).astype(np.float32))
            configs.append({"kwargs": kw, "log": e.log, "seed_call_at": 13})
    return configs


def multi_agent(p05_src):
    sys.path.insert(0, p05_src)
    import multi_agent_env as mae  # noqa: E402
    out = []
    rng = np.random.default_rng(20260111)
    for A, k, at, seed in ((4, 4, "continuous", 11), (4, 4, "discrete", 12), (2, 2, "continuous", 13)):
        m = mae.MultiAgentLoadBalanceEnv(num_agents=A, servers_per_agent=k, action_type=at,
                                         max_steps=6)
        m.env.seed(seed)            # the wrapper passes no seed (multi_agent_env.py:63-69)
        m.env.step_interval = 0.0   # nor step_interval: no wall-clock sleep
        rec = Recorder(m.env)
        m.env = rec
        steps = [{"obs": [o.tolist() for o in m.reset()], "state": m.get_state().tolist()}]
        for t in range(8):
            if at == "discrete":
                acts = [rng.integers(0, 3, k) for _ in range(A)]
            else:
                acts = [rng.uniform(-1.0, 4.0, k).astype(np.float32) for _ in range(A)]
            obs, rew, done, info = m.step(acts)
            steps.append({"actions": [a.tolist() for a in acts],
                          "obs": [o.tolist() for o in obs], "rewards": [float(r) for r in rew],
                          "done": bool(done), "info": _info_json(info),
                          "state": m.get_state().tolist()})
        combine = []
        for acts in ([[1.0, 2.0, 3.0, 4.0][:k]] * A, [[0.5] * (k // 2)] * A,
                     [list(range(k)) for _ in range(A)], [[]] * A):
            combine.append({"actions": acts, "global": m._combine_actions(acts).tolist()})
        local = []
        for _ in range(6):
            loads = rng.integers(0, 6, A * k).astype(float).tolist()
            if _ % 3 == 0:
                loads[:k] = [0.0] * k
            local.append({"server_loads": loads,
                          "rewards": [float(x) for x in m._compute_local_rewards(
                              {"server_loads": loads})]})
        out.append({"num_agents": A, "servers_per_agent": k, "action_type": at, "seed": seed,
                    "max_steps": 6, "steps": steps,
                    "global_obs": [np.asarray(x[2]).tolist() for x in rec.log],
                    "obs_dim": m.obs_dim, "state_dim": m.state_dim,
                    "combine_actions": combine, "local_rewards": local})
    return out


def trainer_episode(p04_src, refenv, make_ours):
    """Run the reference Trainer (2 episodes of 12 steps, 5 random warm-up steps, then the SAC
    actor with gradient updates, one evaluation) on the reference env, then on our facade, with
    identical torch / action-space seeds; record the reference stream, assert ours equals it."""
    import torch
    sys.path.insert(0, p04_src)
    import trainer as trmod  # noqa: E402
    from sac_agent import SAC_GRU_Agent  # noqa: E402

    def run(env):
        torch.manual_seed(0)
        np.random.seed(0)  # replay-buffer sampling draws from the global RNGs
        random.seed(0)
        env.action_space.np_random = np.random.RandomState(5)
        agent = SAC_GRU_Agent(state_dim=44, action_dim=4, batch_size=8, buffer_size=1000,
                              device="cpu")
        rec = Recorder(env)
        with tempfile.TemporaryDirectory() as d:
            t = trmod.Trainer(rec, agent, max_episodes=2, max_steps=12, start_steps=5,
                              eval_interval=2, save_interval=1000, save_dir=d, log_interval=1)
            t.evaluate = lambda num_episodes=1, _f=t.evaluate: _f(num_episodes=1)
            t.train()
        return rec.log

    kw = dict(num_servers=4, action_type="continuous", max_steps=10, step_interval=0.0, seed=7)
    ref = run(refenv.LoadBalanceEnv(**kw))
    ours = run(make_ours(**kw))
    assert len(ref) == len(ours), (len(ref), len(ours))
    for i, (x, y) in enumerate(zip(ref, ours)):
        assert x[0] == y[0], i
        if x[1] is not None:
            assert np.array_equal(x[1], y[1]), f"action {i}"
        assert x[2].dtype == y[2].dtype and x[2].tobytes() == y[2].tobytes(), f"obs {i}"
        assert x[3] == y[3] and x[4] == y[4], f"reward/done {i}"
        assert _info_json(x[5]) == _info_json(y[5]), f"info {i}"
    print(f"trainer episode: {len(ref)} calls, facade (reference_plumbing) identical")
    return {"kwargs": kw, "log": ref}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reference", default="/root/reference")
    args = ap.parse_args()
    r = args.reference
    p03 = os.path.join(r, "simulation-mode/problem-03-rl-environment/src")
    p04 = os.path.join(r, "simulation-mode/problem-04-sac-gru/src")
    p05 = os.path.join(r, "simulation-mode/problem-05-qmix/src")
    sys.path[:0] = [os.path.join(HERE, "gym_shim"), p03]
    import env as refenv  # noqa: E402
    sys.path.insert(0, ROOT)
    from marllb_amd.env import LoadBalanceEnv  # noqa: E402

    arrays, meta = {}, {"env_traces": [], "multi_agent": None, "trainer": None}

    def put_log(prefix, log):
        calls = []
        for i, (kind, a, o, rew, done, info) in enumerate(log):
            arrays[f"{prefix}_obs{i}"] = o
            if a is not None:
                arrays[f"{prefix}_act{i}"] = a
            calls.append({"kind": kind, "reward": _reward_json(rew),
                          "done": None if done is None else bool(done), "info": _info_json(info)})
        return calls

    for ci, c in enumerate(env_traces(refenv)):
        meta["env_traces"].append({"kwargs": c["kwargs"], "seed_call_at": c["seed_call_at"],
                                   "calls": put_log(f"env{ci}", c["log"])})
    meta["multi_agent"] = multi_agent(p05)
    tr = trainer_episode(p04, refenv,
                         lambda **kw: LoadBalanceEnv(reference_plumbing=True, **kw))
    meta["trainer"] = {"kwargs": tr["kwargs"], "calls": put_log("trainer", tr["log"])}
    np.savez_compressed(os.path.join(HERE, "plumbing.npz"), **arrays)
    with open(os.path.join(HERE, "plumbing.json"), "w") as fh:
        json.dump(meta, fh)
    print(f"wrote plumbing.npz ({len(arrays)} arrays), plumbing.json")


if __name__ == "__main__":
    main()
