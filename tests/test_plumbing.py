"""The drop-in facades against streams captured from the reference itself (tests/golden/
gen_plumbing.py imports the reference in place and records them; CPU, no GPU needed):

* LoadBalanceEnv(reference_plumbing=True) -- BASELINE configs[0], the reference's CPU simulation
  mode -- replays reference reset()/step()/seed() traces byte for byte: observation dtype and
  bytes (float32, or float64 when normalize_obs), reward value and Python type, done, info.
* the problem-04 Trainer's recorded call stream (trainer.py:78-198: random warm-up, SAC actions,
  gradient updates, evaluation) on the facade gives the same obs / reward / done stream.
* MultiAgentLoadBalanceEnv over the plumbing mode reproduces multi_agent_env.py's per-agent
  observations, rewards, done, info and get_state(), _combine_actions and _compute_local_rewards.
"""
import json
import os

import numpy as np
import pytest

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


@pytest.fixture(scope="module")
def gold():
    meta = json.load(open(os.path.join(GOLD, "plumbing.json")))
    arrs = np.load(os.path.join(GOLD, "plumbing.npz"))
    return meta, arrs


def _info(info):
    return json.loads(json.dumps({k: (v.tolist() if isinstance(v, np.ndarray) else v)
                                  for k, v in info.items()}))


def _replay(env, calls, arrs, prefix, seed_call_at=None):
    for i, c in enumerate(calls):
        if seed_call_at is not None and i == seed_call_at:
            assert env.seed(123) == [123]
        want = arrs[f"{prefix}_obs{i}"]
        if c["kind"] == "reset":
            got = env.reset()
        else:
            got, r, d, info = env.step(arrs[f"{prefix}_act{i}"])
            assert r == c["reward"]["value"], f"call {i}: reward"
            assert type(r).__name__ == c["reward"]["type"], f"call {i}: reward type"
            assert d == c["done"], f"call {i}: done"
            assert _info(info) == c["info"], f"call {i}: info"
        assert got.dtype == want.dtype and got.shape == want.shape, f"call {i}"
        assert got.tobytes() == want.tobytes(), f"call {i}: observation bytes"


def test_reference_env_traces(gold):
    from marllb_amd import LoadBalanceEnv
    meta, arrs = gold
    assert len(meta["env_traces"]) >= 9
    for ci, tr in enumerate(meta["env_traces"]):
        env = LoadBalanceEnv(reference_plumbing=True, **tr["kwargs"])
        _replay(env, tr["calls"], arrs, f"env{ci}", tr["seed_call_at"])
        env.close()


def test_trainer_driven_episode(gold):
    """The problem-04 Trainer's recorded stream: 2 training episodes (done at max_steps 10 inside
    the trainer's 12-step loop) and one evaluation episode, replayed on the facade."""
    from marllb_amd import LoadBalanceEnv
    meta, arrs = gold
    tr = meta["trainer"]
    kinds = [c["kind"] for c in tr["calls"]]
    assert kinds.count("reset") == 3 and sum(1 for c in tr["calls"] if c["done"]) == 3
    env = LoadBalanceEnv(reference_plumbing=True, **tr["kwargs"])
    _replay(env, tr["calls"], arrs, "trainer")


def test_multi_agent_wrapper(gold):
    from marllb_amd import MultiAgentLoadBalanceEnv
    meta, _ = gold
    for case in meta["multi_agent"]:
        A, k = case["num_agents"], case["servers_per_agent"]
        env = MultiAgentLoadBalanceEnv(num_agents=A, servers_per_agent=k,
                                       action_type=case["action_type"],
                                       max_steps=case["max_steps"], seed=case["seed"],
                                       step_interval=0.0, reference_plumbing=True)
        # the wrapper declares obs_dim 4k + 4 but emits 4k + 7S values: ours keeps
        # the declared value as declared_obs_dim, obs_dim is what reset()/step() really return
        assert (env.declared_obs_dim, env.state_dim) == (case["obs_dim"], case["state_dim"])
        assert env.obs_dim == len(case["steps"][0]["obs"][0])
        for t, st in enumerate(case["steps"]):
            if t == 0:
                obs = env.reset()
            else:
                acts = [np.asarray(a, np.float32 if case["action_type"] == "continuous"
                                   else np.int64) for a in st["actions"]]
                obs, rew, done, info = env.step(acts)
                assert [float(r) for r in rew] == st["rewards"], f"step {t}"
                assert done == st["done"]
                got = _info(info)
                loads = got.pop("server_loads")  # FIX 2 (the reference emits none)
                assert got == st["info"], f"step {t}: info"
                g = np.asarray(case["global_obs"][t], np.float32)
                assert loads == [float(x) for x in g[:, 0]]
            assert len(obs) == A
            for a in range(A):
                assert obs[a].dtype == np.float64
                assert obs[a].tolist() == st["obs"][a], f"step {t} agent {a}"
            assert env.get_state().tolist() == st["state"], f"step {t}: state"
        for c in case["combine_actions"]:
            assert env._combine_actions(c["actions"]).tolist() == c["global"]
        for c in case["local_rewards"]:
            assert env._compute_local_rewards({"server_loads": c["server_loads"]}) == c["rewards"]
        env.close()
