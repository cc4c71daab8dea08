"""problem-05 multi-agent facade (SURVEY §8a a15, §0.6 contract) on the GPU simulator."""
import numpy as np
import pytest

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def need_gpu():
    if not torch.cuda.is_available():
        pytest.fail("GPU test run without a HIP device")


def test_single_env_reference_io():
    """Shapes and values the reference wrapper actually produces: 128-dim float64
    agent obs built from 4-value slices, 74-dim state, replicated global reward."""
    from marllb_amd import MultiAgentLoadBalanceEnv
    env = MultiAgentLoadBalanceEnv(num_agents=4, servers_per_agent=4, max_steps=10, seed=3)
    assert (env.obs_dim, env.declared_obs_dim, env.state_dim) == (128, 20, 74)
    obs = env.reset()
    assert len(obs) == 4 and all(o.shape == (128,) and o.dtype == np.float64 for o in obs)
    st = env.get_state()
    assert st.shape == (74,) and np.all(st[:72] == 0) and st[72] == 0.0 and st[73] == 4
    acts = [np.array([0.5, 1.0, 2.0, 4.0], np.float32) for _ in range(4)]
    obs, rew, done, info = env.step(acts)
    assert len(rew) == 4 and len(set(rew)) == 1 and not done
    for a in range(4):  # own slice flat[16a:16a+16], shared tail flat[64:]
        np.testing.assert_array_equal(obs[a][16:], obs[0][16:])
    loads = np.array(info["server_loads"])
    np.testing.assert_array_equal(obs[0][0:4:4], loads[0:1])  # flat[0] = server 0 n_flow_on
    assert env.get_state()[72] == pytest.approx(0.1)
    assert len(info["server_loads"]) == 16


def test_scalar_agent_actions_and_local_rewards():
    """FIX 1 (one value per agent is broadcast) and FIX 2 (server_loads, local Jain)."""
    from marllb_amd import MultiAgentLoadBalanceEnv
    a = MultiAgentLoadBalanceEnv(num_agents=4, servers_per_agent=4, action_type="discrete",
                                 max_steps=10, seed=5, global_reward=False)
    b = MultiAgentLoadBalanceEnv(num_agents=4, servers_per_agent=4, action_type="discrete",
                                 max_steps=10, seed=5, global_reward=False)
    a.reset()
    b.reset()
    oa, ra, _, ia = a.step([0, 1, 2, 1])
    ob, rb, _, ib = b.step([[0] * 4, [1] * 4, [2] * 4, [1] * 4])
    for x, y in zip(oa, ob):
        np.testing.assert_array_equal(x, y)
    assert ra == rb and len(ra) == 4
    for ag in range(4):
        loads = ia["server_loads"][4 * ag:4 * ag + 4]
        s = sum(loads)
        want = 0.0 if s == 0 else s * s / (4 * sum(x * x for x in loads) + 1e-8)
        assert ra[ag] == pytest.approx(want)


def test_vec_agent_obs_kernel_and_actions():
    """lbsim_agent_obs equals the wrapper's slicing; (B,A), (B,A,k) and (B,S) actions agree."""
    from marllb_amd import VecMultiAgentLoadBalanceEnv
    B, A, k = 256, 4, 4
    envs = [VecMultiAgentLoadBalanceEnv(B, A, k, device="cuda:0", seed=9,
                                        action_type="discrete") for _ in range(3)]
    obs0 = [e.reset() for e in envs]
    assert obs0[0].shape == (B, A, 128)
    assert torch.equal(obs0[0], obs0[1])
    a = torch.randint(0, 3, (B, A), device="cuda:0")
    o1, r1, d1, i1 = envs[0].step(a)
    o2, _, _, _ = envs[1].step(a.unsqueeze(2).expand(B, A, k))
    o3, _, _, _ = envs[2].step(a.repeat_interleave(k, dim=1))
    assert torch.equal(o1, o2) and torch.equal(o1, o3)
    # the wrapper's slicing of the underlying (B, 16, 11) obs
    raw = envs[0].vec.step(a.repeat_interleave(k, dim=1))[0]
    flat = raw.reshape(B, -1)
    want = torch.cat([flat[:, :64].reshape(B, A, 16),
                      flat[:, 64:].unsqueeze(1).expand(B, A, 112)], dim=2)
    assert torch.equal(envs[0].agent_obs(raw), want)
    st = envs[0].get_state()
    assert st.shape == (B, 74) and torch.all(st[:, -1] == 4)
    assert r1.shape == (B, A) and torch.all(r1 == r1[:, :1])


def test_agent_obs_kernel_vs_reference_wrapper(golden_dir):
    """lbsim_agent_obs on the global observations the reference wrapper saw equals
    multi_agent_env.py:152-188's per-agent output (recorded by tests/golden/gen_plumbing.py)."""
    import json
    import os

    from marllb_amd import VecMultiAgentLoadBalanceEnv
    meta = json.load(open(os.path.join(golden_dir, "plumbing.json")))
    for case in meta["multi_agent"]:
        A, k = case["num_agents"], case["servers_per_agent"]
        env = VecMultiAgentLoadBalanceEnv(4, A, k, device="cuda:0", seed=1)
        g = torch.tensor(case["global_obs"], dtype=torch.float32, device="cuda:0")  # (T, S, 11)
        got = env.agent_obs(g).cpu().numpy()
        want = np.array([st["obs"] for st in case["steps"]], np.float64).astype(np.float32)
        np.testing.assert_array_equal(got, want)
        env.close()


def test_vec_terminal_step_local_rewards():
    """global_reward=False: on the step that ends an episode the local Jain rewards and
    info['server_loads'] come from that step's raw n_flow_on, not from the auto-reset's next
    first observation (and not from normalised values)."""
    from marllb_amd import VecLoadBalanceEnv, VecMultiAgentLoadBalanceEnv
    B, A, k, T = 64, 4, 4, 3
    kw = dict(device="cuda:0", seed=21, action_type="discrete", max_steps=T, normalize_obs=True)
    m = VecMultiAgentLoadBalanceEnv(B, A, k, global_reward=False, **kw)
    ref = VecLoadBalanceEnv(B, A * k, autoreset=False, **kw)
    m.reset()
    ref.reset()
    a = torch.randint(0, 3, (B, A), device="cuda:0", generator=torch.Generator("cuda").manual_seed(0))
    for t in range(T + 1):
        _, rew, done, info = m.step(a)
        _, _, _, ri = ref.step(a.repeat_interleave(k, dim=1), raw_obs=True)
        loads = ri["raw_obs"][:, :, 0]
        if t == T - 1:
            assert bool(done.all())
        if t < T:  # ref (no autoreset) and m agree until m's envs restart
            assert torch.equal(info["server_loads"], loads)
            l = loads.double().view(B, A, k)
            s, sq = l.sum(2), (l * l).sum(2)
            want = torch.where(s == 0, torch.zeros_like(s), s * s / (k * sq + 1e-8)).float()
            assert torch.equal(rew, want)


@pytest.mark.parametrize("step_kernel", ["fused", "split"])
@pytest.mark.parametrize("normalize,feature_mode", [(False, "problem01"), (True, "problem01"),
                                                    (False, "upstream")])
def test_step_launch_writes_agent_obs_and_state(step_kernel, normalize, feature_mode):
    """The (B, A, 4k + 7S) agent observations and the (B, 74) state come from the step / reset
    launches themselves (lbsim_step_outputs_t agent_obs / state): equal to lbsim_agent_obs on the
    returned rows and to zeros ++ [step / max_steps, A], across the auto-reset boundary and a
    masked reset.  feature_mode='upstream' replaces columns 1-10 of the returned rows after the
    launch (shm_proxy.py process_reservoir): the agent observations follow those rows."""
    from marllb_amd import VecMultiAgentLoadBalanceEnv
    B, A, k, T = 96, 4, 4, 3
    env = VecMultiAgentLoadBalanceEnv(B, A, k, device="cuda:0", seed=21, action_type="discrete",
                                      max_steps=T, normalize_obs=normalize,
                                      step_kernel=step_kernel, feature_mode=feature_mode)
    ao = env.reset()
    ep = torch.zeros(B, dtype=torch.int32, device="cuda:0")
    g = torch.Generator(device="cuda:0")
    g.manual_seed(4)
    for t in range(2 * T + 2):
        if t == T + 1:  # a masked reset of every other env
            mask = (torch.arange(B, device="cuda:0") % 2 == 0)
            ao = env.reset(mask=mask)
            ep = torch.where(mask, torch.zeros_like(ep), ep)
        elif t > 0:
            a = torch.randint(0, 3, (B, A), device="cuda:0", generator=g)
            ao, _, done, info = env.step(a)
            ep = torch.where(done, torch.zeros_like(ep), info["episode_length"])
        obs = env.vec._last_obs
        assert torch.equal(ao, env.agent_obs(obs)), t
        st = env.get_state()
        want = torch.zeros((B, 74), device="cuda:0")
        want[:, 72] = ep.float() / float(T)
        want[:, 73] = float(A)
        assert torch.equal(st, want), t
    if feature_mode == "upstream":  # the rows really are the upstream features
        ref = VecMultiAgentLoadBalanceEnv(B, A, k, device="cuda:0", seed=21,
                                          action_type="discrete", max_steps=T)
        assert not torch.equal(ref.reset(), env.reset())
        ref.close()
    env.close()
