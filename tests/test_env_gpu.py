"""The reference's env test-suite (simulation-mode/problem-03-rl-environment/tests/test_env.py)
replayed on marllb_amd.LoadBalanceEnv, plus VecLoadBalanceEnv auto-reset semantics and the call
pattern of problem-04's Trainer (trainer.py:92-126) as a drop-in check."""
import numpy as np
import pytest

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def need_gpu():
    if not torch.cuda.is_available():
        pytest.fail("GPU test run without a HIP device")


def make(**kw):
    from marllb_amd import LoadBalanceEnv
    return LoadBalanceEnv(**kw)


# ---- test_env.py:17-123 TestLoadBalanceEnvBasics
def test_initialization():
    env = make(num_servers=4, action_type="discrete", max_steps=100, use_shm=False, seed=42)
    assert (env.num_servers, env.action_type, env.max_steps, env.use_shm) == (4, "discrete", 100, False)


def test_spaces():
    env = make(num_servers=4, seed=42)
    assert env.observation_space.shape == (4, 11)
    assert np.all(env.observation_space.low == 0) and np.all(env.observation_space.high == np.inf)
    assert len(env.action_space.nvec) == 4 and np.all(env.action_space.nvec == 3)
    env = make(num_servers=4, action_type="continuous", max_steps=100)
    assert env.action_space.shape == (4,)
    assert np.all(env.action_space.low == np.float32(0.1)) and np.all(env.action_space.high == 10.0)


def test_reset_and_step():
    env = make(num_servers=4, max_steps=100, seed=42)
    obs = env.reset()
    assert obs.shape == (4, 11) and obs.dtype == np.float32 and np.all(np.isfinite(obs))
    assert env.current_step == 0
    obs, reward, done, info = env.step(env.action_space.sample())
    assert obs.shape == (4, 11) and np.all(np.isfinite(obs))
    assert isinstance(reward, float) and np.isfinite(reward)
    assert isinstance(done, bool)
    assert {"step", "weights", "active_servers", "episode_return"} <= set(info)


def test_episode_termination_and_return():
    env = make(num_servers=4, max_steps=5, seed=42)
    env.reset()
    total = 0.0
    for k in range(5):
        obs, reward, done, info = env.step(env.action_space.sample())
        total += reward
        assert done == (k == 4)
    assert info["episode"]["l"] == 5
    assert info["episode"]["r"] == pytest.approx(total, abs=1e-5)
    obs, reward, done, info = env.step(env.action_space.sample())  # reference keeps stepping
    assert done and info["step"] == 6


def test_seed_reproducibility():
    a, b = make(num_servers=4, seed=42), make(num_servers=4, seed=42)
    np.testing.assert_array_equal(a.reset(), b.reset())
    act = np.array([0, 1, 2, 1])
    np.testing.assert_array_equal(a.step(act)[0], b.step(act)[0])
    c = make(num_servers=4, seed=43)
    assert not np.array_equal(c.reset(), make(num_servers=4, seed=42).reset())
    a.seed(7)
    b.seed(7)
    np.testing.assert_array_equal(a.reset(), b.reset())


def test_action_conversion():
    env = make(num_servers=4, action_type="discrete", discrete_weights=[1.0, 1.5, 2.0])
    np.testing.assert_array_almost_equal(env._action_to_weights(np.array([0, 1, 2, 1])),
                                         [1.0, 1.5, 2.0, 1.5])
    env = make(num_servers=4, action_type="continuous", min_weight=0.5, max_weight=5.0)
    np.testing.assert_array_almost_equal(env._action_to_weights(np.array([0.1, 2.0, 6.0, 3.0])),
                                         [0.5, 2.0, 5.0, 3.0])


def test_reward_in_jain_range():
    env = make(num_servers=4, reward_metric="jain", seed=42)
    env.reset()
    for _ in range(5):
        _, r, _, info = env.step(env.action_space.sample())
        n = len(info["active_servers"])
        assert 1.0 / n - 1e-6 <= r <= 1.0


def test_normalization_updates():
    env = make(num_servers=4, normalize_obs=True, seed=42)
    env.reset()
    obs, _, _, info = env.step(env.action_space.sample())
    assert np.all(np.abs(obs) < 1e4) and info["active_servers"]


def test_render_and_close(capsys):
    env = make(num_servers=4, seed=1)
    env.reset()
    env.step(env.action_space.sample())
    env.render(mode="human")
    out = capsys.readouterr().out
    assert "Step: 1/" in out and "Active Servers" in out
    env.close()


def test_errors_like_reference():
    with pytest.raises(ValueError, match="Unsupported metric"):
        make(num_servers=4, reward_metric="nope")
    with pytest.raises(ValueError, match="Unknown action_type"):
        make(num_servers=4, action_type="hybrid")
    with pytest.raises(ValueError, match="shm_name"):
        make(num_servers=4, use_shm=True)
    env = make(num_servers=4, seed=1)
    env.reset()
    with pytest.raises(IndexError):
        env.step(np.array([0, 1, 3, 0]))


def test_unknown_reward_field_gives_zero():
    env = make(num_servers=4, reward_field="no_such_field", seed=1)
    env.reset()
    assert env.step(np.array([0, 0, 0, 0]))[1] == 0.0


# ---- problem-04 Trainer call pattern (continuous, tanh actions, flattened state)
def test_trainer_call_pattern():
    env = make(num_servers=4, action_type="continuous", max_steps=20, seed=3)
    state = env.reset()
    state = state.flatten() if state.ndim > 1 else state
    assert state.shape == (44,)
    w = torch.randn(44, 4)
    for step in range(20):
        if step < 5:
            action = env.action_space.sample()
        else:
            action = torch.tanh(torch.from_numpy(state) @ w).numpy()  # SAC output in [-1, 1]
        nxt, reward, done, info = env.step(action)
        assert min(info["weights"]) >= np.float32(0.1) - 1e-7  # negatives clip to min_weight
        state = nxt.flatten()
        if done:
            break
    assert done and step == 19


# ---- VecLoadBalanceEnv
def test_vec_autoreset_matches_oracle(oracle_mod):
    from marllb_amd import VecLoadBalanceEnv
    from marllb_amd.env import make_config
    B, S, T = 96, 4, 3
    kw = dict(seed=77, max_steps=T)
    env = VecLoadBalanceEnv(B, S, device="cuda:0", autoreset=True, keep_terminal_obs=True, **kw)
    ora = oracle_mod.OracleEnv(make_config(B, S, **kw), threads=4)
    np.testing.assert_array_equal(env.reset().cpu().numpy(), ora.reset())
    rng = np.random.default_rng(1)
    mask = (np.arange(B) % 2).astype(np.uint8)
    env.reset(mask=torch.from_numpy(mask))
    ora.reset(mask=mask)
    for k in range(2 * T + 1):
        a = rng.integers(0, 3, (B, S)).astype(np.int64)
        obs, rew, done, info = env.step(torch.from_numpy(a))
        oo, ro, do, _ = ora.step(a)
        np.testing.assert_array_equal(rew.cpu().numpy(), ro)
        np.testing.assert_array_equal(done.cpu().numpy(), do.astype(bool))
        if "terminal_obs" in info:
            np.testing.assert_array_equal(info["terminal_obs"].cpu().numpy(), oo)
        if do.any():
            oo = ora.reset(mask=do, obs=oo)
        np.testing.assert_array_equal(obs.cpu().numpy(), oo, err_msg=f"step {k}")
        ln, rt = ora.episode_stats()
        np.testing.assert_array_equal(info["episode_length"].cpu().numpy()[do == 0], ln[do == 0])


def test_vec_synced_autoreset_matches_oracle(oracle_mod):
    """Envs reset together stay in step: every env ends its episode at the same step, so the
    auto-reset launches only then (env._synced) -- three episodes equal the oracle step by step,
    and between episode ends no reset launch is made."""
    from marllb_amd import VecLoadBalanceEnv
    from marllb_amd.env import make_config
    B, S, T = 64, 4, 4
    kw = dict(seed=5, max_steps=T)
    env = VecLoadBalanceEnv(B, S, device="cuda:0", autoreset=True, **kw)
    ora = oracle_mod.OracleEnv(make_config(B, S, **kw), threads=4)
    np.testing.assert_array_equal(env.reset().cpu().numpy(), ora.reset())
    rng = np.random.default_rng(2)
    lib = env.handle.lib  # the shared CDLL: count its reset calls, restore it whatever happens
    real = lib.lbsim_reset_ex
    calls = []
    lib.lbsim_reset_ex = lambda *a: (calls.append(1), real(*a))[1]
    resets_at = []
    try:
        for k in range(3 * T):
            a = rng.integers(0, 3, (B, S)).astype(np.int64)
            n0 = len(calls)
            obs, rew, done, info = env.step(torch.from_numpy(a))
            if len(calls) > n0:
                resets_at.append(k)
            oo, ro, do, _ = ora.step(a)
            np.testing.assert_array_equal(rew.cpu().numpy(), ro)
            np.testing.assert_array_equal(done.cpu().numpy(), do.astype(bool))
            if do.any():
                oo = ora.reset(mask=do, obs=oo)
            np.testing.assert_array_equal(obs.cpu().numpy(), oo, err_msg=f"step {k}")
    finally:
        lib.lbsim_reset_ex = real
    assert resets_at == [T - 1, 2 * T - 1, 3 * T - 1]


def test_vec_actions_any_dtype_and_device():
    from marllb_amd import VecLoadBalanceEnv
    B, S = 64, 4
    envs = [VecLoadBalanceEnv(B, S, device="cuda:0", seed=5, autoreset=False) for _ in range(3)]
    for e in envs:
        e.reset()
    a = np.random.default_rng(0).integers(0, 3, (B, S))
    o1 = envs[0].step(a.astype(np.int64))[0]
    o2 = envs[1].step(torch.from_numpy(a.astype(np.int32)).cuda())[0]
    o3 = envs[2].step(a.tolist())[0]
    assert torch.equal(o1, o2) and torch.equal(o1, o3)


def test_vec_state_snapshot_roundtrip():
    from marllb_amd import VecLoadBalanceEnv
    B, S = 50, 8
    e = VecLoadBalanceEnv(B, S, device="cuda:0", seed=11, autoreset=False)
    e.reset()
    a = torch.ones((B, S), dtype=torch.int64)
    e.step(a)
    snap = e.get_state()
    r1 = [e.step(a)[0].clone() for _ in range(3)]
    e.set_state(snap)
    r2 = [e.step(a)[0].clone() for _ in range(3)]
    assert all(torch.equal(x, y) for x, y in zip(r1, r2))


# ---- SHM bridge (problem-02 wire format): the GPU simulator as the producer
def test_shm_mode_reads_published_frames():
    """A VecLoadBalanceEnv published through marllb_amd.shm.ShmPublisher drives a facade in
    use_shm=True mode: reset/step read the published rows, step's weights arrive in msg_in."""
    import uuid

    from marllb_amd import LoadBalanceEnv, VecLoadBalanceEnv
    from marllb_amd.shm import ShmPublisher
    prefix = f"lbsim_t_{uuid.uuid4().hex[:8]}_"
    vec = VecLoadBalanceEnv(2, 4, device="cuda:0", seed=3, autoreset=False,
                            action_type="continuous")
    pub = ShmPublisher(vec, prefix)
    try:
        o0 = vec.reset()
        pub.publish(o0)
        env = LoadBalanceEnv(num_servers=4, action_type="continuous", use_shm=True,
                             shm_name=prefix + "0", step_interval=0.0, seed=1)
        assert env.use_shm and env.shm is not None
        np.testing.assert_array_equal(env.reset(), o0[0].cpu().numpy())
        o1, r1 = vec.step(torch.full((2, 4), 2.0, device="cuda:0"))[:2]
        pub.publish(o1)  # the producer is a frame ahead of the consumer's step
        obs, reward, done, info = env.step(np.array([0.5, 1.0, 2.0, 4.0], np.float32))
        np.testing.assert_array_equal(obs, o1[0].cpu().numpy())
        assert reward == float(r1[0]) and info["step"] == 1  # lbsim_reward on the frame
        w = pub.poll_actions()
        np.testing.assert_array_equal(w[0], [0.5, 1.0, 2.0, 4.0])
        assert np.isnan(w[1]).all()
        env.close()
    finally:
        pub.close()


# ---- the 1 x 4 GPU facade against the oracle, episode/info semantics against the reference golden
def test_single_env_facade_vs_oracle_and_episode_golden(oracle_mod, golden_dir):
    """LoadBalanceEnv (B=1 on the GPU) stepped past max_steps equals oracle.OracleEnv(B=1) on
    every observation and reward, and its done / info / info['episode'] follow the reference's
    recorded episode (env_plumbing.json['episode'], env.py:262-286 with max_steps=5, 7 steps)."""
    import json
    import os

    from marllb_amd import LoadBalanceEnv
    from marllb_amd.env import make_config
    gold = json.load(open(os.path.join(golden_dir, "env_plumbing.json")))["episode"]
    env = make(num_servers=4, max_steps=5, seed=42, step_interval=0.0)
    ora = oracle_mod.OracleEnv(make_config(1, 4, seed=42, max_steps=5), threads=1)
    np.testing.assert_array_equal(env.reset(), ora.reset()[0])
    total = 0.0
    act = np.array([0, 1, 2, 1])
    for g in gold:
        obs, r, done, info = env.step(act)
        oo, ro, do, _ = ora.step(act[None].astype(np.int64))
        np.testing.assert_array_equal(obs, oo[0])
        assert r == float(ro[0])
        total += r
        assert done == g["done"] and info["step"] == g["info_step"] == g["step"]
        assert sorted(k for k in info if k != "episode") == \
            [k for k in g["info_keys"] if k != "episode"]
        assert ("episode" in info) == g["has_episode"]
        if g["has_episode"]:
            assert info["episode"]["l"] == g["episode_l"]
            assert info["episode"]["r"] == pytest.approx(total, abs=0, rel=1e-12)
        assert isinstance(env, LoadBalanceEnv)


def test_single_env_normalized_matches_oracle(oracle_mod):
    """normalize_obs through the single-transfer step path: obs normalised on the device, reward
    and active servers from the raw row (oracle normalises with the same f64 statistics)."""
    from marllb_amd.env import make_config
    env = make(num_servers=4, normalize_obs=True, seed=9, action_type="continuous")
    ora = oracle_mod.OracleEnv(make_config(1, 4, seed=9, normalize_obs=True,
                                           action_type="continuous"), threads=1)
    np.testing.assert_array_equal(env.reset(), ora.reset()[0])
    rng = np.random.default_rng(4)
    for _ in range(4):
        a = rng.uniform(-1, 3, 4).astype(np.float32)
        obs, r, _, info = env.step(a)
        oo, ro, _, _ = ora.step(a[None])
        np.testing.assert_array_equal(obs, oo[0])
        assert r == float(ro[0])


def test_shm_fallback_when_producer_is_idle():
    """use_shm=True: a step that finds no new frame falls back to the simulator (env.py:246-254)
    instead of raising; the SHM reset already reset the simulator."""
    import uuid

    from marllb_amd import LoadBalanceEnv, VecLoadBalanceEnv
    from marllb_amd.shm import ShmPublisher
    prefix = f"lbsim_f_{uuid.uuid4().hex[:8]}_"
    vec = VecLoadBalanceEnv(1, 4, device="cuda:0", seed=3, autoreset=False)
    pub = ShmPublisher(vec, prefix)
    try:
        pub.publish(vec.reset())
        env = LoadBalanceEnv(num_servers=4, use_shm=True, shm_name=prefix + "0",
                             step_interval=0.0, seed=1, normalize_obs=True)
        env.reset()
        for k in range(3):  # the producer never publishes again
            obs, r, done, info = env.step(np.array([0, 1, 2, 1]))
            assert obs.shape == (4, 11) and np.all(np.isfinite(obs)) and info["step"] == k + 1
            assert isinstance(r, float) and np.isfinite(r)
        assert env._norm[0] == 4  # one host running statistic over the frame and 3 fallbacks
        env.close()
    finally:
        pub.close()


def test_reset_mask_validation():
    from marllb_amd import VecLoadBalanceEnv
    env = VecLoadBalanceEnv(32, 4, device="cuda:0", seed=1)
    env.reset()
    with pytest.raises(ValueError, match="num_envs"):
        env.reset(mask=torch.ones(16, dtype=torch.bool))
    with pytest.raises(ValueError, match="bool or uint8"):
        env.reset(mask=torch.ones(32, dtype=torch.float32))
    env.reset(mask=torch.zeros(32, dtype=torch.bool, device="cuda:0"))
    with pytest.raises(ValueError, match="expected 32 x 4"):
        env.step(torch.zeros((32, 3), dtype=torch.int64))
    strict = VecLoadBalanceEnv(8, 4, device="cuda:0", seed=1, strict_actions=True)
    strict.reset()
    with pytest.raises(IndexError):
        strict.step(torch.full((8, 4), 3, dtype=torch.int64))
    strict.step(torch.full((8, 4), -3, dtype=torch.int64))  # python indexing: -n is valid


def test_profiler_counts_and_times_every_launch():
    """lbsim_profile_begin/end (bench.py's live kernel timing): every step's dynamics and observe
    launches are timed (the step's middle event shared by both), resets are their own classes, and
    the per-class sums are positive and below the wall time of the region."""
    import ctypes
    import time
    from marllb_amd import _lib
    from marllb_amd.env import VecLoadBalanceEnv
    env = VecLoadBalanceEnv(4096, 4, device="cuda:0", seed=3, step_kernel="split")
    env.reset()
    lib, h = _lib.load(), env.handle
    h.check(lib.lbsim_profile_begin(h.h, 64))
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(7):
        env.step(torch.randint(0, 3, (4096, 4), device="cuda:0"))
    env.reset()
    torch.cuda.synchronize()
    wall_ms = (time.perf_counter() - t0) * 1e3
    ms = (ctypes.c_double * 4)()
    cnt = (ctypes.c_int64 * 4)()
    h.check(lib.lbsim_profile_end(h.h, ms, cnt))
    assert list(cnt) == [7, 7, 1, 1]
    assert all(m > 0 for m in ms) and sum(ms) < wall_ms
    # capacity: with room for 3 launches only the first ones are timed, nothing overflows
    h.check(lib.lbsim_profile_begin(h.h, 2))
    for _ in range(3):
        env.step(torch.randint(0, 3, (4096, 4), device="cuda:0"))
    h.check(lib.lbsim_profile_end(h.h, ms, cnt))
    assert cnt[0] + cnt[1] <= 3 and cnt[0] >= 1
    env.close()
    # the fused step kernel: one launch per step, class 4 (lbsim_profile_end_ex)
    env = VecLoadBalanceEnv(4096, 4, device="cuda:0", seed=3, step_kernel="fused")
    env.reset()
    h = env.handle
    h.check(lib.lbsim_profile_begin(h.h, 64))
    for _ in range(5):
        env.step(torch.randint(0, 3, (4096, 4), device="cuda:0"))
    ms5 = (ctypes.c_double * 5)()
    cnt5 = (ctypes.c_int64 * 5)()
    h.check(lib.lbsim_profile_end_ex(h.h, ms5, cnt5, 5))
    assert list(cnt5) == [0, 0, 0, 0, 5] and ms5[4] > 0
    assert lib.lbsim_profile_end_ex(h.h, ms5, cnt5, 6) == _lib.EINVAL
    env.close()


def test_timing_event_times_a_launch_on_torch_stream():
    """_lib.TimingEvent (the fence-free HIP event bench.py times the policy launches with) brackets
    work on torch's current stream: positive, below the wall time, and ordered like torch's own
    events around the same work."""
    import time
    from marllb_amd import _lib
    x = torch.randn(4096, 4096, device="cuda:0")
    stream = torch.cuda.current_stream().cuda_stream
    e0, e1 = _lib.TimingEvent(), _lib.TimingEvent()
    t0, t1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    w0 = time.perf_counter()
    e0.record(stream)
    t0.record()
    for _ in range(4):
        x = x @ x * 1e-3
    t1.record()
    e1.record(stream)
    torch.cuda.synchronize()
    wall_ms = (time.perf_counter() - w0) * 1e3
    ms, ref = e0.elapsed_time(e1), t0.elapsed_time(t1)
    assert 0.0 < ms < wall_ms
    assert ms >= 0.5 * ref  # the fence-free pair encloses torch's pair
