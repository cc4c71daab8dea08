"""The duration sample and the optional dynamics of DESIGN.md §3.4 / §3.9 on the CPU oracle (their GPU parity is in
tests/test_gpu_parity.py CONFIGS): lost-FIN flows (VPP's timed-out flow sample,
src/vpp/lb/lbhash.h:175-217) and server failure / recovery (problem-03 THEORY.md §6.4).

Parity vs the reference is unpinned for both, as for the rest of the flow dynamics (the reference's
simulation mode has none): these tests pin the oracle's restatement to the semantics it states --
off means bit-identical, the right flows are changed by the right amount, failed servers are empty,
ineligible and inactive.
"""
import numpy as np
import pytest

from tests import statelayout

pytest.importorskip("torch")


def _run(oracle_mod, B, S, steps, seed=5, **kw):
    from marllb_amd.env import make_config
    cfg = make_config(B, S, seed=seed, **kw)
    ora = oracle_mod.OracleEnv(cfg, threads=4)
    ora.reset()
    rng = np.random.default_rng(seed)
    out = []
    for _ in range(steps):
        out.append(ora.step(rng.integers(0, 3, (B, S)).astype(np.int64)))
    st = statelayout.parse(ora.state_bytes(), B, S, cfg.queue_capacity, False, cfg.fail_prob > 0,
                           statelayout.has_leak(cfg), split_P=statelayout.split_p(cfg))
    ora.close()
    return st, out


def test_options_off_are_bit_identical(oracle_mod):
    """lost_fin_prob = 0 ignores flow_timeout / flow_buckets and fail_prob = 0 ignores
    recover_prob: the state and every output equal the default run's."""
    st0, out0 = _run(oracle_mod, 64, 4, 6)
    st1, out1 = _run(oracle_mod, 64, 4, 6, flow_timeout=3.0, flow_buckets=7, recover_prob=0.9)
    for k in st0:
        np.testing.assert_array_equal(st0[k], st1[k], err_msg=k)
    for a, b in zip(out0, out1):
        for x, y in zip(a, b):
            np.testing.assert_array_equal(x, y)


def _run_split(oracle_mod, B, S, steps, seed=5, **kw):
    """_run for a lost-FIN handle: its snapshot has the split sections (statelayout.split_p)."""
    from marllb_amd.env import make_config
    cfg = make_config(B, S, seed=seed, **kw)
    ora = oracle_mod.OracleEnv(cfg, threads=4)
    ora.reset()
    rng = np.random.default_rng(seed)
    states = []
    for _ in range(steps):
        ora.step(rng.integers(0, 3, (B, S)).astype(np.int64))
        states.append(statelayout.parse(ora.state_bytes(), B, S, cfg.queue_capacity, False,
                                        split_P=statelayout.split_p(cfg)))
    ora.close()
    return cfg, states


def test_lost_fin_guesses_wait_for_their_wrap_up(oracle_mod):
    """Lost-FIN flows (lbhash.h:175-217): the data plane wraps a timed-out flow up only when the
    next flow hits its bucket, flow_timeout + wait after its last packet, recording
    now - t_init - 40 s at that moment.  So: the queues and the duration reservoir (every flow's
    age at its last packet, recorded at the completion, lbhash.h:129-136) are exactly those of a
    run without losses; each lost flow's fct sample waits in its server's pending ring, sorted by
    due time, and enters the fct reservoir at the wrap-up; completions = fct samples of
    delivered flows + flushed guesses + pending + dropped at a full ring."""
    B, S, steps = 96, 4, 10
    st0, _ = _run(oracle_mod, B, S, steps)
    for p, timeout, buckets, P in ((1.0, 40.0, 1024, 256), (0.3, 0.3, 16, 256),
                                   (0.5, 0.2, 32, 3)):
        cfg, states = _run_split(oracle_mod, B, S, steps, lost_fin_prob=p, flow_timeout=timeout,
                                 flow_buckets=buckets, lost_fin_pending=P)
        st = states[-1]
        for k in ("res_count", "dropped", "clock", "arr_idx"):
            if k == "res_count":  # all completions: the duration reservoir's count
                np.testing.assert_array_equal(st["res_count_dur"], st0["res_count"])
            else:
                np.testing.assert_array_equal(st[k], st0[k], err_msg=k)
        np.testing.assert_array_equal(st["hc"] & ~np.uint32(0x8000), st0["hc"] & ~np.uint32(0x8000))
        # the duration reservoir is the lossless run's reservoir, slot for slot
        n = np.minimum(st0["res_count"], 128).reshape(B, S)
        valid = (np.arange(128)[None, None, :] < n[:, :, None]).reshape(-1)
        np.testing.assert_array_equal(st["res_dur"][valid], st0["res_dur"][valid])
        np.testing.assert_array_equal(st["res_dur_ts"][valid], st0["res_ts"][valid])
        # conservation: completions = fct samples + pending + dropped guesses
        pend = (st["pend_hc"] >> 16).astype(np.int64).reshape(B, S)
        fct_n = st["res_count"].astype(np.int64).reshape(B, S)
        comp = st["res_count_dur"].astype(np.int64).reshape(B, S)
        over = st["lf_over"].astype(np.int64)
        np.testing.assert_array_equal((comp - fct_n - pend).sum(1), over)
        assert (pend <= P).all()
        if P < 8:
            assert over.sum() > 0  # full rings drop guesses (counted)
        # every pending guess is due after the step's end, rings sorted by due time
        live = statelayout.live_pend(st, B, S, P)
        clock = st["clock"].astype(np.int64)
        dt = int(round(cfg.step_interval * 1e6))
        now = (clock * dt) & 0xFFFFFFFF
        for bb in range(B):
            for ss in range(S):
                c = int(pend[bb, ss])
                due = live[bb, ss, :c, 0].astype(np.int64)
                rel = ((due - now[bb] + 2**31) % 2**32) - 2**31
                assert (rel > 0).all()
                assert (np.diff(rel) >= 0).all()
        if timeout == 40.0:
            # 10 steps of 0.25 s: no guess is due yet, so the fct reservoir holds exactly the
            # delivered flows -- none at p = 1
            assert fct_n.sum() == 0
            np.testing.assert_array_equal(pend, np.minimum(comp, P))  # full rings drop the rest
        else:
            # a 0.2-0.3 s timeout and a ~40-80 ms bucket wait: the guesses (fct + timeout - 40 s
            # + wait: negative) reach the fct reservoir a step or two after their flows
            nf = np.minimum(st["res_count"], 128).reshape(B, S)
            vf = (np.arange(128)[None, None, :] < nf[:, :, None]).reshape(-1)
            f = st["res_fct"].view(np.int32)[vf]
            neg = (f < 0).mean()
            if P >= 8:
                assert abs(neg - p) < 0.08, (neg, p)
            else:  # most guesses dropped at the 3-entry rings
                assert 0 < neg < p - 0.1, (neg, p)
            # each guess is stamped with its wrap-up time: no earlier than the timeout after the
            # earliest possible completion (the episode start)
            ts = st["res_ts"][vf][f < 0]
            assert (ts >= int(timeout * 1000)).all()


def test_server_failures(oracle_mod):
    """fail_prob / recover_prob per server and step: the stationary down fraction is
    fail / (fail + recover); a down server is empty (no queue, no samples: an all-zero
    observation row, inactive in the reward, env.py:410-413), takes no flows, and its lost queue
    counts as dropped."""
    from marllb_amd.env import make_config
    B, S, steps, pf, pr = 128, 4, 40, 0.1, 0.15
    cfg = make_config(B, S, seed=11, fail_prob=pf, recover_prob=pr)
    ora = oracle_mod.OracleEnv(cfg, threads=4)
    ora.reset()
    rng = np.random.default_rng(0)
    down_frac = []
    dropped_prev = 0
    for k in range(steps):
        obs, rew, done, assign = ora.step(rng.integers(0, 3, (B, S)).astype(np.int64))
        st = statelayout.parse(ora.state_bytes(), B, S, cfg.queue_capacity, False, True)
        down = st["down"].reshape(B, S).astype(bool)
        assert (obs[down] == 0).all(), "a down server's row is all zeros"
        assert (assign[down] == 0).all(), "a down server takes no flows"
        assert (st["res_count"].reshape(B, S)[down] == 0).all()
        assert ((st["hc"] >> 16).reshape(B, S)[down] == 0).all()
        if k >= 15:
            down_frac.append(down.mean())
        dropped_prev = int(st["dropped"].sum())
    ora.close()
    f = float(np.mean(down_frac))
    assert abs(f - pf / (pf + pr)) < 0.05, f
    assert dropped_prev > 0, "failed queues count as dropped"


def test_server_failures_reward_uses_active_rows(oracle_mod):
    """The reward of a step with down servers equals the reference rule over the rows with any
    column > 0 (env.py:410-413 -> rewards.py compute), evaluated by the library's stateless
    reward entry point's oracle twin on the returned observation."""
    from marllb_amd.env import make_config
    B, S = 64, 6
    cfg = make_config(B, S, seed=3, fail_prob=0.25, recover_prob=0.2, reward_metric="jain",
                      reward_field="fct_mean")
    ora = oracle_mod.OracleEnv(cfg, threads=4)
    ora.reset()
    rng = np.random.default_rng(1)
    some_down = False
    for _ in range(8):
        obs, rew, _, _ = ora.step(rng.integers(0, 3, (B, S)).astype(np.int64))
        active = (obs > 0).any(2)
        some_down |= bool((~active).any())
        for b in range(B):
            x = obs[b, active[b], 1].astype(np.float64)  # fct_mean column
            if len(x) == 0:
                want = 0.0
            else:
                sv, sq = x.sum(), (x * x).sum()
                want = 1.0 if sv < 1e-10 or sq < 1e-10 else sv * sv / (len(x) * sq)
            assert abs(float(rew[b]) - want) <= 1e-6 * max(1.0, abs(want)), (b, rew[b], want)
    assert some_down
    ora.close()


def test_next_step_reset_equals_same_step_shifted(oracle_mod):
    """Next-step auto-reset (gymnasium NEXT_STEP) on the oracle: the step that ends an episode
    returns the terminal obs with done; the next step resets the env instead of stepping it
    (action ignored; reward 0, done 0) and returns exactly the observation a same-step reset
    returns (a reset does not depend on the episode before it), after which both runs walk the
    same trajectory when fed the same actions."""
    from marllb_amd.env import make_config
    B, S, T = 48, 4, 3
    nxt = oracle_mod.OracleEnv(make_config(B, S, seed=9, max_steps=T, next_step_reset=True), threads=4)
    same = oracle_mod.OracleEnv(make_config(B, S, seed=9, max_steps=T), threads=4)
    np.testing.assert_array_equal(nxt.reset(), same.reset())
    rng = np.random.default_rng(2)
    acts = [rng.integers(0, 3, (B, S)).astype(np.int64) for _ in range(3 * T)]
    for k in range(T):  # the first episode: identical
        o1, r1, d1, a1 = nxt.step(acts[k])
        o2, r2, d2, a2 = same.step(acts[k])
        for x, y in ((o1, o2), (r1, r2), (d1, d2), (a1, a2)):
            np.testing.assert_array_equal(x, y)
    assert d1.all()
    reset_obs = same.reset(mask=d2.astype(np.uint8), obs=o2.copy())  # same-step: reset now
    o1, r1, d1, a1 = nxt.step(acts[T])  # next-step: this step resets, its action ignored
    np.testing.assert_array_equal(o1, reset_obs)
    assert (r1 == 0).all() and not d1.any() and (a1 == 0).all()
    ln, rt = nxt.episode_stats()
    assert (ln == 0).all() and (rt == 0).all()
    for k in range(T + 1, 2 * T + 1):  # the second episode, actions shifted by one step
        o1, r1, d1, _ = nxt.step(acts[k])
        o2, r2, d2, _ = same.step(acts[k])
        np.testing.assert_array_equal(o1, o2)
        np.testing.assert_array_equal(r1, r2)
        np.testing.assert_array_equal(d1, d2)
    np.testing.assert_array_equal(nxt.state_bytes(), same.state_bytes())
    nxt.close()
    same.close()


def test_duration_sample_is_the_flow_age(oracle_mod):
    """duration_mode="age" (default): the flow-duration sample is the flow's age at its last data
    packet, completion - arrival (VPP records time_now - t_init on every plain ACK after the first,
    src/vpp/lb/lbhash.h:129-136), so it includes the backlog wait: with lost-FIN off it equals the
    fct sample slot for slot, it is >= the service time of duration_mode="service", and strictly
    larger for flows that queued.  Everything else (queues, slots, counts, fct, timestamps) is the
    same in both modes (the feature cache and the episode return follow the samples)."""
    B, S, steps = 96, 4, 8
    age, _ = _run(oracle_mod, B, S, steps, load=1.1)
    svc, _ = _run(oracle_mod, B, S, steps, load=1.1, duration_mode="service")
    for k in age:
        if k not in ("res", "res_dur", "fcache", "ep_return"):
            np.testing.assert_array_equal(age[k], svc[k], err_msg=k)
    n = np.minimum(age["res_count"], 128).reshape(B, S)
    valid = (np.arange(128)[None, None, :] < n[:, :, None]).reshape(-1)
    a = age["res_dur"][valid].astype(np.int64)
    s = svc["res_dur"][valid].astype(np.int64)
    np.testing.assert_array_equal(a, age["res_fct"][valid].astype(np.int64))
    assert (a >= s).all() and (s >= 1).all()
    assert (a > s).mean() > 0.3, "at load 1.1 most flows wait behind another"


def _reward_balanced_vs_skewed(oracle_mod, **kw):
    """Mean default reward (Jain over column 10, flow_duration_avg_decay) of 512 envs x 4 servers
    over 40 steps after 20, all weights 1.0 vs weights [2, 1, 1, 1] (discrete levels 0 / 2)."""
    from marllb_amd.env import make_config
    out = []
    for row in ([0, 0, 0, 0], [2, 0, 0, 0]):
        ora = oracle_mod.OracleEnv(make_config(512, 4, seed=7, **kw), threads=8)
        ora.reset()
        a = np.tile(np.array(row, np.int64), (512, 1))
        for _ in range(20):
            ora.step(a)
        out.append(float(np.mean([ora.step(a)[1].mean() for _ in range(40)])))
        ora.close()
    return out


def test_default_reward_sees_the_policy(oracle_mod):
    """problem-03's reward is Jain fairness over flow_duration_avg_decay (THEORY.md:616, env.py:79).
    With the duration sample as the flow's age the skewed weights [2, 1, 1, 1] -- server 0 carries
    ~2.7x the flows in flight -- lower the reward by >= 0.03; with the service-time sample
    (duration_mode="service") the reward cannot see the policy (the two differ by < 0.005)."""
    bal, skew = _reward_balanced_vs_skewed(oracle_mod)
    assert bal - skew >= 0.03, (bal, skew)
    bal_s, skew_s = _reward_balanced_vs_skewed(oracle_mod, duration_mode="service")
    assert abs(bal_s - skew_s) < 0.005, (bal_s, skew_s)


def test_lost_fin_guess_at_the_accepted_limit(oracle_mod):
    """The largest accepted lost-FIN timeout (flow_timeout + 16.7 x the mean bucket wait = 1040 s):
    every guess stays a positive signed 32-bit us value and its wrap-up delay flow_timeout + wait
    a positive signed 32-bit us offset (no int32 wrap); all of them still pending
    after 6 steps."""
    B, S, steps = 64, 4, 6
    timeout = 1040.0 - 16.7 * 1024 / 400.0  # flow_buckets 1024 at 400 flows/s: 997.25 s
    st, _ = _run(oracle_mod, B, S, steps, lost_fin_prob=1.0, flow_timeout=timeout)
    pend = (st["pend_hc"] >> 16).reshape(B, S)
    comp = st["res_count_dur"].reshape(B, S).astype(np.int64)
    # every flow lost and nothing due for 997 s: the 256-entry rings fill, the rest is dropped
    np.testing.assert_array_equal(pend, np.minimum(comp, 256))
    np.testing.assert_array_equal(st["lf_over"], np.maximum(comp - 256, 0).sum(1))
    assert (st["res_count"] == 0).all()
    live = statelayout.live_pend(st, B, S, 256)
    now = (st["clock"].astype(np.int64) * 250000) & 0xFFFFFFFF
    for bb in range(B):
        for ss in range(S):
            c = int(pend[bb, ss])
            g = live[bb, ss, :c, 1].view(np.int32).astype(np.int64)
            assert (g > 0).all() and (g < 2 ** 31 - 1).all()
            rel = ((live[bb, ss, :c, 0].astype(np.int64) - now[bb] + 2**31) % 2**32) - 2**31
            assert (rel > 0).all() and (rel <= 1040e6).all()
    # a larger timeout is rejected
    from marllb_amd.env import make_config
    with pytest.raises(ValueError):
        make_config(B, S, lost_fin_prob=1.0, flow_timeout=timeout + 1.0)


def test_n_flow_on_vpp_counts_lost_flows(oracle_mod):
    """n_flow_on_mode="vpp": VPP's n_flow_on is +1 at a flow's first ACK and -1 at its RSTACK
    (lbhash.h:116-120,138-142,167) and a lost-FIN flow is never decremented (lbhash.h:193,214):
    column 0 = the flows in flight + the server's lost-FIN flows since the episode start, and the
    SED / LSQ scores read that same count (node.c:395-437 score on as_stat n_flow_on).
    The leak grows step by step at about lost_fin_prob x the completions; off without lost-FIN (no
    state section, bit-identical)."""
    from marllb_amd.env import make_config
    B, S, steps = 64, 4, 6
    outs = {}
    for mode in ("queue", "vpp"):
        cfg = make_config(B, S, seed=5, lost_fin_prob=0.25, n_flow_on_mode=mode)
        ora = oracle_mod.OracleEnv(cfg, threads=4)
        ora.reset()
        rng = np.random.default_rng(5)
        outs[mode] = [ora.step(rng.integers(0, 3, (B, S)).astype(np.int64)) for _ in range(steps)]
        outs[mode + "_st"] = statelayout.parse(ora.state_bytes(), B, S, cfg.queue_capacity, False,
                                               False, statelayout.has_leak(cfg),
                                               split_P=statelayout.split_p(cfg))
        ora.close()
    st_q, st_v = outs["queue_st"], outs["vpp_st"]
    # the leaky count steers the assignments, so the two runs differ ...
    assert not np.array_equal(st_q["hc"], st_v["hc"])
    # ... and column 0 is the queue plus the lost flows, the other columns the reservoirs
    leak = st_v["lost_on"].reshape(B, S).astype(np.float32)
    queue = (st_v["hc"] >> 16).reshape(B, S).astype(np.float32)
    o_v = outs["vpp"][-1][0]
    np.testing.assert_array_equal(o_v[:, :, 0], queue + leak)
    prev = None
    for (ov, *_), (oq, *_) in zip(outs["vpp"], outs["queue"]):
        d = ov[:, :, 0]
        if prev is not None:
            assert (d.sum(1) >= prev.sum(1) - 2 * S * 8).all()  # in flight may drop; leak never
        prev = d
    # completions per server-step ~ arrivals (100 per env-step over 4 servers) at 25 % lost
    per_step = leak.mean() / (steps + 8)  # 8 warm-up steps
    assert 0.15 * 25 < per_step < 0.35 * 25, per_step

    # every flow lost, LSQ: a server's leaky count only grows (+1 per assignment, the completion
    # moves the flow from the queue to the leak), so LSQ on it balances the flows ASSIGNED since
    # the episode start -- within one of each other in every env after every step
    for policy in ("lsq", "sed"):
        cfg = make_config(B, S, seed=9, lost_fin_prob=1.0, n_flow_on_mode="vpp",
                          assign_policy=policy)
        ora = oracle_mod.OracleEnv(cfg, threads=4)
        ora.reset()
        for _ in range(4):  # equal weights: SED = (n + 1) / w is the same order as LSQ
            obs, *_ = ora.step(np.zeros((B, S), np.int64))
            col0 = obs[:, :, 0]
            assert (col0.max(1) - col0.min(1) <= 1).all(), (policy, col0[:4])
        ora.close()
    # without lost-FIN the mode changes nothing (no section)
    a = make_config(B, S, seed=5, n_flow_on_mode="vpp")
    assert not statelayout.has_leak(a)
