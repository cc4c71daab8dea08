"""GPU (liblbsim, gfx950 kernels) against the CPU oracle and the reference golden vectors.

Bar (north star): server-assignment indices and every integer state word bit-exact under the same
Philox key; fp32 observations/rewards within 1e-5 — in practice the kernels reproduce the oracle
bit for bit on every observation column (same op order, -ffp-contract=off), so the
tests assert exact equality and fall back to the tolerance only where noted.
"""
import ctypes
import os

import numpy as np
import pytest

from tests import statelayout

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

FIELD_COL = {"flow_duration_avg_decay": 10, "n_flow_on": 0, "fct_mean": 1, "no_such_field": -1}


@pytest.fixture(scope="module")
def lib():
    if not torch.cuda.is_available():
        pytest.fail("GPU test run without a HIP device")
    from marllb_amd import _lib
    return _lib


def dev(a, dtype=None):
    t = torch.from_numpy(np.ascontiguousarray(a))
    return t.to("cuda:0") if dtype is None else t.to("cuda:0", dtype)


# ------------------------------------------------------------------ stateless kernels
def test_features_kernel_matches_reference_and_oracle(lib, oracle_mod, golden_dir):
    g = np.load(os.path.join(golden_dir, "reservoir_features.npz"))
    v, t, c = dev(g["values"]), dev(g["ts_ms"]), dev(g["counts"])
    n = len(g["counts"])
    out = torch.empty((n, 5), dtype=torch.float32, device="cuda:0")
    rc = lib.load().lbsim_reservoir_features(v.data_ptr(), t.data_ptr(), c.data_ptr(), n, 0.9,
                                             out.data_ptr(), None)
    assert rc == 0
    torch.cuda.synchronize()
    got = out.cpu().numpy()
    ora = oracle_mod.features(g["values"], g["ts_ms"], g["counts"], 0.9)
    np.testing.assert_array_equal(got, ora)  # all 5 columns bit-exact vs the oracle
    exp = g["expected"]
    for f in (0, 1, 2, 4):
        np.testing.assert_array_equal(got[:, f], exp[:, f].astype(np.float32))
    rel = np.abs(got[:, 3] - exp[:, 3]) / np.maximum(np.abs(exp[:, 3]), 1e-30)
    assert rel.max() < 2e-6


@pytest.mark.parametrize("S", [1, 2, 3, 4, 8, 16])
def test_reward_kernel_matches_reference(lib, oracle_mod, golden_dir, S):
    g = np.load(os.path.join(golden_dir, "rewards.npz"))
    obs, exp = g[f"obs_S{S}"], g[f"expected_S{S}"]
    metrics, fields = list(g["metrics"]), list(g["fields"])
    o = dev(obs)
    out = torch.empty(len(obs), dtype=torch.float32, device="cuda:0")
    for m in range(len(metrics)):
        for fi, fname in enumerate(fields):
            cfg = lib.default_config()
            cfg.num_servers, cfg.reward_metric, cfg.reward_field = S, m, FIELD_COL[str(fname)]
            assert lib.load().lbsim_reward(ctypes.byref(cfg), o.data_ptr(), len(obs),
                                           out.data_ptr(), None) == 0
            torch.cuda.synchronize()
            got = out.cpu().numpy()
            want = exp[:, m, fi].astype(np.float32)
            tol = 0 if metrics[m] != "product" else 1e-6  # device log() vs glibc log()
            np.testing.assert_allclose(got, want, rtol=tol, atol=0, err_msg=f"{metrics[m]} {fname}")
            np.testing.assert_allclose(got, oracle_mod.rewards(obs, m, FIELD_COL[str(fname)]),
                                       rtol=tol, atol=0)


def test_alias_tables_kernel_matches_reference(lib, oracle_mod, golden_dir):
    """The per-step ALIAS table build (dynamics_kernel's build_alias) against the reference
    gen_alias (src/lb/shm_proxy.py:127-146): odd as the float32 the reference packs, alias index
    exact, on every golden row (padded rows of equal S share one launch)."""
    import json
    cases = json.load(open(os.path.join(golden_dir, "alias.json")))["cases"]
    for S in sorted({len(c["weights"]) for c in cases}):
        rows = [c for c in cases if len(c["weights"]) == S]
        w = dev(np.array([c["weights"] for c in rows], np.float32))
        n = len(rows)
        odd = torch.empty((n, S), dtype=torch.float32, device="cuda:0")
        ali = torch.empty((n, S), dtype=torch.int32, device="cuda:0")
        act = torch.empty((n, S), dtype=torch.int32, device="cuda:0")
        assert lib.load().lbsim_alias_tables(w.data_ptr(), n, S, odd.data_ptr(), ali.data_ptr(),
                                             act.data_ptr(), None) == 0
        torch.cuda.synchronize()
        np.testing.assert_array_equal(odd.cpu().numpy(),
                                      np.array([c["odd"] for c in rows], np.float32))
        np.testing.assert_array_equal(ali.cpu().numpy(), np.array([c["alias"] for c in rows]))
        np.testing.assert_array_equal(act.cpu().numpy(), np.tile(np.arange(S), (n, 1)))
    # rows with non-positive weights: the active list skips them (register_as_weights)
    w = np.array([[0.0, 2.0, 0.0, 1.0], [0.0, 0.0, 0.0, 0.0], [3.0, -1.0, 1.0, 1.0]], np.float32)
    odd = torch.empty((3, 4), dtype=torch.float32, device="cuda:0")
    ali = torch.empty((3, 4), dtype=torch.int32, device="cuda:0")
    act = torch.empty((3, 4), dtype=torch.int32, device="cuda:0")
    assert lib.load().lbsim_alias_tables(dev(w).data_ptr(), 3, 4, odd.data_ptr(), ali.data_ptr(),
                                         act.data_ptr(), None) == 0
    torch.cuda.synchronize()
    for r in range(3):
        keep = np.flatnonzero(w[r] > 0)
        o, a = oracle_mod.gen_alias(w[r, keep])
        np.testing.assert_array_equal(act.cpu().numpy()[r, :len(keep)], keep)
        np.testing.assert_array_equal(odd.cpu().numpy()[r, :len(keep)], o.astype(np.float32))
        np.testing.assert_array_equal(ali.cpu().numpy()[r, :len(keep)], a)
        assert (act.cpu().numpy()[r, len(keep):] == -1).all()


def test_vose_kernels_match_oracle(lib, oracle_mod):
    """problem-07's Vose alias tables (vpp-plugin/alias_table.h:82-158) built on the GPU equal
    oracle_vose_build bit for bit (prob as float32 bits, alias indices), and alias_table_sample
    (:163-209) driven from the same xorshift32 states gives the same picks, histograms and final
    states.  Rows: ragged S 1..64, zero / all-zero / negative-sum / wide-range weights.
    (Parity vs the C itself is unpinned: alias_table.h needs vppinfra to compile.)"""
    from tests.test_oracle_golden import vose_rows
    rows = vose_rows(11)
    by_s = {}
    for w in rows:
        by_s.setdefault(len(w), []).append(w)
    K = 300
    for S, ws in sorted(by_s.items()):
        w = np.stack(ws).astype(np.float32)
        n = len(w)
        prob = torch.empty((n, S), dtype=torch.float32, device="cuda:0")
        ali = torch.empty((n, S), dtype=torch.int32, device="cuda:0")
        assert lib.load().lbsim_vose_tables(dev(w).data_ptr(), n, S, prob.data_ptr(),
                                            ali.data_ptr(), None) == 0
        states0 = (np.arange(n, dtype=np.uint64) * 2654435761 + S + 1).astype(np.uint32)
        st = dev(states0.view(np.int32))
        idx = torch.empty((n, K), dtype=torch.int32, device="cuda:0")
        hist = torch.empty((n, S), dtype=torch.int64, device="cuda:0")
        assert lib.load().lbsim_vose_sample(prob.data_ptr(), ali.data_ptr(), n, S, st.data_ptr(),
                                            K, idx.data_ptr(), hist.data_ptr(), None) == 0
        torch.cuda.synchronize()
        gp, ga = prob.cpu().numpy(), ali.cpu().numpy().view(np.uint32)
        gi, gh = idx.cpu().numpy(), hist.cpu().numpy()
        gs = st.cpu().numpy().view(np.uint32)
        for r in range(n):
            p, a = oracle_mod.vose_build(w[r])
            np.testing.assert_array_equal(gp[r].view(np.uint32), p.view(np.uint32))
            np.testing.assert_array_equal(ga[r], a)
            oi, oh, os_ = oracle_mod.vose_sample(p, a, int(states0[r]), K)
            np.testing.assert_array_equal(gi[r], oi)
            np.testing.assert_array_equal(gh[r], oh.astype(np.int64))
            assert int(gs[r]) == os_
    # large batch, histogram only: frequencies follow the weights
    n, S, K = 4096, 8, 20000
    w = np.tile(np.array([1, 2, 0, 4, 1, 1, 0.5, 0.5], np.float32), (n, 1))
    prob = torch.empty((n, S), dtype=torch.float32, device="cuda:0")
    ali = torch.empty((n, S), dtype=torch.int32, device="cuda:0")
    assert lib.load().lbsim_vose_tables(dev(w).data_ptr(), n, S, prob.data_ptr(), ali.data_ptr(),
                                        None) == 0
    st = dev((np.arange(n, dtype=np.uint32) * 7 + 1).view(np.int32))
    hist = torch.empty((n, S), dtype=torch.int64, device="cuda:0")
    assert lib.load().lbsim_vose_sample(prob.data_ptr(), ali.data_ptr(), n, S, st.data_ptr(), K,
                                        None, hist.data_ptr(), None) == 0
    freq = hist.sum(0).double().cpu().numpy() / (n * K)
    np.testing.assert_allclose(freq, w[0] / w[0].sum(), atol=2e-4)
    assert lib.load().lbsim_vose_sample(prob.data_ptr(), ali.data_ptr(), n, 0, st.data_ptr(), K,
                                        None, None, None) < 0


# ------------------------------------------------------------------ the simulator
CONFIGS = [
    dict(B=257, S=4, kw={}),
    dict(B=130, S=1, kw={}),
    dict(B=96, S=8, kw={"assign_policy": "sed2", "arrival_rate": 500.0}),
    dict(B=64, S=16, kw={"assign_policy": "lsq", "action_type": "continuous"}),
    dict(B=70, S=5, kw={"assign_policy": "lsq2", "normalize_obs": True, "queue_capacity": 3,
                        "server_rates": [30.0, 60.0, 90.0, 120.0, 40.0]}),
    dict(B=33, S=4, kw={"action_type": "continuous", "reward_metric": "gini",
                        "server_rates": [50.0, 100.0, 200.0, 400.0], "warmup_steps": 0,
                        "step_interval": 0.05}),
    dict(B=40, S=6, kw={"reward_metric": "variance", "reward_field": "fct_mean",
                        "discrete_weights": [0.25, 1.0, 4.0, 9.0], "queue_capacity": 64,
                        "max_steps": 7}),
    # slow servers, 5 s steps: flows wait > 2^25 us (33 s), so observe takes the two-pass sort
    dict(B=48, S=4, kw={"server_rates": [1.0, 1.0, 1.5, 2.0], "arrival_rate": 20.0,
                        "step_interval": 5.0, "queue_capacity": 64}),
    # ALIAS (node.c:442-460 over gen_alias): continuous weights; discrete with a zero level, so
    # servers drop out of the active list and all-zero rows drop every arrival
    dict(B=100, S=6, kw={"assign_policy": "alias", "action_type": "continuous"}),
    dict(B=80, S=4, kw={"assign_policy": "alias", "discrete_weights": [0.0, 1.0, 3.0]}),
    # TRACE arrivals (configs[2] shape, small B): the converted rate_500 trace, and a 37-row
    # synthetic trace that every env wraps around many times per episode
    dict(B=64, S=8, kw={"trace": "builtin"}),
    dict(B=50, S=4, kw={"trace": "short", "assign_policy": "sed2", "step_interval": 0.5}),
    # NaN continuous actions pass np.clip (env.py:349-351): NaN SED scores take the exact scan
    dict(B=60, S=5, kw={"action_type": "continuous", "_nan_actions": 0.15}),
    # observe's unchanged-reservoir skip: sparse arrivals -> many env-steps write
    # no reservoir slot (cached features) next to env-steps that do; a flood -> >= 64 written
    # slots per server-step
    dict(B=64, S=4, kw={"arrival_rate": 6.0, "server_rates": [3.0, 4.0, 5.0, 6.0]}),
    dict(B=48, S=8, kw={"arrival_rate": 3000.0, "warmup_steps": 1}),
    # S > 16 (server-per-lane only: 32 / 64 lanes per env): configs[4] read literally, 4 agents x
    # 16 servers = 64, and a 20-server env on a 32-lane group with two-choice SED
    dict(B=24, S=64, kw={"arrival_rate": 1600.0}),
    dict(B=40, S=20, kw={"assign_policy": "sed2", "arrival_rate": 800.0, "normalize_obs": True}),
    # overloaded servers with long queues: reservoirs fill (>= 128 samples) while flows start to
    # wait > 33 s -- full 4-server chunks holding a sample >= 2^25 - 1 us (observe's general path
    # with the two-pass sort, after steps on its register-resident path)
    dict(B=32, S=4, kw={"arrival_rate": 12.0, "server_rates": [1.2, 1.4, 1.6, 1.8],
                        "step_interval": 10.0, "queue_capacity": 64}),
    # above the small-batch threshold (B > 8192, S <= 4): the 4-lane groups of the headline shape
    dict(B=8256, S=4, kw={}),
    # one wave per env (lbsim_dyn_wave.h, S <= 4, Q <= 32): overloaded servers whose rings fill
    # (full-ring pushes keep the last completion, drops) with one ring register (Q <= 16) and
    # two (Q = 32), LSQ / LSQ2 on small envs, NaN SED scores on 4 servers
    dict(B=72, S=3, kw={"assign_policy": "lsq", "queue_capacity": 6, "load": 1.3}),
    dict(B=40, S=2, kw={"assign_policy": "lsq2", "server_rates": [100.0, 150.0]}),
    dict(B=36, S=4, kw={"load": 1.25, "discrete_weights": [0.5, 1.0, 8.0]}),
    dict(B=30, S=4, kw={"queue_capacity": 16, "load": 1.4, "action_type": "continuous"}),
    dict(B=60, S=4, kw={"action_type": "continuous", "_nan_actions": 0.2}),
    # lost-FIN flows (src/vpp/lb/lbhash.h:175-217): VPP's timed-out fct guess, recorded when the
    # bucket's next flow wraps the flow up (completion + flow_timeout + wait) -- with the default
    # 40 s timeout every guess is still pending at the end; 0.6 s and 0.3 s timeouts (2-3 steps
    # of 0.25 s) flush them into the fct reservoir as negative samples (fct - 39.4 s + wait:
    # observe's signed two-pass sort), every flow lost on a 3-server LSQ env; a 4-entry pending
    # ring that overflows
    dict(B=90, S=4, kw={"lost_fin_prob": 0.3}),
    dict(B=64, S=8, kw={"lost_fin_prob": 0.25, "flow_timeout": 0.6, "flow_buckets": 64,
                        "assign_policy": "sed2"}),
    dict(B=50, S=3, kw={"lost_fin_prob": 1.0, "flow_timeout": 0.3, "assign_policy": "lsq",
                        "action_type": "continuous", "flow_buckets": 64}),
    dict(B=40, S=4, kw={"lost_fin_prob": 0.8, "flow_timeout": 1.5, "flow_buckets": 32,
                        "lost_fin_pending": 4}),
    # server failure / recovery (THEORY.md §6.4): queues and reservoirs lost, down servers never
    # chosen (every policy), their all-zero rows inactive in the reward (env.py:410-413)
    dict(B=100, S=4, kw={"fail_prob": 0.15, "recover_prob": 0.3}),
    dict(B=72, S=6, kw={"fail_prob": 0.1, "recover_prob": 0.2, "assign_policy": "alias",
                        "action_type": "continuous"}),
    dict(B=64, S=5, kw={"fail_prob": 0.2, "recover_prob": 0.25, "assign_policy": "lsq2",
                        "normalize_obs": True, "reward_metric": "gini"}),
    dict(B=40, S=20, kw={"fail_prob": 0.05, "recover_prob": 0.5, "assign_policy": "sed2",
                         "lost_fin_prob": 0.2}),
    dict(B=48, S=8, kw={"fail_prob": 0.3, "recover_prob": 0.1, "lost_fin_prob": 0.1,
                        "trace": "short", "load": 1.2}),
    # next-step auto-reset (gymnasium NEXT_STEP): envs done last step reset inside the step
    # launches (warm-up included, action ignored, reward 0) -- short episodes cross several
    # boundaries; one-wave-per-env and group dispatch, S > 16 (two-launch observe), failures
    dict(B=70, S=4, kw={"max_steps": 3, "next_step_reset": True}),
    dict(B=40, S=6, kw={"max_steps": 4, "next_step_reset": True, "assign_policy": "sed2",
                        "normalize_obs": True}),
    dict(B=30, S=20, kw={"max_steps": 2, "next_step_reset": True, "fail_prob": 0.1,
                         "lost_fin_prob": 0.2}),
    dict(B=8256, S=4, kw={"max_steps": 5, "next_step_reset": True}),
    # duration_mode="service" (the service-time duration sample; the default is the flow's age,
    # lbhash.h:129-136): one-wave-per-env (full rings), server-per-lane groups (S = 20, B > the
    # small-batch limit), lost-FIN guesses beside it
    dict(B=64, S=3, kw={"duration_mode": "service", "queue_capacity": 6, "load": 1.3}),
    dict(B=40, S=20, kw={"duration_mode": "service", "assign_policy": "sed2",
                         "arrival_rate": 800.0}),
    dict(B=48, S=8, kw={"duration_mode": "service", "lost_fin_prob": 0.2, "flow_timeout": 0.4,
                        "flow_buckets": 64}),
    dict(B=8256, S=4, kw={"duration_mode": "service", "load": 1.1}),
    # paired observe of wide envs (S = 16: two waves per env, observe_pair16_kernel; S = 32:
    # one wave per 8-row group + the rows kernel): next-step auto-reset with normalisation,
    # sparse arrivals (unchanged groups keep cached features, rows with n < 8 take the chunk
    # fallback), waits > 33 s (the fallback's two-pass sort)
    dict(B=50, S=16, kw={"max_steps": 3, "next_step_reset": True, "normalize_obs": True}),
    dict(B=40, S=16, kw={"arrival_rate": 12.0, "server_rates": [1.0, 1.2] * 8,
                         "assign_policy": "sed2"}),
    dict(B=32, S=16, kw={"server_rates": [1.0, 1.5, 2.0, 2.5] * 4, "arrival_rate": 20.0,
                         "step_interval": 5.0, "queue_capacity": 64}),
    dict(B=24, S=32, kw={"max_steps": 2, "next_step_reset": True, "arrival_rate": 900.0}),
    # n_flow_on_mode "vpp" (column 0 never drops a lost-FIN flow, lbhash.h:193,214): with
    # failures (counts cleared), on 3 servers, on 20 servers, and the headline group shape
    dict(B=64, S=4, kw={"n_flow_on_mode": "vpp", "lost_fin_prob": 0.3, "fail_prob": 0.1}),
    dict(B=50, S=3, kw={"n_flow_on_mode": "vpp", "lost_fin_prob": 0.5, "flow_timeout": 10.0,
                        "assign_policy": "lsq"}),
    dict(B=40, S=20, kw={"n_flow_on_mode": "vpp", "lost_fin_prob": 0.2, "assign_policy": "sed2"}),
    dict(B=8256, S=4, kw={"n_flow_on_mode": "vpp", "lost_fin_prob": 0.2, "max_steps": 5,
                          "next_step_reset": True}),
    # ... whose SED / LSQ scores read the leaky count (node.c:395-437): every flow
    # lost on two-choice LSQ, and SED with unequal weights
    dict(B=48, S=8, kw={"n_flow_on_mode": "vpp", "lost_fin_prob": 1.0, "assign_policy": "lsq2",
                        "action_type": "continuous"}),
    dict(B=66, S=5, kw={"n_flow_on_mode": "vpp", "lost_fin_prob": 0.6,
                        "discrete_weights": [0.5, 1.0, 3.0]}),
    # reservoir_mode "vpp" (lbhash.h:108,179: every sample to slot rand() % 128 of a zeroed
    # reservoir): the headline group shape with next-step resets, lost-FIN deferral with failures,
    # ALIAS on 16 servers, sparse arrivals (bins that stay zero), service durations
    dict(B=64, S=4, kw={"reservoir_mode": "vpp"}),
    dict(B=8256, S=4, kw={"reservoir_mode": "vpp", "max_steps": 5, "next_step_reset": True}),
    dict(B=40, S=6, kw={"reservoir_mode": "vpp", "lost_fin_prob": 0.3, "flow_timeout": 0.5,
                        "flow_buckets": 32, "fail_prob": 0.1, "recover_prob": 0.3}),
    dict(B=48, S=16, kw={"reservoir_mode": "vpp", "assign_policy": "alias",
                         "action_type": "continuous"}),
    dict(B=64, S=4, kw={"reservoir_mode": "vpp", "arrival_rate": 6.0,
                        "server_rates": [3.0, 4.0, 5.0, 6.0], "duration_mode": "service"}),
]


def resolve_kw(kw):
    """CONFIGS entries name traces; build them here (module import stays cheap).  Keys starting
    with '_' are test options, not config kwargs."""
    from marllb_amd import trace
    kw = {k: v for k, v in kw.items() if not k.startswith("_")}
    if kw.get("trace") == "builtin":
        kw["trace"] = trace.builtin()
    elif kw.get("trace") == "short":
        kw["trace"] = trace.synthetic(37, 300.0, seed=7)
    return kw


def _actions(rng, B, S, cfgkw):
    if cfgkw.get("action_type") == "continuous":
        a = rng.uniform(-1.0, 11.0, (B, S)).astype(np.float32)
        a[rng.random((B, S)) < cfgkw.get("_nan_actions", 0.0)] = np.nan
        return a
    n = len(cfgkw.get("discrete_weights", [1, 1.5, 2]))
    return rng.integers(-n, n, (B, S)).astype(np.int64)


def _compare_state(h_gpu, ora, B, S, Q, norm, fail=False, leak=False, split_P=0):
    g = statelayout.parse(h_gpu.state_bytes(), B, S, Q, norm, fail, leak, split_P=split_P)
    o = statelayout.parse(ora.state_bytes(), B, S, Q, norm, fail, leak, split_P=split_P)
    for name in g:
        if name in ("ring", "pend"):
            continue
        np.testing.assert_array_equal(g[name], o[name], err_msg=name)
    np.testing.assert_array_equal(statelayout.live_ring(g, B, S, Q), statelayout.live_ring(o, B, S, Q))
    if split_P:  # the pending lost-FIN guesses in their rings
        np.testing.assert_array_equal(statelayout.live_pend(g, B, S, split_P),
                                      statelayout.live_pend(o, B, S, split_P))


def _run_vs_oracle(oracle_mod, B, S, kw, akw, case, mapping="auto", steps=12, post_steps=4,
                   threads=4, autoreset=False):
    """Step a VecLoadBalanceEnv and the oracle side by side from the same seeds: observations,
    rewards, done and per-server assignment counts every step, the full device state word for word
    after `steps` steps and again after a masked reset of every third env and `post_steps` more
    steps.  Returns the env (open) for further checks."""
    from marllb_amd.env import VecLoadBalanceEnv, make_config
    env = VecLoadBalanceEnv(B, S, device="cuda:0", autoreset=autoreset, dyn_mapping=mapping, **kw)
    ora = oracle_mod.OracleEnv(make_config(B, S, **kw), threads=threads, trace=kw.get("trace"))
    Q, norm, fail = env.cfg.queue_capacity, bool(env.cfg.normalize_obs), env.cfg.fail_prob > 0
    leak = statelayout.has_leak(env.cfg)
    sp = statelayout.split_p(env.cfg)
    obs_g = env.reset().cpu().numpy()
    obs_o = ora.reset()
    np.testing.assert_array_equal(obs_g, obs_o)
    rng = np.random.default_rng(case)
    for k in range(steps):
        a = _actions(rng, B, S, akw)
        og, rg, dg, info = env.step(torch.from_numpy(a), assign_counts=True)
        oo, ro, do, ao = ora.step(a)
        np.testing.assert_array_equal(info["assign_counts"].cpu().numpy(), ao, err_msg=f"assign step {k}")
        np.testing.assert_array_equal(og.cpu().numpy(), oo, err_msg=f"obs step {k}")
        np.testing.assert_array_equal(rg.cpu().numpy(), ro, err_msg=f"reward step {k}")
        np.testing.assert_array_equal(dg.cpu().numpy().astype(np.uint8), do)
    _compare_state(env.handle, ora, B, S, Q, norm, fail, leak, sp)
    # masked reset of every third env, then more steps
    mask = (np.arange(B) % 3 == 0).astype(np.uint8)
    og = env.reset(mask=torch.from_numpy(mask)).cpu().numpy()
    oo = ora.reset(mask=mask, obs=og.copy())
    np.testing.assert_array_equal(og, oo)
    for k in range(post_steps):
        a = _actions(rng, B, S, akw)
        og, rg, dg, _ = env.step(torch.from_numpy(a))
        oo, ro, do, _ = ora.step(a)
        np.testing.assert_array_equal(og.cpu().numpy(), oo)
        np.testing.assert_array_equal(rg.cpu().numpy(), ro)
    _compare_state(env.handle, ora, B, S, Q, norm, fail, leak, sp)
    ora.close()
    return env


@pytest.mark.parametrize("mapping", ["env", "server", "server-fused"])
@pytest.mark.parametrize("case", range(len(CONFIGS)))
def test_simulator_bit_exact_vs_oracle(lib, oracle_mod, case, mapping):
    """Both dynamics mappings (one lane per env / one lane per server) against the oracle; the
    server mapping both as two launches (the default) and as the fused step kernel (S <= 16)."""
    from marllb_amd.env import VecLoadBalanceEnv
    c = CONFIGS[case]
    B, S, kw = c["B"], c["S"], resolve_kw(c["kw"])
    if mapping == "server-fused":
        mapping, kw["step_kernel"] = "server", "fused"
    if mapping == "env" and S > 16:
        with pytest.raises(ValueError, match="at most 16 servers"):
            VecLoadBalanceEnv(B, S, device="cuda:0", dyn_mapping=mapping, **kw)
        return
    kw.setdefault("seed", 1000 + case)
    env = _run_vs_oracle(oracle_mod, B, S, kw, dict(c["kw"]), case, mapping)
    env.close()


def _simds():
    return 4 * torch.cuda.get_device_properties(0).multi_processor_count


def _expected_step_kernels(B, S, simds):
    """The default dispatch (lbsim_api.hip use_step_wave, lbsim_internal.h dyn_wave_ok /
    dyn_group_lanes, lbsim_step.hip launch_w) of a SED, Poisson, Q = 32 handle: {profile class:
    kernel-name prefix} of one step."""
    if B <= 4 * simds and S <= 8:  # one launch; S = 5-8: both chunks observed by the wave
        ng = 1 if S <= 2 else 2 if S <= 4 else 4
        occ = 2 if B <= 2 * simds else 4
        return {4: f"step_wave_kernel<{ng}, 0, false, {occ}, {4 if S <= 4 else 8}>"}
    g = 2 if S <= 2 else (8 if B * 4 // 64 <= simds // 2 else 4) if S <= 4 else 8 if S <= 8 else 16
    # paired records (duration = the flow's age, lost-FIN off), S <= 8: 8 // S envs per wave;
    # S = 16: two waves per env
    obs = ("observe_pair_kernel<0, " if S <= 8 else "observe_pair16_kernel<0, " if S == 16
           else "observe_pair_chunks_kernel<0>" if S % 8 == 0 else "observe_kernel<")
    return {0: f"dynamics_group_kernel<{g}, 0, 0, false", 1: obs}


def test_configs1_default_dispatch_4096x4(lib, oracle_mod):
    """BASELINE configs[1] as it runs by default: VecLoadBalanceEnv(4096, 4) with no override
    (on 256 CUs the one-launch step_wave_kernel at 4 waves per SIMD), every env against the
    oracle step by step and the full device state word for word (env.py:215-286,
    reservoir.py:50-196)."""
    from marllb_amd import _lib
    B, S = 4096, 4
    kw = {"seed": 4096}
    env = _run_vs_oracle(oracle_mod, B, S, kw, {}, 77, threads=8)
    names = _lib.launch_names(env.handle)
    for cls, pfx in _expected_step_kernels(B, S, _simds()).items():
        assert names.get(cls, "").startswith(pfx), (names, pfx)
    env.close()


@pytest.mark.parametrize("S,where", [(4, "2s"), (4, "2s+1"), (4, "4s"), (4, "4s+1"),
                                     (8, "2s"), (8, "2s+1"), (8, "4s"), (8, "4s+1")])
def test_dispatch_boundaries_bit_exact(lib, oracle_mod, S, where):
    """Batches at the dispatch boundaries of the default step (in envs per SIMD of this device):
    S = 4 and S = 8 at 2 and 4 envs per SIMD (step_wave_kernel OCC 2 -> OCC 4 -> server-per-lane
    groups; S = 8: the two-chunk forms).  The kernel that ran is checked by
    name (lbsim_launch_names), the results against the oracle on every env."""
    from marllb_amd import _lib
    simds = _simds()
    k, plus = (2, 0) if where == "2s" else (2, 1) if where == "2s+1" else (4, 0) if where == "4s" else (4, 1)
    B = k * simds + plus
    kw = {"seed": 500 + B + S, "assign_policy": "sed"}
    env = _run_vs_oracle(oracle_mod, B, S, kw, {}, B + S, steps=6, post_steps=2, threads=8)
    names = _lib.launch_names(env.handle)
    for cls, pfx in _expected_step_kernels(B, S, simds).items():
        assert names.get(cls, "").startswith(pfx), (B, S, names, pfx)
    env.close()


@pytest.mark.parametrize("occ", ["2", "4"])
def test_step_wave_occupancy_forms_bit_exact(occ):
    """LBSIM_STEP_WAVE_OCC forces one occupancy form of the one-launch step_wave_kernel at every
    batch size, so each simulator case the default dispatch sends to it (S <= 8, Q <= 32, not
    ALIAS, B <= 4 envs per SIMD: SED2, LSQ, LSQ2, trace arrivals, continuous and NaN actions, full
    rings, normalisation off) runs on the OCC-4 form that serves 2-4 envs per SIMD -- BASELINE
    configs[1]'s 4096 x 4 -- and on the OCC-2 form, the two-chunk S = 5-8 forms included.  Child
    process (read once per process)."""
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    ks = [f"test_simulator_bit_exact_vs_oracle[{c}-{m}]" for c in range(len(CONFIGS))
          for m in ("server", "server-fused")
          if CONFIGS[c]["S"] <= 8 and CONFIGS[c]["B"] <= 4096
          and CONFIGS[c]["kw"].get("queue_capacity", 32) <= 32
          and CONFIGS[c]["kw"].get("assign_policy") != "alias"]
    assert len(ks) >= 20
    r = subprocess.run([sys.executable, "-m", "pytest", "-q", "-x", "-m", "gpu", "-p",
                        "no:cacheprovider"] +
                       [os.path.join(root, "tests", "test_gpu_parity.py") + "::" + k for k in ks],
                       cwd=root, env={**os.environ, "LBSIM_STEP_WAVE_OCC": occ},
                       capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]


@pytest.mark.parametrize("lanes,epw", [("4", ""), ("8", ""), ("16", ""), ("4", "13"), ("8", "3")])
def test_wider_groups_bit_exact(lanes, epw):
    """LBSIM_DYN_GROUP_LANES forces the server-per-lane group width (lanes past S hold no server and
    only draw arrivals ahead): the simulator cases with S <= lanes stay bit-exact vs the oracle.
    lanes = 4 runs the headline 65536 x 4 kernel (4-lane groups) on every S <= 4 case -- every
    policy, trace arrivals, NaN fallbacks -- which the default small-batch dispatch sends to 8-lane
    groups.  epw (LBSIM_DYN_EPW): fewer envs per wave than 64 / lanes (lanes of the groups past it
    idle), e.g. 13 4-lane envs per wave.  The settings are read once per process, so the cases run
    in a child process."""
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    ks = [f"test_simulator_bit_exact_vs_oracle[{c}-{m}]" for c in range(len(CONFIGS))
          for m in ("server", "server-fused") if CONFIGS[c]["S"] <= int(lanes)]
    r = subprocess.run([sys.executable, "-m", "pytest", "-q", "-x", "-m", "gpu", "-p",
                        "no:cacheprovider"] +
                       [os.path.join(root, "tests", "test_gpu_parity.py") + "::" + k for k in ks],
                       cwd=root, env={**os.environ, "LBSIM_DYN_GROUP_LANES": lanes,
                                      **({"LBSIM_DYN_EPW": epw} if epw else {})},
                       capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]


@pytest.mark.parametrize("step", ["auto", "fused"])
def test_wave_kernel_bit_exact(step):
    """LBSIM_DYN_WAVE=1 runs the one-wave-per-env dynamics (lbsim_dyn_wave.h) on every simulator
    case it applies to (S <= 8, queue capacity <= 32, every policy but ALIAS) at any batch size,
    the 8256-env case included: bit-exact vs the oracle.  step = auto: a dynamics_wave_kernel
    launch then an observe launch; fused (LBSIM_STEP_KERNEL=fused, opt-in): one step_wave_kernel
    launch (dynamics then observe per wave).  Resets use dynamics_wave_kernel in both.  The
    settings are read once per process, so the cases run in a child process."""
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    ks = [f"test_simulator_bit_exact_vs_oracle[{c}-{m}]" for c in range(len(CONFIGS))
          for m in ("server", "server-fused")
          if CONFIGS[c]["S"] <= 8 and CONFIGS[c]["kw"].get("queue_capacity", 32) <= 32
          and CONFIGS[c]["kw"].get("assign_policy") != "alias"]
    assert len(ks) >= 20
    r = subprocess.run([sys.executable, "-m", "pytest", "-q", "-x", "-m", "gpu", "-p",
                        "no:cacheprovider"] +
                       [os.path.join(root, "tests", "test_gpu_parity.py") + "::" + k for k in ks],
                       cwd=root, env={**os.environ, "LBSIM_DYN_WAVE": "1",
                                      **({"LBSIM_STEP_KERNEL": "fused"} if step == "fused" else {})},
                       capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]


@pytest.mark.parametrize("S,world,B", [(4, 2, 200), (8, 4, 1003), (8, 8, 8400), (16, 8, 777)])
def test_sharding_invariance(lib, S, world, B):
    """Global env ids key the RNG: `world` uneven shards (each its own handle with its
    env_id_offset, as one rank per GPU runs them) reproduce the monolithic run exactly (SURVEY
    §8e), whatever kernel each shard's size dispatches to (8400 x 8 whole: server-per-lane groups;
    its ~1k-env shards: one wave per env) -- observations, rewards, done and assignment counts."""
    from marllb_amd.env import VecLoadBalanceEnv
    rng = np.random.default_rng(S * 100 + world)
    cuts = np.sort(rng.choice(np.arange(1, B), world - 1, replace=False))
    bounds = [0, *cuts.tolist(), B]
    full = VecLoadBalanceEnv(B, S, device="cuda:0", seed=9, autoreset=False)
    parts = [VecLoadBalanceEnv(hi - lo, S, device="cuda:0", seed=9, autoreset=False,
                               env_id_offset=lo) for lo, hi in zip(bounds[:-1], bounds[1:])]
    f = full.reset()
    p = torch.cat([e.reset() for e in parts])
    assert torch.equal(f, p)
    for _ in range(5):
        a = torch.from_numpy(rng.integers(0, 3, (B, S)))
        fo, fr, fd, fi = full.step(a, assign_counts=True)
        po = [e.step(a[lo:hi], assign_counts=True) for e, lo, hi in zip(parts, bounds[:-1], bounds[1:])]
        assert torch.equal(fo, torch.cat([x[0] for x in po]))
        assert torch.equal(fr, torch.cat([x[1] for x in po]))
        assert torch.equal(fd, torch.cat([x[2] for x in po]))
        assert torch.equal(fi["assign_counts"], torch.cat([x[3]["assign_counts"] for x in po]))
    for e in [full, *parts]:
        e.close()


def test_sharding_invariance_qmix_shape(lib):
    """configs[4]'s env shape (4 agents x 4 servers, problem-05 facade) split over 8 uneven
    shards equals one handle: agent observations, rewards, done and the global state."""
    from marllb_amd.multi_agent import VecMultiAgentLoadBalanceEnv
    B, world = 1000, 8
    rng = np.random.default_rng(44)
    bounds = [0, *np.sort(rng.choice(np.arange(1, B), world - 1, replace=False)).tolist(), B]
    full = VecMultiAgentLoadBalanceEnv(B, 4, 4, device="cuda:0", seed=21, action_type="discrete")
    parts = [VecMultiAgentLoadBalanceEnv(hi - lo, 4, 4, device="cuda:0", seed=21,
                                         action_type="discrete", env_id_offset=lo)
             for lo, hi in zip(bounds[:-1], bounds[1:])]
    assert torch.equal(full.reset(), torch.cat([e.reset() for e in parts]))
    for _ in range(4):
        a = torch.from_numpy(rng.integers(0, 3, (B, 4)))
        fo, fr, fd, _ = full.step(a)
        po = [e.step(a[lo:hi]) for e, lo, hi in zip(parts, bounds[:-1], bounds[1:])]
        assert torch.equal(fo, torch.cat([x[0] for x in po]))
        assert torch.equal(fr, torch.cat([x[1] for x in po]))
        assert torch.equal(fd, torch.cat([x[2] for x in po]))
        assert torch.equal(full.get_state(), torch.cat([e.get_state() for e in parts]))
    for e in [full, *parts]:
        e.close()


def test_full_size_properties(lib, oracle_mod):
    """BASELINE configs[2] size (65536 envs x 8 servers): size-independent invariants, plus the
    oracle on a 512-env slice of the same global ids."""
    from marllb_amd.env import VecLoadBalanceEnv, make_config
    B, S = 65536, 8
    env = VecLoadBalanceEnv(B, S, device="cuda:0", seed=3, autoreset=False, arrival_rate=500.0)
    obs = env.reset()
    rng = np.random.default_rng(0)
    steps = 6
    acts = [rng.integers(0, 3, (B, S)) for _ in range(steps)]
    tot = torch.zeros(S, dtype=torch.int64, device="cuda:0")
    for a in acts:
        obs, rew, done, info = env.step(torch.from_numpy(a), assign_counts=True)
        tot += info["assign_counts"].sum(0)
        assert torch.isfinite(obs).all()
        assert (rew >= 1.0 / S - 1e-6).all() and (rew <= 1.0).all()  # Jain range
        assert not done.any()
    st = statelayout.parse(env.handle.state_bytes(), B, S, env.cfg.queue_capacity, False)
    # conservation: every arrival drawn (arr_idx counts arrivals since reset) is assigned or dropped
    expected_rate = 500.0 * 0.25
    per_step = tot.sum().item() / (B * steps)
    assert abs(per_step - expected_rate) < 0.5, per_step
    # oracle on a slice of the same global ids (sharding invariance makes this exact)
    off, n = 40000, 512
    ora = oracle_mod.OracleEnv(make_config(n, S, seed=3, env_id_offset=off, arrival_rate=500.0),
                               threads=8)
    ora.reset()
    for a in acts:
        oo, ro, _, _ = ora.step(np.ascontiguousarray(a[off:off + n]))
    np.testing.assert_array_equal(obs[off:off + n].cpu().numpy(), oo)
    np.testing.assert_array_equal(rew[off:off + n].cpu().numpy(), ro)
    assert st["dropped"].sum() == 0


@pytest.mark.parametrize("B", [512, 65536])
def test_default_reward_sees_the_policy(lib, oracle_mod, B):
    """problem-03's default reward, Jain over flow_duration_avg_decay (THEORY.md:616, env.py:79),
    with the duration sample as the flow's age (lbhash.h:129-136): weights
    [2, 1, 1, 1] lower the mean reward by >= 0.03 against all-1.0 weights (40 steps after 20) on
    the HIP path, at 512 x 4 bit-exact vs the oracle and at the headline 65536 x 4."""
    from marllb_amd.env import VecLoadBalanceEnv, make_config
    S = 4
    means = []
    for row in ([0, 0, 0, 0], [2, 0, 0, 0]):
        env = VecLoadBalanceEnv(B, S, device="cuda:0", seed=7, autoreset=False)
        ora = None
        if B <= 512:
            ora = oracle_mod.OracleEnv(make_config(B, S, seed=7), threads=8)
            ora.reset()
        env.reset()
        a = torch.tensor(row, dtype=torch.int64).repeat(B, 1)
        acc = []
        for k in range(60):
            _, rew, _, _ = env.step(a)
            if ora is not None:
                _, ro, _, _ = ora.step(a.numpy())
                np.testing.assert_array_equal(rew.cpu().numpy(), ro)
            if k >= 20:
                acc.append(rew.double().mean().item())
        means.append(float(np.mean(acc)))
        env.close()
        if ora is not None:
            ora.close()
    assert means[0] - means[1] >= 0.03, means


def test_grid_above_four_waves_per_simd_s4(lib, oracle_mod):
    """A 4-lane step grid of more than 4 waves per SIMD (B > 65536 at S = 4 on 256 CUs) runs the
    5-wave register budget of dynamics_group_kernel: an oracle slice of the same global ids stays
    bit-exact."""
    from marllb_amd.env import VecLoadBalanceEnv, make_config
    B, S, steps = 70000, 4, 3
    env = VecLoadBalanceEnv(B, S, device="cuda:0", seed=21, autoreset=False)
    env.reset()
    rng = np.random.default_rng(4)
    acts = [rng.integers(0, 3, (B, S)) for _ in range(steps)]
    for a in acts:
        obs, rew, done, _ = env.step(torch.from_numpy(a))
    off, n = 66000, 384  # the slice straddles the last 4-wave-per-SIMD boundary of the grid
    ora = oracle_mod.OracleEnv(make_config(n, S, seed=21, env_id_offset=off), threads=8)
    ora.reset()
    for a in acts:
        oo, ro, _, _ = ora.step(np.ascontiguousarray(a[off:off + n]))
    np.testing.assert_array_equal(obs[off:off + n].cpu().numpy(), oo)
    np.testing.assert_array_equal(rew[off:off + n].cpu().numpy(), ro)


def test_full_size_trace_replay_c3(lib, oracle_mod):
    """BASELINE configs[2]: 65536 envs x 8 servers replaying data/trace poisson_for_loop
    rate_500 (the Wikipedia-trace stand-in).  Arrival conservation against the
    trace rows, and the oracle on a slice of the same global ids, bit-exact."""
    from marllb_amd import trace
    from marllb_amd.env import VecLoadBalanceEnv, make_config
    tr = trace.builtin()
    B, S, steps = 65536, 8, 4
    env = VecLoadBalanceEnv(B, S, device="cuda:0", seed=11, autoreset=False, trace=tr)
    env.reset()
    rng = np.random.default_rng(3)
    acts = [rng.integers(0, 3, (B, S)) for _ in range(steps)]
    tot = torch.zeros(B, dtype=torch.int64, device="cuda:0")
    for a in acts:
        obs, rew, done, info = env.step(torch.from_numpy(a), assign_counts=True)
        tot += info["assign_counts"].sum(1)
        assert torch.isfinite(obs).all() and not done.any()
    st = statelayout.parse(env.handle.state_bytes(), B, S, env.cfg.queue_capacity, False)
    # arrivals since reset = rows consumed from each env's offset (warm-up included)
    arrived = tot + torch.from_numpy(st["dropped"].astype(np.int64)).cuda()
    idx = torch.from_numpy(st["arr_idx"].astype(np.int64)).cuda()
    assert bool((arrived <= idx).all())
    off, n = 30000, 256
    ora = oracle_mod.OracleEnv(make_config(n, S, seed=11, env_id_offset=off, trace=tr),
                               threads=8, trace=tr)
    ora.reset()
    for a in acts:
        oo, ro, _, _ = ora.step(np.ascontiguousarray(a[off:off + n]))
    np.testing.assert_array_equal(obs[off:off + n].cpu().numpy(), oo)
    np.testing.assert_array_equal(rew[off:off + n].cpu().numpy(), ro)


def test_dynamics_kernel_dispatch(lib):
    """lbsim_dynamics_kernel names the kernel the launches use: one wave per env for small S <= 8
    batches (at most 4 envs per SIMD for S <= 4, 2 for S <= 8, queue capacity <= 32, not ALIAS),
    server-per-lane groups otherwise, one lane per env when asked for.  The batch limits are in
    envs per SIMD of this device (dyn_wave_ok's rule), not a 256-CU constant."""
    from marllb_amd.env import VecLoadBalanceEnv
    simds = _simds()
    cases = [(dict(num_envs=257, num_servers=4), 2), (dict(num_envs=1, num_servers=4), 2),
             (dict(num_envs=4 * simds + 1, num_servers=4), 1),
             (dict(num_envs=64, num_servers=8), 2),
             (dict(num_envs=4 * simds, num_servers=4), 2),
             (dict(num_envs=2 * simds, num_servers=8), 2),
             (dict(num_envs=2 * simds + 1, num_servers=8), 1),
             (dict(num_envs=64, num_servers=16), 1),
             (dict(num_envs=64, num_servers=4, assign_policy="alias"), 1),
             (dict(num_envs=64, num_servers=4, queue_capacity=64), 1),
             (dict(num_envs=64, num_servers=4, dyn_mapping="env"), 0)]
    for kw, want in cases:
        kw = dict(kw)
        B, S = kw.pop("num_envs"), kw.pop("num_servers")
        env = VecLoadBalanceEnv(B, S, device="cuda:0", **kw)
        assert env.handle.lib.lbsim_dynamics_kernel(env.handle.h) == want, (B, S, kw)
        env.close()
