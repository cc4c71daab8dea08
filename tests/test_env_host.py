"""Host-side plumbing of the facades against the reference's own outputs (env_plumbing.json):
spaces (env.py:156-184), _action_to_weights (334-353), _array_to_dict (391-423), config errors."""
import json
import os

import numpy as np
import pytest

from marllb_amd import env as E


@pytest.fixture(scope="module")
def plumb(golden_dir):
    return json.load(open(os.path.join(golden_dir, "env_plumbing.json")))


def test_feature_names(plumb):
    assert E.FEATURE_NAMES == plumb["feature_names"]


def test_spaces(plumb):
    for sp in plumb["spaces"]:
        obs, act = E.make_spaces(sp["S"], sp["action_type"], [1.0, 1.5, 2.0], 0.1, 10.0,
                                 sp["use_ground_truth"])
        assert list(obs.shape) == sp["obs_shape"]
        assert float(obs.low.min()) == sp["obs_low"] and float(obs.high.max()) == sp["obs_high"]
        if sp["action_type"] == "discrete":
            assert act.nvec.tolist() == sp["nvec"]
            s = act.sample()
            assert s.shape == (sp["S"],) and (s >= 0).all() and (s < 3).all()
        else:
            assert list(act.shape) == sp["act_shape"]
            assert float(act.low.min()) == pytest.approx(sp["act_low"])
            assert float(act.high.max()) == pytest.approx(sp["act_high"])
            s = act.sample()
            assert act.contains(s)


def test_action_to_weights(plumb):
    for case in plumb["action_to_weights"]:
        kw = case["kwargs"]
        w = E.action_to_weights(np.array(case["action"]), kw["action_type"],
                                kw.get("discrete_weights", [1.0, 1.5, 2.0]),
                                kw.get("min_weight", 0.1), kw.get("max_weight", 10.0))
        assert w.dtype == np.float32 and str(w.dtype) == case["dtype"]
        assert w.tolist() == case["weights"]


def test_array_to_dict_active_rule(plumb):
    for case in plumb["array_to_dict"]:
        d = E.array_to_dict(np.array(case["obs"], np.float32))
        assert d["active_servers"] == case["active"]
    obs = np.arange(44, dtype=np.float32).reshape(4, 11) + 1
    back = E.dict_to_array(E.array_to_dict(obs), 4)
    np.testing.assert_array_equal(back, obs)


def test_make_config_errors():
    with pytest.raises(ValueError, match="Unsupported metric"):
        E.make_config(4, reward_metric="fairness")
    with pytest.raises(ValueError, match="Unknown action_type"):
        E.make_config(4, action_type="hybrid")
    with pytest.raises(ValueError, match="server_rates"):
        E.make_config(4, 4, server_rates=[1.0, 2.0])
    c = E.make_config(8, 4, reward_field="no_such_field", seed=5)
    assert c.reward_field == -1 and c.seed == 5
    c = E.make_config(8, 4, arrival_rate=400.0, load=0.8)
    assert list(c.server_rate)[:4] == [125.0] * 4


def test_optional_dynamics_config():
    """The round-4 config fields (include/lbsim.h): defaults (VPP's 40 s flow timeout and 1024
    sticky buckets, lb.c:1437 / lb.h:46; failures and lost-FIN off; same-step auto-reset), their
    validation, and the facade's autoreset_mode."""
    c = E.make_config(8, 4)
    assert c.lost_fin_prob == 0.0 and c.flow_timeout_s == 40.0 and c.flow_buckets == 1024
    assert c.fail_prob == 0.0 and c.recover_prob == pytest.approx(0.1) and c.next_step_reset == 0
    c = E.make_config(8, 4, lost_fin_prob=0.5, flow_timeout=10.0, flow_buckets=64, fail_prob=0.2,
                      recover_prob=0.3, next_step_reset=True)
    assert (c.lost_fin_prob, c.flow_timeout_s, c.flow_buckets) == (0.5, 10.0, 64)
    assert c.fail_prob == pytest.approx(0.2) and c.next_step_reset == 1
    for kw, msg in [({"lost_fin_prob": 1.5}, "lost_fin_prob"),
                    ({"lost_fin_prob": 0.1, "flow_timeout": -1.0}, "flow_timeout_s"),
                    ({"lost_fin_prob": 0.1, "flow_buckets": 0}, "flow_buckets"),
                    ({"lost_fin_prob": 0.1, "flow_buckets": 10 ** 6}, "flow_buckets"),
                    ({"fail_prob": -0.1}, "fail_prob"),
                    ({"recover_prob": 2.0}, "recover_prob"),
                    # a nonzero probability below the 24-bit threshold's resolution
                    ({"fail_prob": 1e-9}, "fail_prob"),
                    ({"lost_fin_prob": 1e-9}, "lost_fin_prob"),
                    # the guessed fct and its wrap-up delay must fit signed 32-bit us (ADVICE
                    # r04); the message states the limit for the given timeout
                    ({"lost_fin_prob": 0.1, "flow_timeout": 3600.0}, "flow_timeout_s must be < 1040"),
                    ({"lost_fin_prob": 0.1, "flow_timeout": 600.0, "flow_buckets": 40000},
                     r"signed 32-bit.*must be <= 26\.347 s \(got 100\.000\)"),
                    ({"lost_fin_prob": 0.1, "lost_fin_pending": 0}, "lost_fin_pending"),
                    ({"lost_fin_prob": 0.1, "lost_fin_pending": 5000}, "lost_fin_pending"),
                    ({"reservoir_mode": "random"}, "reservoir_mode"),
                    ({"duration_mode": "wall"}, "duration_mode")]:
        with pytest.raises(ValueError, match=msg):
            E.make_config(8, 4, **kw)
    with pytest.raises(ValueError, match="autoreset_mode"):
        E.VecLoadBalanceEnv(8, 4, autoreset_mode="sometimes")


def test_duration_mode_config():
    """duration_mode (include/lbsim.h lbsim_duration_mode): the flow's age (lbhash.h:129-136) by
    default, the service time on request."""
    assert E.make_config(8, 4).duration_mode == 0
    assert E.make_config(8, 4, duration_mode="service").duration_mode == 1
