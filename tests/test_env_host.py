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
