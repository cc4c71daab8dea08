"""LoadBalanceEnv.step's simulator path (`_step_sim`, round 6) against the reference's step
bookkeeping (env.py:255-286): the weights reported in `info` (env.py:334-353: discrete_weights[int(a)]
as the float32 values np.array holds, negative indices as Python's, IndexError before any step;
continuous np.clip in float32), `active_servers` (env.py:410-413: any feature > 0), `done`, the
episode return and the action handed to the simulator.  CPU only: the simulator call is replaced by
a stub returning fixed rows, so the host logic is what is tested (the GPU facade tests run the
whole step, tests/test_env_gpu.py).
"""
import numpy as np
import pytest

from marllb_amd import LoadBalanceEnv


def _env(action_type="discrete", **kw):
    env = LoadBalanceEnv(num_servers=4, action_type=action_type, max_steps=3, seed=1,
                         reference_plumbing=True, **kw)
    env.reset()
    # the simulator path with a stub simulator (white box: the plumbing mode's constructor is the
    # only GPU-free one)
    env._plumb = None
    env._dw32 = None
    env._active_lut = {}
    raw = np.zeros((4, 11), np.float32)
    raw[0, 1] = 0.5
    raw[2, 0] = 3.0
    raw[3, 5] = -1.0  # negative only: not active
    calls = []

    def sim(act):
        calls.append(act.copy())
        return raw * 2, raw.copy(), 0.25

    env._sim_step = sim
    return env, raw, calls


def test_discrete_weights_info_and_action():
    env, raw, calls = _env()
    obs, r, done, info = env.step(np.array([0, 1, 2, -1]))
    assert info["weights"] == [1.0, 1.5, 2.0, 2.0]
    assert all(type(w) is float for w in info["weights"])
    assert info["active_servers"] == [0, 2]
    assert info["step"] == 1 and info["episode_return"] == 0.25
    assert r == 0.25 and done is False
    assert calls[-1].dtype == np.int64 and calls[-1].tolist() == [0, 1, 2, -1]
    np.testing.assert_array_equal(obs, raw * 2)
    # float actions truncate like int(a) (env.py:346)
    _, _, _, info = env.step([1.7, 0.2, 2.9, 1.0])
    assert info["weights"] == [1.5, 1.0, 2.0, 1.5]
    assert calls[-1].tolist() == [1, 0, 2, 1]
    _, _, done, info = env.step([0, 0, 0, 0])
    assert done is True and info["episode"] == {"r": 0.75, "l": 3}


def test_discrete_weights_are_float32_values_and_follow_updates():
    env, _, _ = _env(discrete_weights=[0.1, 1.0, 3.3])
    _, _, _, info = env.step([0, 1, 2, 0])
    assert info["weights"] == [float(np.float32(0.1)), 1.0, float(np.float32(3.3)),
                               float(np.float32(0.1))]
    env.discrete_weights[1] = 7.0  # an in-place change is seen at the next step
    _, _, _, info = env.step([1, 1, 1, 1])
    assert info["weights"] == [7.0] * 4


def test_bad_index_raises_before_stepping():
    env, _, calls = _env()
    with pytest.raises(IndexError):
        env.step([0, 3, 0, 0])
    with pytest.raises(IndexError):
        env.step([0, -4, 0, 0])
    assert calls == []


def test_continuous_weights_clip_in_float32():
    env, _, calls = _env(action_type="continuous", min_weight=0.1, max_weight=10.0)
    _, _, _, info = env.step(np.array([0.05, 0.3, 12.0, 1.0], np.float64))
    assert info["weights"] == [float(np.float32(0.1)), float(np.float32(0.3)), 10.0, 1.0]
    assert calls[-1].dtype == np.float32
    np.testing.assert_array_equal(calls[-1], np.array([0.05, 0.3, 12.0, 1.0], np.float32))
