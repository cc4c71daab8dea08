"""The C ABI (include/lbsim.h) without a GPU: liblbsim.so loads, exports every declared symbol,
reports its layout sizes, fills the reference defaults and validates configs with the reference's
error behaviour (ValueError for an unknown metric / action type, env.py:184, rewards.py:321)."""
import ctypes

import pytest

from marllb_amd import _lib


def test_library_loads_and_exports_every_header_symbol():
    lib = _lib.load()
    names = _lib.header_functions()
    assert len(names) >= 20
    missing = [n for n in names if not hasattr(lib, n)]
    assert missing == []


def test_version_and_layout_sizes():
    lib = _lib.load()
    assert lib.lbsim_version().startswith(b"lbsim")
    assert lib.lbsim_abi_version() == 10
    assert lib.lbsim_config_size() == ctypes.sizeof(_lib.LbsimConfig)
    assert lib.lbsim_step_outputs_size() == ctypes.sizeof(_lib.StepOutputs)


def test_defaults_mirror_reference_kwargs():
    c = _lib.default_config()  # env.py:71-87
    assert (c.num_servers, c.action_type, c.num_discrete) == (4, _lib.ACTION_DISCRETE, 3)
    assert list(c.discrete_weights)[:3] == [1.0, 1.5, 2.0]
    assert c.min_weight == pytest.approx(0.1) and c.max_weight == 10.0
    assert c.reward_metric == _lib.METRICS.index("jain") and c.reward_field == 10
    assert c.step_interval == 0.25 and c.max_steps == 10000 and c.normalize_obs == 0
    assert c.decay_factor == pytest.approx(0.9)


@pytest.mark.parametrize("field,value,msg", [
    ("reward_metric", 9, "Unsupported metric"),
    ("action_type", 2, "Unknown action_type"),
    ("num_servers", 65, "num_servers"),
    ("num_servers", 0, "num_servers"),
    ("queue_capacity", 65, "queue_capacity"),
    ("step_interval", 0.0, "step_interval"),
    ("arrival_rate", 0.0, "arrival_rate"),
    ("decay_factor", 1.0, "decay_factor"),
    ("reward_field", 11, "reward_field"),
])
def test_validate_rejects(field, value, msg):
    c = _lib.default_config()
    setattr(c, field, value)
    with pytest.raises(ValueError, match=msg):
        _lib.validate(c)


def test_create_without_device_fails_cleanly():
    torch = pytest.importorskip("torch")
    if torch.cuda.is_available():
        pytest.skip("a GPU is present")
    lib = _lib.load()
    c = _lib.default_config()
    h = ctypes.c_void_p()
    rc = lib.lbsim_create(ctypes.byref(c), 0, ctypes.byref(h))
    assert rc == _lib.EDEVICE and not h.value
    assert lib.lbsim_last_error(None)


def test_null_arguments_are_rejected():
    lib = _lib.load()
    assert lib.lbsim_reset(None, None, None, None) == _lib.EINVAL
    assert lib.lbsim_step(None, None, 0, None, None, None, None, None) == _lib.EINVAL
    assert lib.lbsim_reward(None, None, 0, None, None) == _lib.EINVAL
    assert lib.lbsim_destroy(None) == _lib.OK


def test_integration_ctypes_stub_matches_config_size():
    """The lbsim_config_t mirror shown to maintainers in INTEGRATION.md §2 has the library's size
    (the stub would otherwise hand the library a short struct)."""
    import ctypes
    import os
    import re
    from marllb_amd import _lib
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    txt = open(os.path.join(root, "INTEGRATION.md")).read()
    m = re.search(r"^class Cfg\(ctypes\.Structure\):.*?\]\n", txt, re.S | re.M)
    assert m, "INTEGRATION.md lost its lbsim_config_t stub"
    ns = {"ctypes": ctypes}
    exec(m.group(0), ns)
    assert ctypes.sizeof(ns["Cfg"]) == _lib.load().lbsim_config_size() == ctypes.sizeof(_lib.LbsimConfig)
