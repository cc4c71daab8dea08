"""ctypes binding of liblbsim.so (the C ABI declared in include/lbsim.h).

The library is built in-tree (marllb_amd/liblbsim.so, see marllb_amd/build.py).  There is no
fallback: if the shared object is missing or fails to load, every entry point raises.
"""
from __future__ import annotations

import ctypes
import os
import re

_HERE = os.path.dirname(os.path.abspath(__file__))
# LBSIM_LIBRARY: an alternative build of the same ABI (the A/B variants of
# `python -m marllb_amd.build --variant NAME -DMACRO`, marllb_amd/exp/liblbsim_NAME.so)
LIB_PATH = os.environ.get("LBSIM_LIBRARY") or os.path.join(_HERE, "liblbsim.so")
HEADER_PATH = os.path.join(os.path.dirname(_HERE), "include", "lbsim.h")

MAX_SERVERS = 64
RESERVOIR_K = 128
NUM_FEATURES = 11
MAX_DISCRETE = 8

OK, EINVAL, ENOMEM, EDEVICE, ESHAPE, ENOTSUP = 0, -1, -2, -3, -4, -5
ACTION_DISCRETE, ACTION_CONTINUOUS = 0, 1
ARRIVAL_POISSON, ARRIVAL_TRACE = 0, 1
DYN_MAPPINGS = ("auto", "env", "server")  # lbsim_dyn_mapping
STEP_KERNELS = ("auto", "split", "fused")  # lbsim_step_kernel
PROFILE_CLASSES = 5  # dynamics step, observe step, dynamics reset, observe reset, fused step
DTYPE_I32, DTYPE_I64, DTYPE_F32 = 0, 1, 2
METRICS = ["jain", "variance", "std", "cv", "max", "min", "product", "range", "gini"]
POLICIES = ["sed", "sed2", "lsq", "lsq2", "alias"]
DURATION_MODES = ("age", "service")  # lbsim_duration_mode
N_FLOW_ON_MODES = ("queue", "vpp")  # lbsim_n_flow_on_mode
RESERVOIR_MODES = ("algr", "vpp")  # lbsim_reservoir_mode


class LbsimConfig(ctypes.Structure):
    """Mirror of lbsim_config_t (include/lbsim.h)."""

    _fields_ = [
        ("num_envs", ctypes.c_int32),
        ("num_servers", ctypes.c_int32),
        ("env_id_offset", ctypes.c_int64),
        ("seed", ctypes.c_uint64),
        ("action_type", ctypes.c_int32),
        ("num_discrete", ctypes.c_int32),
        ("discrete_weights", ctypes.c_float * MAX_DISCRETE),
        ("min_weight", ctypes.c_float),
        ("max_weight", ctypes.c_float),
        ("reward_metric", ctypes.c_int32),
        ("reward_field", ctypes.c_int32),
        ("step_interval", ctypes.c_float),
        ("max_steps", ctypes.c_int32),
        ("normalize_obs", ctypes.c_int32),
        ("assign_policy", ctypes.c_int32),
        ("arrival_source", ctypes.c_int32),
        ("arrival_rate", ctypes.c_float),
        ("server_rate", ctypes.c_float * MAX_SERVERS),
        ("decay_factor", ctypes.c_float),
        ("queue_capacity", ctypes.c_int32),
        ("warmup_steps", ctypes.c_int32),
        ("dyn_mapping", ctypes.c_int32),
        ("step_kernel", ctypes.c_int32),
        ("lost_fin_prob", ctypes.c_float),
        ("flow_timeout_s", ctypes.c_float),
        ("flow_buckets", ctypes.c_int32),
        ("fail_prob", ctypes.c_float),
        ("recover_prob", ctypes.c_float),
        ("next_step_reset", ctypes.c_int32),
        ("duration_mode", ctypes.c_int32),
        ("n_flow_on_mode", ctypes.c_int32),
        ("lost_fin_pending", ctypes.c_int32),
        ("reservoir_mode", ctypes.c_int32),
    ]


class StepOutputs(ctypes.Structure):
    """Mirror of lbsim_step_outputs_t (include/lbsim.h); every field a device pointer or NULL."""

    _fields_ = [
        ("obs", ctypes.c_void_p),
        ("reward", ctypes.c_void_p),
        ("done", ctypes.c_void_p),
        ("assign_count", ctypes.c_void_p),
        ("raw_obs", ctypes.c_void_p),
        ("episode_length", ctypes.c_void_p),
        ("episode_return", ctypes.c_void_p),
        ("agent_obs", ctypes.c_void_p),
        ("state", ctypes.c_void_p),
        ("num_agents", ctypes.c_int32),
        ("servers_per_agent", ctypes.c_int32),
        ("done_word", ctypes.c_void_p),
        ("done_value", ctypes.c_uint32),
    ]


_SAC_WEIGHTS = ("w_ih", "w_hh", "b_ih", "b_hh", "w1", "b1", "wh", "bh")
_QMIX_WEIGHTS = ("w_ih", "w_hh", "b_ih", "b_hh", "w1", "b1", "w2", "b2", "w3", "b3",
                 "m0", "mb0", "mw1", "mbw1", "mw2", "mbw2", "mb2", "mbb2")


class SacActor(ctypes.Structure):
    """Mirror of lbsim_sac_actor_t (include/lbsim.h); weight fields are device pointers."""

    _fields_ = ([("state_dim", ctypes.c_int32), ("gru_dim", ctypes.c_int32),
                 ("hidden_dim", ctypes.c_int32), ("action_dim", ctypes.c_int32)]
                + [(n, ctypes.c_void_p) for n in _SAC_WEIGHTS]
                + [("log_std_min", ctypes.c_float), ("log_std_max", ctypes.c_float),
                   ("action_scale", ctypes.c_float), ("action_bias", ctypes.c_float),
                   ("step_dev", ctypes.c_void_p)])


class QmixPolicy(ctypes.Structure):
    """Mirror of lbsim_qmix_policy_t (include/lbsim.h); weight fields are device pointers."""

    _fields_ = ([(n, ctypes.c_int32) for n in ("num_agents", "obs_dim", "gru_dim", "hidden_dim",
                                               "n_actions", "state_dim", "mixing_embed_dim",
                                               "hypernet_embed_dim", "servers_per_agent")]
                + [("epsilon", ctypes.c_float)]
                + [(n, ctypes.c_void_p) for n in _QMIX_WEIGHTS]
                + [("step_dev", ctypes.c_void_p)])


class LbsimError(RuntimeError):
    """A liblbsim call returned a negative status."""

    def __init__(self, code: int, msg: str):
        super().__init__(f"liblbsim error {code}: {msg}")
        self.code = code


_P = ctypes.c_void_p
_SIGNATURES = {
    "lbsim_version": (ctypes.c_char_p, []),
    "lbsim_abi_version": (ctypes.c_int, []),
    "lbsim_config_default": (ctypes.c_int, [ctypes.POINTER(LbsimConfig)]),
    "lbsim_config_validate": (ctypes.c_int, [ctypes.POINTER(LbsimConfig), ctypes.c_char_p,
                                             ctypes.c_size_t]),
    "lbsim_create": (ctypes.c_int, [ctypes.POINTER(LbsimConfig), ctypes.c_int,
                                    ctypes.POINTER(_P)]),
    "lbsim_destroy": (ctypes.c_int, [_P]),
    "lbsim_last_error": (ctypes.c_char_p, [_P]),
    "lbsim_seed": (ctypes.c_int, [_P, ctypes.c_uint64]),
    "lbsim_dynamics_kernel": (ctypes.c_int, [_P]),
    "lbsim_reset": (ctypes.c_int, [_P, _P, _P, _P]),
    "lbsim_step": (ctypes.c_int, [_P, _P, ctypes.c_int, _P, _P, _P, _P, _P]),
    "lbsim_step_ex": (ctypes.c_int, [_P, _P, ctypes.c_int, ctypes.POINTER(StepOutputs), _P]),
    "lbsim_reset_ex": (ctypes.c_int, [_P, _P, ctypes.POINTER(StepOutputs), _P]),
    "lbsim_config_size": (ctypes.c_size_t, []),
    "lbsim_step_outputs_size": (ctypes.c_size_t, []),
    "lbsim_episode_stats": (ctypes.c_int, [_P, _P, _P, _P]),
    "lbsim_step_stats": (ctypes.c_int, [_P, _P]),
    "lbsim_reward": (ctypes.c_int, [ctypes.POINTER(LbsimConfig), _P, ctypes.c_int64, _P, _P]),
    "lbsim_gru_gates": (ctypes.c_int, [_P, _P, _P, _P, ctypes.c_int64, ctypes.c_int, _P]),
    "lbsim_sac_head": (ctypes.c_int, [_P, ctypes.c_int64, ctypes.c_int, ctypes.c_float,
                                      ctypes.c_float, ctypes.c_float, ctypes.c_float, ctypes.c_int,
                                      ctypes.c_uint64, ctypes.c_uint32, _P, _P, _P]),
    "lbsim_qmix_tail": (ctypes.c_int, [_P, _P, ctypes.c_int64, _P, ctypes.c_int64, _P,
                                       ctypes.c_int64, _P, ctypes.c_int64, ctypes.c_int64,
                                       ctypes.c_int, ctypes.c_int, _P, _P]),
    "lbsim_sac_actor_size": (ctypes.c_size_t, []),
    "lbsim_qmix_policy_size": (ctypes.c_size_t, []),
    "lbsim_sac_actor_step": (ctypes.c_int, [ctypes.POINTER(SacActor), _P, _P, _P, ctypes.c_int64,
                                            ctypes.c_int, ctypes.c_uint64, ctypes.c_uint32, _P,
                                            _P, _P]),
    "lbsim_qmix_policy_step": (ctypes.c_int, [ctypes.POINTER(QmixPolicy), _P, _P, _P, _P,
                                              ctypes.c_int64, ctypes.c_uint64, ctypes.c_uint32,
                                              _P, _P, _P, _P, _P, _P]),
    "lbsim_agent_obs": (ctypes.c_int, [_P, ctypes.c_int64, ctypes.c_int, ctypes.c_int,
                                       ctypes.c_int, _P, _P]),
    "lbsim_set_trace": (ctypes.c_int, [_P, _P, _P, ctypes.c_int64, _P]),
    "lbsim_alias_tables": (ctypes.c_int, [_P, ctypes.c_int64, ctypes.c_int, _P, _P, _P, _P]),
    "lbsim_vose_tables": (ctypes.c_int, [_P, ctypes.c_int64, ctypes.c_int, _P, _P, _P]),
    "lbsim_vose_sample": (ctypes.c_int, [_P, _P, ctypes.c_int64, ctypes.c_int, _P, ctypes.c_int64,
                                         _P, _P, _P]),
    "lbsim_reservoir_features": (ctypes.c_int, [_P, _P, _P, ctypes.c_int64, ctypes.c_float, _P,
                                                _P]),
    "lbsim_vpp_export": (ctypes.c_int, [_P, ctypes.c_int64, ctypes.c_int64, _P, _P, _P, _P]),
    "lbsim_vpp_features": (ctypes.c_int, [_P, _P, ctypes.c_int64, ctypes.c_int64, ctypes.c_double,
                                          _P, _P]),
    "lbsim_profile_begin": (ctypes.c_int, [_P, ctypes.c_int]),
    "lbsim_profile_end": (ctypes.c_int, [_P, _P, _P]),
    "lbsim_profile_end_ex": (ctypes.c_int, [_P, _P, _P, ctypes.c_int]),
    "lbsim_launch_names": (ctypes.c_int, [_P, ctypes.c_int, ctypes.c_char_p, ctypes.c_size_t]),
    "lbsim_state_size": (ctypes.c_int, [_P, ctypes.POINTER(ctypes.c_size_t)]),
    "lbsim_get_state": (ctypes.c_int, [_P, _P, ctypes.c_size_t]),
    "lbsim_set_state": (ctypes.c_int, [_P, _P, ctypes.c_size_t]),
}

_lib = None


def header_functions(path: str = HEADER_PATH) -> list[str]:
    """Names of every function declared in include/lbsim.h."""
    txt = open(path).read()
    return sorted(set(re.findall(r"^\s*(?:const\s+)?\w+\*?\s+\*?(lbsim_\w+)\s*\(", txt, re.M)))


def load() -> ctypes.CDLL:
    """Load liblbsim.so once.  Raises if the HIP library was not built (no CPU fallback)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise RuntimeError(
            f"{LIB_PATH} not found: build it with `python -m marllb_amd.build` "
            "(hipcc --offload-arch=gfx950); there is no CPU fallback")
    try:  # share torch's HIP runtime when torch is present (same SONAME, one instance)
        import torch  # noqa: F401
    except ImportError:
        pass
    lib = ctypes.CDLL(LIB_PATH)
    for name, (res, args) in _SIGNATURES.items():
        if os.environ.get("LBSIM_LIBRARY") and not hasattr(lib, name):
            continue  # an A/B build of an older ABI: only the entry points it has
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    _lib = lib
    return lib


class TimingEvent:
    """A HIP timing event created with hipEventDisableSystemFence, for bench.py's per-launch times
    of the policy kernels (lbsim_profile_begin's events are made the same way): a default event's
    record writes back and invalidates the caches between the launches it brackets.  Resolved
    through liblbsim.so's own HIP runtime (the one torch shares).  Read elapsed_time only after the
    device is synchronised."""

    _DISABLE_SYSTEM_FENCE = 0x20000000

    def __init__(self):
        self._lib = load()
        self.ev = ctypes.c_void_p()
        if self._lib.hipEventCreateWithFlags(ctypes.byref(self.ev),
                                             ctypes.c_uint(self._DISABLE_SYSTEM_FENCE)) != 0:
            raise RuntimeError("hipEventCreateWithFlags failed")

    def record(self, stream: int = 0) -> None:
        if self._lib.hipEventRecord(self.ev, ctypes.c_void_p(stream or None)) != 0:
            raise RuntimeError("hipEventRecord failed")

    def elapsed_time(self, end: "TimingEvent") -> float:
        ms = ctypes.c_float()
        if self._lib.hipEventElapsedTime(ctypes.byref(ms), self.ev, end.ev) != 0:
            raise RuntimeError("hipEventElapsedTime failed (events not complete?)")
        return ms.value

    def __del__(self):
        if getattr(self, "ev", None) and self.ev.value:
            self._lib.hipEventDestroy(self.ev)


def launch_names(handle, which: int = 0) -> dict:
    """{profile class: kernel signature} of the last step (which=0) / reset (1) of a Handle
    (lbsim_launch_names), e.g. {0: 'dynamics_group_kernel<4, 0, 0, false, 1>', 1: ...}."""
    buf = ctypes.create_string_buffer(4096)
    check(load().lbsim_launch_names(handle.h, which, buf, len(buf)), handle.h)
    out = {}
    for item in buf.value.decode().split(";"):
        if item:
            cls, name = item.split("=", 1)
            out[int(cls)] = name
    return out


def default_config() -> LbsimConfig:
    cfg = LbsimConfig()
    check(load().lbsim_config_default(ctypes.byref(cfg)))
    return cfg


def validate(cfg: LbsimConfig) -> None:
    buf = ctypes.create_string_buffer(256)
    if load().lbsim_config_validate(ctypes.byref(cfg), buf, 256) != OK:
        raise ValueError(buf.value.decode())


def check(rc: int, handle=None) -> None:
    """Raise on a negative status: ValueError for EINVAL (as the reference does), else LbsimError."""
    if rc != OK:
        msg = load().lbsim_last_error(handle).decode()
        if rc == EINVAL:
            raise ValueError(msg or "invalid argument")
        raise LbsimError(rc, msg)
