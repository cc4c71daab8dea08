"""ctypes binding of the CPU oracle (oracle/liblbsim_oracle.so).  TEST INFRASTRUCTURE ONLY.

Imported only by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg, as the checker
or the timed CPU baseline.  The product (marllb_amd/) never imports this package.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "liblbsim_oracle.so")
K = 128
NF = 11

_P = ctypes.c_void_p
_lib = None


def build(quiet: bool = True) -> None:
    """Compile the oracle with its Makefile (gcc, -ffp-contract=off)."""
    subprocess.run(["make", "-C", HERE], check=True,
                   stdout=subprocess.DEVNULL if quiet else None)


def load() -> ctypes.CDLL:
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        build()
    lib = ctypes.CDLL(LIB_PATH)
    sig = {
        "oracle_philox": (None, [_P, _P, _P]),
        "oracle_logf": (ctypes.c_float, [ctypes.c_float]),
        "oracle_exp2f": (ctypes.c_float, [ctypes.c_float]),
        "oracle_decay_c": (ctypes.c_float, [ctypes.c_float]),
        "oracle_reward": (ctypes.c_double, [_P, ctypes.c_int, ctypes.c_int, ctypes.c_int]),
        "oracle_reward_batch": (None, [_P, ctypes.c_long, ctypes.c_int, ctypes.c_int,
                                       ctypes.c_int, _P]),
        "oracle_reward_batch64": (None, [_P, ctypes.c_long, ctypes.c_int, ctypes.c_int,
                                         ctypes.c_int, _P]),
        "oracle_features_batch": (None, [_P, _P, _P, ctypes.c_long, ctypes.c_float, _P]),
        "oracle_create": (_P, [_P]),
        "oracle_destroy": (None, [_P]),
        "oracle_set_threads": (None, [_P, ctypes.c_int]),
        "oracle_state_size": (ctypes.c_size_t, [_P]),
        "oracle_get_state": (None, [_P, _P]),
        "oracle_set_state": (None, [_P, _P]),
        "oracle_seed": (None, [_P, ctypes.c_uint64]),
        "oracle_reset": (ctypes.c_int, [_P, _P, _P]),
        "oracle_step": (ctypes.c_int, [_P, _P, ctypes.c_int, _P, _P, _P, _P]),
        "oracle_episode_stats": (None, [_P, _P, _P]),
        "oracle_normalize": (None, [_P, ctypes.c_int, _P, _P, _P, _P]),
        "oracle_set_trace": (ctypes.c_int, [_P, _P, _P, ctypes.c_long]),
        "oracle_gen_alias": (None, [_P, ctypes.c_int, _P, _P]),
        "oracle_vose_build": (None, [_P, ctypes.c_int, _P, _P]),
        "oracle_vose_sample": (ctypes.c_uint32, [_P, _P, ctypes.c_int, ctypes.c_uint32,
                                                 ctypes.c_int64, _P, _P]),
        "oracle_algr_slot": (ctypes.c_long, [ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32,
                                             ctypes.c_uint32, _P]),
        "oracle_algr_slot_r32": (ctypes.c_long, [ctypes.c_uint32, ctypes.c_uint32]),
        "oracle_vpp_features": (None, [_P, _P, ctypes.c_long, ctypes.c_long, ctypes.c_double,
                                       _P]),
    }
    for name, (res, args) in sig.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    _lib = lib
    return lib


def ptr(a: np.ndarray) -> int:
    assert a.flags["C_CONTIGUOUS"]
    return a.ctypes.data


def vpp_features(tv, ts, res_per_ts: int = 128, decay: float = 0.9) -> np.ndarray:
    """oracle_vpp_features: process_reservoir (src/lb/shm_proxy.py:518-543) of raw VPP reservoirs
    tv [n, 128, 2] (t, v) f32 at frame times ts [n / res_per_ts] f32 -> [n, 5] f64."""
    tv = np.ascontiguousarray(tv, np.float32).reshape(-1, 128, 2)
    ts = np.ascontiguousarray(np.atleast_1d(ts), np.float32)
    out = np.zeros((len(tv), 5), np.float64)
    load().oracle_vpp_features(ptr(tv), ptr(ts), res_per_ts, len(tv), decay, ptr(out))
    return out


def gen_alias(weights):
    """oracle_gen_alias: (odd float64[n], alias int32[n]) of gen_alias (shm_proxy.py:127-146)."""
    w = np.ascontiguousarray(weights, np.float32)
    odd = np.zeros(len(w), np.float64)
    alias = np.zeros(len(w), np.int32)
    load().oracle_gen_alias(ptr(w), len(w), ptr(odd), ptr(alias))
    return odd, alias


def vose_build(weights):
    """oracle_vose_build: (prob float32[n], alias uint32[n]) of problem-07's alias_table_build
    (vpp-plugin/alias_table.h:82-158)."""
    w = np.ascontiguousarray(weights, np.float32)
    prob = np.zeros(len(w), np.float32)
    alias = np.zeros(len(w), np.uint32)
    load().oracle_vose_build(ptr(w), len(w), ptr(prob), ptr(alias))
    return prob, alias


def vose_sample(prob, alias, state, k):
    """oracle_vose_sample: k alias_table_sample picks (alias_table.h:163-209) from xorshift32
    `state` -> (picks int32[k], histogram uint64[n], final state)."""
    p = np.ascontiguousarray(prob, np.float32)
    a = np.ascontiguousarray(alias, np.uint32)
    idx = np.zeros(k, np.int32)
    hist = np.zeros(len(p), np.uint64)
    st = load().oracle_vose_sample(ptr(p), ptr(a), len(p), int(state) & 0xFFFFFFFF, k,
                                   ptr(idx), ptr(hist))
    return idx, hist, st


def philox(ctr, key) -> np.ndarray:
    out = np.zeros(4, np.uint32)
    c = np.asarray(ctr, np.uint32)
    k = np.asarray(key, np.uint32)
    load().oracle_philox(ptr(c), ptr(k), ptr(out))
    return out


def features(values: np.ndarray, ts_ms: np.ndarray, counts: np.ndarray, decay=0.9) -> np.ndarray:
    values = np.ascontiguousarray(values, np.float32).reshape(-1, K)
    ts_ms = np.ascontiguousarray(ts_ms, np.uint32).reshape(-1, K)
    counts = np.ascontiguousarray(counts, np.uint32).reshape(-1)
    out = np.zeros((len(counts), 5), np.float32)
    load().oracle_features_batch(ptr(values), ptr(ts_ms), ptr(counts), len(counts), decay, ptr(out))
    return out


def rewards(obs: np.ndarray, metric: int, field: int, f64: bool = False) -> np.ndarray:
    obs = np.ascontiguousarray(obs, np.float32)
    n, S = obs.shape[0], obs.shape[1]
    if f64:
        out = np.zeros(n, np.float64)
        load().oracle_reward_batch64(ptr(obs), n, S, metric, field, ptr(out))
    else:
        out = np.zeros(n, np.float32)
        load().oracle_reward_batch(ptr(obs), n, S, metric, field, ptr(out))
    return out


class OracleEnv:
    """B envs of the CPU restatement with the same config struct and state layout as liblbsim."""

    def __init__(self, cfg, threads: int = 1, trace=None):
        self.lib = load()
        self.cfg = cfg
        self.B, self.S = cfg.num_envs, cfg.num_servers
        self.h = self.lib.oracle_create(ctypes.byref(cfg))
        if not self.h:
            raise MemoryError("oracle_create failed")
        self.lib.oracle_set_threads(self.h, threads)
        if trace is not None:
            self.set_trace(trace)

    def set_trace(self, trace):
        gap = np.ascontiguousarray(trace.gap_us, np.uint32)
        work = np.ascontiguousarray(trace.work, np.float32)
        assert self.lib.oracle_set_trace(self.h, ptr(gap), ptr(work), len(gap)) == 0

    def close(self):
        if self.h:
            self.lib.oracle_destroy(self.h)
            self.h = None

    def __del__(self):
        self.close()

    def set_threads(self, n: int):
        self.lib.oracle_set_threads(self.h, n)

    def seed(self, seed: int):
        self.lib.oracle_seed(self.h, seed)

    def reset(self, mask=None, obs=None) -> np.ndarray:
        if obs is None:
            obs = np.zeros((self.B, self.S, NF), np.float32)
        m = None if mask is None else np.ascontiguousarray(mask, np.uint8)
        rc = self.lib.oracle_reset(self.h, None if m is None else ptr(m), ptr(obs))
        assert rc == 0
        return obs

    def step(self, action: np.ndarray):
        a = np.ascontiguousarray(action)
        dt = {np.dtype(np.int32): 0, np.dtype(np.int64): 1, np.dtype(np.float32): 2}[a.dtype]
        obs = np.zeros((self.B, self.S, NF), np.float32)
        rew = np.zeros(self.B, np.float32)
        done = np.zeros(self.B, np.uint8)
        assign = np.zeros((self.B, self.S), np.int32)
        rc = self.lib.oracle_step(self.h, ptr(a), dt, ptr(obs), ptr(rew), ptr(done), ptr(assign))
        if rc != 0:
            raise ValueError("oracle_step before reset")
        return obs, rew, done, assign

    def episode_stats(self):
        ln = np.zeros(self.B, np.int32)
        rt = np.zeros(self.B, np.float64)
        self.lib.oracle_episode_stats(self.h, ptr(ln), ptr(rt))
        return ln, rt

    def state_bytes(self) -> bytes:
        n = self.lib.oracle_state_size(self.h)
        buf = ctypes.create_string_buffer(n)
        self.lib.oracle_get_state(self.h, buf)
        return buf.raw

    def load_state(self, data: bytes):
        assert len(data) == self.lib.oracle_state_size(self.h)
        self.lib.oracle_set_state(self.h, data)
