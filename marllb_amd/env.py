"""Gym-style facades over liblbsim.

VecLoadBalanceEnv   B independent LB environments resident on one GPU; torch tensors in/out,
                    no host synchronisation on the step path (the batched hot path).
LoadBalanceEnv      the reference's single-environment API, call for call
                    (simulation-mode/problem-03-rl-environment/src/env.py:41-470): numpy in/out,
                    same kwargs, spaces, info dict, done rule, seed/render/close and ValueErrors,
                    so problem-04's Trainer and problem-05's wrapper drop in unchanged.

Both run every step through the gfx950 kernels (marllb_amd/csrc).  What differs from the
reference by design: observations come from a real flow simulator (arrivals ->
server assignment -> FIFO service -> reservoir features) instead of np.random draws, and there is
no wall-clock sleep (step_interval is SIMULATED seconds).  The reference's own random-observation
simulation mode is available on the host as LoadBalanceEnv(reference_plumbing=True)
(BASELINE configs[0], marllb_amd/plumbing.py).
"""
from __future__ import annotations

import ctypes
import os
import time
from typing import Any, Dict, List, Optional, Tuple

import numpy as np

from . import _lib
from .spaces import Box, MultiDiscrete

# the single-env facade's step polls its completion word for at most this long before a stream
# synchronisation (a step that runs longer, or a device fault, then goes through the runtime)
_POLL_S = 0.05

NF = 11  # observation columns per server (env.py:46-48)

# env.py:377-381 — observation column order (column 10 is named flow_duration_avg_decay there)
FEATURE_NAMES = [
    "n_flow_on", "fct_mean", "fct_p90", "fct_std", "fct_mean_decay", "fct_p90_decay",
    "flow_duration_mean", "flow_duration_p90", "flow_duration_std",
    "flow_duration_mean_decay", "flow_duration_avg_decay",
]
DEFAULT_DISCRETE_WEIGHTS = [1.0, 1.5, 2.0]  # env.py:69


def action_to_weights(action, action_type: str, discrete_weights, min_weight: float,
                      max_weight: float) -> np.ndarray:
    """env.py:334-353: discrete index -> discrete_weights[int(a)]; continuous -> clip (f32)."""
    if action_type == "discrete":
        return np.array([discrete_weights[int(a)] for a in action], dtype=np.float32)
    return np.clip(np.asarray(action, dtype=np.float32), min_weight, max_weight)


def array_to_dict(obs: np.ndarray, sequence_id: int = 0) -> dict:
    """env.py:391-423: active = any(obs[s] > 0); per-server dict of the 11 named features."""
    active = np.flatnonzero((obs > 0).any(axis=1)).tolist()
    rows = obs.tolist()  # the float32 values as Python floats (= float(obs[sid, i]))
    stats = {sid: dict(zip(FEATURE_NAMES, rows[sid])) for sid in active}
    return {"active_servers": active, "server_stats": stats, "sequence_id": sequence_id}


def dict_to_array(obs_dict: dict, num_servers: int) -> np.ndarray:
    """env.py:355-389."""
    obs = np.zeros((num_servers, 11), dtype=np.float32)
    stats = obs_dict.get("server_stats", {})
    for sid in obs_dict.get("active_servers", []):
        if sid < num_servers and sid in stats:
            for i, name in enumerate(FEATURE_NAMES):
                obs[sid, i] = stats[sid].get(name, 0.0)
    return obs


def make_spaces(num_servers: int, action_type: str, discrete_weights, min_weight: float,
                max_weight: float, use_ground_truth: bool = False):
    """env.py:156-184 (observation space is (S, 11 [+3]) even though arrays are (S, 11))."""
    num_features = 11 + (3 if use_ground_truth else 0)
    obs_space = Box(low=0, high=np.inf, shape=(num_servers, num_features), dtype=np.float32)
    if action_type == "discrete":
        act_space = MultiDiscrete([len(discrete_weights)] * num_servers)
    elif action_type == "continuous":
        act_space = Box(low=min_weight, high=max_weight, shape=(num_servers,), dtype=np.float32)
    else:
        raise ValueError(f"Unknown action_type: {action_type}")
    return obs_space, act_space


def _torch():
    import torch
    return torch


def _device_index(device) -> int:
    torch = _torch()
    if device is None:
        return torch.cuda.current_device()
    d = torch.device(device)
    if d.type != "cuda":
        raise ValueError(f"lbsim runs on a HIP device (cuda:N), got {device!r}")
    return torch.cuda.current_device() if d.index is None else d.index


def make_config(num_envs: int, num_servers: int = 4, action_type: str = "discrete",
                discrete_weights: Optional[List[float]] = None, max_weight: float = 10.0,
                min_weight: float = 0.1, reward_metric: str = "jain",
                reward_field: str = "flow_duration_avg_decay", step_interval: float = 0.25,
                max_steps: int = 10000, normalize_obs: bool = False, seed: Optional[int] = None,
                env_id_offset: int = 0, arrival_rate: float = 400.0,
                server_rates: Optional[List[float]] = None, load: float = 0.8,
                queue_capacity: int = 32, warmup_steps: int = 8, decay_factor: float = 0.9,
                assign_policy: str = "sed", trace=None,
                dyn_mapping: str = "auto", step_kernel: str = "auto",
                lost_fin_prob: float = 0.0, flow_timeout: float = 40.0, flow_buckets: int = 1024,
                fail_prob: float = 0.0, recover_prob: float = 0.1,
                next_step_reset: bool = False,
                duration_mode: str = "age", n_flow_on_mode: str = "queue",
                lost_fin_pending: int = 256, reservoir_mode: str = "algr") -> _lib.LbsimConfig:
    """Build and validate an lbsim_config_t from reference-style kwargs.

    server_rates defaults to identical servers at utilisation `load`: mu = rate / (load * S).
    trace (marllb_amd.trace.Trace): replay its arrivals (LBSIM_ARRIVAL_TRACE); its empirical rate
    replaces arrival_rate.  The arrays themselves go to the handle (Handle.set_trace).
    dyn_mapping: "auto" | "env" (one lane per env) | "server" (one lane per server): how the
    dynamics kernel lays envs onto lanes; results are identical, only speed differs.
    step_kernel: "auto" | "split" (dynamics launch + observe launch) | "fused" (one launch that
    simulates then observes each workgroup's envs); results are identical.
    lost_fin_prob / flow_timeout / flow_buckets: flows whose FIN/RST the VPP data plane misses
    record its timed-out guess fct = now - t_init - 40 s (src/vpp/lb/lbhash.h:175-217) instead of
    their fct, at the wrap-up time (completion + flow_timeout + the wait for the next flow in the
    bucket, of mean flow_buckets / arrival_rate) and stamped with it.  0 = off.
    lost_fin_pending: the guesses each server holds until their wrap-up (a guess arriving at a
    full ring is dropped and counted, Handle.lost_fin_overflow).
    reservoir_mode: "algr" = problem-01's Algorithm R (reservoir.py:64-85); "vpp" = the data
    plane's rule, every sample overwrites slot rand() % 128 of a zeroed reservoir
    (lbhash.h:108,179), for feature_mode="upstream" / the VPP export.
    fail_prob / recover_prob: per server and step, an up server fails (its queue and reservoirs are
    lost) and a down one recovers (THEORY.md §6.4 server_failure ~ Bernoulli(p_fail)).  0 = off.
    next_step_reset: lbsim_step resets, in place of stepping, the envs whose last step returned
    done (gymnasium's NEXT_STEP autoreset; VecLoadBalanceEnv(autoreset_mode="next_step")).
    duration_mode: the flow-duration sample (obs columns 6-10, the default reward field): "age"
    = the flow's age at its last data packet, completion - arrival, backlog wait included
    (src/vpp/lb/lbhash.h:129-136 records time_now - t_init on every plain ACK after the first);
    "service" = the service time alone.
    n_flow_on_mode: observation column 0: "queue" = the flows in flight at the server; "vpp" =
    the data plane's n_flow_on, which never decrements a lost-FIN flow (lbhash.h:193,214): the
    flows in flight plus the server's lost-FIN flows since the episode start.
    """
    if reward_metric not in _lib.METRICS:  # rewards.py:321-323
        raise ValueError(f"Unsupported metric: {reward_metric}. Supported: {_lib.METRICS}")
    if action_type not in ("discrete", "continuous"):  # env.py:183-184
        raise ValueError(f"Unknown action_type: {action_type}")
    if assign_policy not in _lib.POLICIES:
        raise ValueError(f"Unknown assign_policy: {assign_policy}. Supported: {_lib.POLICIES}")
    cfg = _lib.default_config()
    cfg.num_envs = int(num_envs)
    cfg.num_servers = int(num_servers)
    cfg.env_id_offset = int(env_id_offset)
    if seed is None:
        seed = int.from_bytes(os.urandom(8), "little")
    cfg.seed = int(seed) & 0xFFFFFFFFFFFFFFFF
    cfg.action_type = _lib.ACTION_DISCRETE if action_type == "discrete" else _lib.ACTION_CONTINUOUS
    dw = list(discrete_weights or DEFAULT_DISCRETE_WEIGHTS)
    if len(dw) > _lib.MAX_DISCRETE:
        raise ValueError(f"at most {_lib.MAX_DISCRETE} discrete weight levels")
    cfg.num_discrete = len(dw)
    for i in range(_lib.MAX_DISCRETE):
        cfg.discrete_weights[i] = float(dw[i]) if i < len(dw) else 0.0
    cfg.min_weight = float(min_weight)
    cfg.max_weight = float(max_weight)
    cfg.reward_metric = _lib.METRICS.index(reward_metric)
    cfg.reward_field = FEATURE_NAMES.index(reward_field) if reward_field in FEATURE_NAMES else -1
    cfg.step_interval = float(step_interval)
    cfg.max_steps = int(max_steps)
    cfg.normalize_obs = 1 if normalize_obs else 0
    cfg.assign_policy = _lib.POLICIES.index(assign_policy)
    if trace is not None:
        cfg.arrival_source = _lib.ARRIVAL_TRACE
        arrival_rate = float(trace.rate)
    cfg.arrival_rate = float(arrival_rate)
    if server_rates is None:
        server_rates = [float(arrival_rate) / (float(load) * num_servers)] * num_servers
    if len(server_rates) != num_servers:
        raise ValueError("server_rates must have num_servers entries")
    for s in range(_lib.MAX_SERVERS):
        cfg.server_rate[s] = float(server_rates[s]) if s < num_servers else 0.0
    cfg.decay_factor = float(decay_factor)
    cfg.queue_capacity = int(queue_capacity)
    cfg.warmup_steps = int(warmup_steps)
    if dyn_mapping not in _lib.DYN_MAPPINGS:
        raise ValueError(f"Unknown dyn_mapping: {dyn_mapping}. Supported: {_lib.DYN_MAPPINGS}")
    cfg.dyn_mapping = _lib.DYN_MAPPINGS.index(dyn_mapping)
    if step_kernel not in _lib.STEP_KERNELS:
        raise ValueError(f"Unknown step_kernel: {step_kernel}. Supported: {_lib.STEP_KERNELS}")
    cfg.step_kernel = _lib.STEP_KERNELS.index(step_kernel)
    cfg.lost_fin_prob = float(lost_fin_prob)
    cfg.flow_timeout_s = float(flow_timeout)
    cfg.flow_buckets = int(flow_buckets)
    cfg.fail_prob = float(fail_prob)
    cfg.recover_prob = float(recover_prob)
    cfg.next_step_reset = 1 if next_step_reset else 0
    if duration_mode not in _lib.DURATION_MODES:
        raise ValueError(f"Unknown duration_mode: {duration_mode}. Supported: {_lib.DURATION_MODES}")
    cfg.duration_mode = _lib.DURATION_MODES.index(duration_mode)
    if n_flow_on_mode not in _lib.N_FLOW_ON_MODES:
        raise ValueError(f"Unknown n_flow_on_mode: {n_flow_on_mode}. Supported: {_lib.N_FLOW_ON_MODES}")
    cfg.n_flow_on_mode = _lib.N_FLOW_ON_MODES.index(n_flow_on_mode)
    cfg.lost_fin_pending = int(lost_fin_pending)
    if reservoir_mode not in _lib.RESERVOIR_MODES:
        raise ValueError(f"Unknown reservoir_mode: {reservoir_mode}. Supported: {_lib.RESERVOIR_MODES}")
    cfg.reservoir_mode = _lib.RESERVOIR_MODES.index(reservoir_mode)
    _lib.validate(cfg)
    return cfg


class Handle:
    """Owns one lbsim_t (device state of B envs on one GPU)."""

    def __init__(self, cfg: _lib.LbsimConfig, device_index: int):
        self.lib = _lib.load()
        self.cfg = cfg
        self.device_index = device_index
        h = ctypes.c_void_p()
        _lib.check(self.lib.lbsim_create(ctypes.byref(cfg), device_index, ctypes.byref(h)))
        self.h = h

    def check(self, rc: int) -> None:
        _lib.check(rc, self.h)

    def close(self) -> None:
        if getattr(self, "h", None) is not None and self.h.value is not None:
            self.lib.lbsim_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def state_bytes(self) -> bytes:
        n = ctypes.c_size_t()
        self.check(self.lib.lbsim_state_size(self.h, ctypes.byref(n)))
        buf = ctypes.create_string_buffer(n.value)
        self.check(self.lib.lbsim_get_state(self.h, buf, n.value))
        return buf.raw

    def load_state(self, data: bytes) -> None:
        self.check(self.lib.lbsim_set_state(self.h, data, len(data)))

    def set_trace(self, trace) -> None:
        """Copy a marllb_amd.trace.Trace to the device and install it (lbsim_set_trace)."""
        torch = _torch()
        dev = torch.device("cuda", self.device_index)
        gap = torch.from_numpy(trace.gap_us.view(np.int32)).to(dev)
        work = torch.from_numpy(trace.work).to(dev)
        stream = torch.cuda.current_stream(dev).cuda_stream
        self.check(self.lib.lbsim_set_trace(self.h, ctypes.c_void_p(gap.data_ptr()),
                                            ctypes.c_void_p(work.data_ptr()), trace.rows,
                                            ctypes.c_void_p(stream)))


class VecLoadBalanceEnv:
    """num_envs independent LoadBalanceEnv instances stepped together on one GPU.

    reset(mask=None) -> obs (B, S, 11) f32 cuda tensor
    step(actions)    -> obs, reward (B,) f32, done (B,) bool, info dict of tensors
    Actions: (B, S) int32/int64 indices (discrete) or float32 weights (continuous), any device.
    Discrete indices follow Python list indexing for -n <= a < n (env.py:346); out-of-range
    indices are CLAMPED on the device (a >= n -> n-1, a < -n -> 0) where the reference raises
    IndexError -- a device-side raise would need a host sync per step.  strict_actions=True checks
    the range on the host before every launch (one sync per step; for debugging callers).
    With autoreset=True, envs whose episode ended are reset inside step(); their returned obs is
    the first obs of the new episode and info['terminal_obs'] (if keep_terminal_obs) holds the
    last one, as gym/SB3 vector envs do (autoreset_mode="same_step", a masked reset launch after
    the step when some env can be done).  autoreset_mode="next_step" is gymnasium's NEXT_STEP
    mode: the step that ends an episode returns its last obs with done True, and the NEXT step
    resets that env instead of stepping it (its action is ignored; reset obs, reward 0, done
    False, episode length 0) -- inside the step's own launches, so no reset launch ever runs.
    graph_mode=True makes one step() capturable into a torch.cuda.CUDAGraph (hipGraph) and
    replayable: every output is a buffer allocated once and rewritten by each step (callers that
    keep a step's outputs must copy them), and the masked auto-reset launch runs every step (it
    leaves envs that are not done untouched) instead of being skipped on a host-side count.
    """

    def __init__(self, num_envs: int, num_servers: int = 4, *, device=None,
                 autoreset: bool = True, keep_terminal_obs: bool = False,
                 strict_actions: bool = False, feature_mode: str = "problem01",
                 graph_mode: bool = False, autoreset_mode: str = "same_step", **kwargs):
        torch = _torch()
        if autoreset_mode not in ("same_step", "next_step"):
            raise ValueError(f"Unknown autoreset_mode: {autoreset_mode}")
        if autoreset_mode == "next_step" and feature_mode == "upstream":
            raise ValueError("autoreset_mode='next_step' does not combine with feature_mode='upstream'")
        self.next_step = bool(autoreset) and autoreset_mode == "next_step"
        if self.next_step:
            kwargs["next_step_reset"] = True
        self.graph_mode = graph_mode
        self._static = {}  # graph_mode: output buffers by name
        # feature_mode "upstream": columns 1-10 follow the live agent's process_reservoir
        # (src/lb/shm_proxy.py:518-543: value-decayed mean / p90 over all 128 raw bins, f64) on the
        # simulator's reservoirs seen the VPP way (lbsim_vpp_export + lbsim_vpp_features), and the
        # reward is computed on those rows (lbsim_reward); default: problem-01's features
        if feature_mode not in ("problem01", "upstream"):
            raise ValueError(f"Unknown feature_mode: {feature_mode}")
        if feature_mode == "upstream" and kwargs.get("normalize_obs"):
            raise ValueError("feature_mode='upstream' does not combine with normalize_obs")
        self.feature_mode = feature_mode
        self._up_buf = None
        self._up_decay = float(kwargs.get("decay_factor", 0.9))  # RES_DECAY, a Python float
        self._up_ret = None  # episode returns of the upstream reward
        self.device_index = _device_index(device)
        self.device = torch.device("cuda", self.device_index)
        self.cfg = make_config(num_envs, num_servers, **kwargs)
        self.trace = kwargs.get("trace")
        self.num_envs = int(num_envs)
        self.num_servers = int(num_servers)
        self.action_type = "discrete" if self.cfg.action_type == _lib.ACTION_DISCRETE else "continuous"
        self.autoreset = autoreset
        self.keep_terminal_obs = keep_terminal_obs
        self.strict_actions = strict_actions
        self.handle = Handle(self.cfg, self.device_index)
        if self.trace is not None:
            self.handle.set_trace(self.trace)
        self._reset_done = False
        # upper bound on every env's episode step since the last full reset: while it is below
        # max_steps no env can be done, so the masked auto-reset launch is provably a no-op
        self._step_bound = 0
        # every env at the same episode step (since a full reset, and kept by auto-resets: done
        # is exactly ep_step >= max_steps, so all envs end their episodes together and the
        # auto-reset restarts all of them); a masked reset() or set_state() clears it
        self._synced = False

    # -- helpers
    def _stream(self) -> int:
        return _torch().cuda.current_stream(self.device).cuda_stream

    def _buf(self, name, shape, dtype):
        """An output tensor: fresh per call, or (graph_mode) the same buffer every call."""
        torch = _torch()
        if self.graph_mode:
            t = self._static.get(name)
            if t is None:
                t = self._static[name] = torch.empty(shape, dtype=dtype, device=self.device)
            return t
        return torch.empty(shape, dtype=dtype, device=self.device)

    def _obs_buffer(self, name="obs"):
        return self._buf(name, (self.num_envs, self.num_servers, 11), _torch().float32)

    def _action(self, actions):
        torch = _torch()
        a = torch.as_tensor(actions)
        if self.action_type == "discrete":
            if a.dtype not in (torch.int32, torch.int64):
                a = a.to(torch.int64)
            dt = _lib.DTYPE_I64 if a.dtype == torch.int64 else _lib.DTYPE_I32
        else:
            if a.dtype != torch.float32:
                a = a.to(torch.float32)
            dt = _lib.DTYPE_F32
        if a.numel() != self.num_envs * self.num_servers:
            raise ValueError(f"actions: expected {self.num_envs} x {self.num_servers} values, "
                             f"got shape {tuple(a.shape)}")
        a = a.to(self.device).reshape(self.num_envs, self.num_servers).contiguous()
        if self.strict_actions and self.action_type == "discrete":
            n = int(self.cfg.num_discrete)
            if bool(((a >= n) | (a < -n)).any()):  # env.py:346 list indexing
                raise IndexError("list index out of range")
        return a, dt

    def _mask(self, mask):
        """A reset mask as a contiguous u8 device tensor of exactly num_envs entries (the kernels
        read mask[b] for every b < B)."""
        torch = _torch()
        m = torch.as_tensor(mask)
        if m.dtype not in (torch.bool, torch.uint8):
            raise ValueError(f"reset mask must be bool or uint8, got {m.dtype}")
        if m.numel() != self.num_envs:
            raise ValueError(f"reset mask must have num_envs={self.num_envs} entries, "
                             f"got {m.numel()}")
        return m.reshape(-1).to(self.device).to(torch.uint8).contiguous()

    def _upstream(self, obs, reward=None, rows=None):
        """Overwrite obs[:, :, 1:] (and reward) with the upstream features of the current state;
        rows (bool [B]): only those envs."""
        torch = _torch()
        B, S = self.num_envs, self.num_servers
        if self._up_buf is None:
            self._up_buf = (torch.empty((B, S, 2, 128, 2), dtype=torch.float32, device=self.device),
                            torch.empty(B, dtype=torch.float32, device=self.device),
                            torch.empty((B * S * 2, 5), dtype=torch.float64, device=self.device))
        tv, ts, feats = self._up_buf
        lib, h, st = self.handle.lib, self.handle.h, self._stream()
        self.handle.check(lib.lbsim_vpp_export(h, 0, B, tv.data_ptr(), None, ts.data_ptr(), st))
        _lib.check(lib.lbsim_vpp_features(tv.data_ptr(), ts.data_ptr(), 2 * S, 2 * B * S,
                                          self._up_decay,
                                          feats.data_ptr(), st))
        f = feats.view(B, S, 10).to(torch.float32)
        if rows is None:
            obs[:, :, 1:] = f
        else:
            obs[:, :, 1:] = torch.where(rows.view(B, 1, 1), f, obs[:, :, 1:])
        if reward is not None:
            _lib.check(lib.lbsim_reward(ctypes.byref(self.cfg), obs.data_ptr(), B,
                                        reward.data_ptr(), st))
        return obs

    # -- API
    @staticmethod
    def _facade_outputs(out, facade):
        """facade = (num_agents, servers_per_agent, agent_obs, state): the problem-05 outputs the
        step / reset launch writes beside the observation (lbsim_step_outputs_t)."""
        if facade is None:
            return
        A, k, ao, stt = facade
        out.num_agents, out.servers_per_agent = A, k
        out.agent_obs = ao.data_ptr() if ao is not None else None
        out.state = stt.data_ptr() if stt is not None else None

    def reset(self, mask=None, *, facade=None):
        """Reset all envs (mask None) or those with mask[b] true; returns obs for all envs.

        With a mask, rows of envs that are not reset hold the obs of their last step() (or of
        the previous reset), so the returned tensor is always a complete batch.  facade: see
        _facade_outputs (rows of reset envs are written).
        """
        torch = _torch()
        if mask is None:
            obs = self._obs_buffer()
            out = _lib.StepOutputs()
            out.obs = obs.data_ptr()
            self._facade_outputs(out, facade)
            self.handle.check(self.handle.lib.lbsim_reset_ex(self.handle.h, None,
                                                             ctypes.byref(out), self._stream()))
            self._reset_done = True
            self._step_bound = 0
            self._synced = True
            if self.feature_mode == "upstream":
                self._upstream(obs)
                self._up_ret = None
            self._last_obs = obs
            return obs
        if not self._reset_done:
            raise RuntimeError("call reset() without a mask first")
        self._synced = False  # the reset envs restart at episode step 0, the others do not
        m = self._mask(mask)
        obs = self._last_obs if self.graph_mode else self._last_obs.clone()
        out = _lib.StepOutputs()
        out.obs = obs.data_ptr()
        self._facade_outputs(out, facade)
        self.handle.check(self.handle.lib.lbsim_reset_ex(self.handle.h, m.data_ptr(),
                                                         ctypes.byref(out), self._stream()))
        if self.feature_mode == "upstream":
            self._upstream(obs, rows=m.bool())
            if self._up_ret is not None:
                self._up_ret.masked_fill_(m.bool(), 0.0)
        self._last_obs = obs
        return obs

    def step(self, actions, *, assign_counts: bool = False, raw_obs: bool = False, facade=None
             ) -> Tuple[Any, Any, Any, Dict[str, Any]]:
        torch = _torch()
        if not self._reset_done:
            raise RuntimeError("call reset() before step()")
        a, dt = self._action(actions)
        B, S = self.num_envs, self.num_servers
        obs = self._obs_buffer()
        reward = self._buf("reward", (B,), torch.float32)
        done = self._buf("done", (B,), torch.bool)  # 1-byte 0/1, as u8
        out = _lib.StepOutputs()
        out.obs, out.reward, out.done = obs.data_ptr(), reward.data_ptr(), done.data_ptr()
        assign = raw = None
        if assign_counts:
            assign = self._buf("assign", (B, S), torch.int32)
            out.assign_count = assign.data_ptr()
        if raw_obs:
            raw = self._obs_buffer("raw_obs")
            out.raw_obs = raw.data_ptr()
        ep_len = self._buf("ep_len", (B,), torch.int32)
        ep_ret = self._buf("ep_ret", (B,), torch.float64)
        out.episode_length = ep_len.data_ptr()
        out.episode_return = ep_ret.data_ptr()
        self._facade_outputs(out, facade)
        self.handle.check(self.handle.lib.lbsim_step_ex(self.handle.h, a.data_ptr(), dt,
                                                        ctypes.byref(out), self._stream()))
        if self.feature_mode == "upstream":
            self._upstream(obs, reward)
            if raw is not None:
                raw.copy_(obs)
            if self._up_ret is None:
                self._up_ret = torch.zeros(B, dtype=torch.float64, device=self.device)
            self._up_ret += reward.to(torch.float64)
            ep_ret = self._up_ret.clone()
            if self.autoreset:  # done envs start a new episode inside this step
                self._up_ret.masked_fill_(done, 0.0)
        info: Dict[str, Any] = {"episode_length": ep_len, "episode_return": ep_ret}
        if assign is not None:
            info["assign_counts"] = assign
        if raw is not None:
            info["raw_obs"] = raw
        self._step_bound += 1
        if self.next_step:  # done envs reset inside the next step's launches
            pass
        elif self.autoreset and (self.graph_mode or self._step_bound >= self.cfg.max_steps):
            if self.keep_terminal_obs:
                info["terminal_obs"] = obs.clone()
            if self._synced and not self.graph_mode:
                self._step_bound = 0  # every env is done now and restarts at episode step 0
            # envs with done == 0 are untouched by the masked reset (no host sync needed)
            rout = _lib.StepOutputs()
            rout.obs = obs.data_ptr()
            self._facade_outputs(rout, facade)
            self.handle.check(self.handle.lib.lbsim_reset_ex(self.handle.h, done.data_ptr(),
                                                             ctypes.byref(rout), self._stream()))
            if self.feature_mode == "upstream":
                self._upstream(obs, rows=done)
        self._last_obs = obs
        return obs, reward, done, info

    def seed(self, seed: Optional[int] = None):
        if seed is None:
            seed = int.from_bytes(os.urandom(8), "little")
        self.handle.check(self.handle.lib.lbsim_seed(self.handle.h, int(seed) & (2**64 - 1)))
        return [seed]

    def get_state(self) -> bytes:
        return self.handle.state_bytes()

    def set_state(self, data: bytes) -> None:
        self.handle.load_state(data)
        self._reset_done = True
        self._step_bound = self.cfg.max_steps  # unknown episode steps: keep auto-reset armed
        self._synced = False

    def close(self) -> None:
        self.handle.close()


class LoadBalanceEnv:
    """Drop-in for the reference LoadBalanceEnv (env.py:41-470), one env, numpy I/O.

    Modes (all behind the reference's constructor, env.py:71-87):
      default                 the GPU flow simulator (one env of a VecLoadBalanceEnv); one
                              device->host copy per step (obs, raw obs, reward in one buffer)
      use_shm=True            problem-02 frames from shared memory (env.py:197-254), falling back
                              to the simulator when attach / read fails, as the reference does
      reference_plumbing=True BASELINE configs[0]: the reference's own CPU simulation mode
                              (MT19937 random observations, marllb_amd/plumbing.py), host only,
                              byte-identical to env.py for the same seed; opt-in, never a fallback
    """

    DEFAULT_DISCRETE_WEIGHTS = DEFAULT_DISCRETE_WEIGHTS

    def __init__(self, num_servers: int = 4, action_type: str = "discrete",
                 discrete_weights: Optional[List[float]] = None, max_weight: float = 10.0,
                 min_weight: float = 0.1, reward_metric: str = "jain",
                 reward_field: str = "flow_duration_avg_decay", step_interval: float = 0.25,
                 max_steps: int = 10000, use_shm: bool = False, shm_name: Optional[str] = None,
                 use_ground_truth: bool = False, normalize_obs: bool = False,
                 seed: Optional[int] = None, *, device=None, reference_plumbing: bool = False,
                 **sim_kwargs):
        self.num_servers = num_servers
        self.action_type = action_type
        self.discrete_weights = discrete_weights or self.DEFAULT_DISCRETE_WEIGHTS
        self.max_weight = max_weight
        self.min_weight = min_weight
        self.step_interval = step_interval
        self.max_steps = max_steps
        self.use_shm = use_shm
        self.shm_name = shm_name
        self.use_ground_truth = use_ground_truth
        self.normalize_obs = normalize_obs
        self.reward_metric = reward_metric
        self.reward_field = reward_field
        if reward_metric not in _lib.METRICS:  # RewardFunction.__init__ (rewards.py:321-323)
            raise ValueError(f"Unsupported metric: {reward_metric}. Supported: {_lib.METRICS}")
        self._setup_spaces()
        self.shm = None
        if self.use_shm:  # env.py:134-143: attach, or fall back to simulation
            if self.shm_name is None:
                raise ValueError("shm_name required when use_shm=True")
            from .shm import ShmRegion
            try:
                self.shm = ShmRegion.attach(self.shm_name)
                print(f"Connected to shared memory: {self.shm_name}")
            except Exception as e:
                print(f"Warning: Failed to attach shared memory: {e}")
                print("Falling back to simulation mode")
                self.use_shm = False
        self.current_step = 0
        self.last_observation = None
        self.episode_rewards: List[float] = []
        self.episode_return = 0.0
        self._last_raw = None  # un-normalised obs of the last reset/step (problem-05 loads)
        self._plumb = None
        self._vec = None
        if reference_plumbing:
            from .plumbing import ReferencePlumbing
            self._plumb = ReferencePlumbing(num_servers, seed, normalize_obs, reward_metric,
                                            reward_field)
            return
        # With a live SHM region, frames and the simulator fallback share ONE running
        # normalisation (host float64, env.py:450-470), as the reference's single obs_mean/obs_std
        # do; otherwise the device kernel normalises.
        self._host_norm = self.shm is not None and normalize_obs
        self._norm = None
        self._vec = VecLoadBalanceEnv(
            1, num_servers, device=device, autoreset=False, action_type=action_type,
            discrete_weights=self.discrete_weights, max_weight=max_weight, min_weight=min_weight,
            reward_metric=reward_metric, reward_field=reward_field,
            # step_interval is the reference's wall-clock sleep (env.py:257; 0 = none, used by
            # its tests); the simulator needs simulated time per step, 0.25 s when it is 0
            step_interval=step_interval if step_interval > 0 else 0.25,
            max_steps=max_steps, normalize_obs=normalize_obs and not self._host_norm, seed=seed,
            **sim_kwargs)
        self._io = None
        self._seq = 0
        self._dw32 = None  # (discrete_weights as a tuple, the same as float32 values in a list)
        self._active_lut: Dict[bytes, List[int]] = {}

    # ---- spaces (env.py:156-184)
    def _setup_spaces(self):
        self.observation_space, self.action_space = make_spaces(
            self.num_servers, self.action_type, self.discrete_weights, self.min_weight,
            self.max_weight, self.use_ground_truth)

    # ---- single-env I/O, zero-copy: the step kernels read the action from and write [obs | raw |
    # reward] and done into pinned host memory (device-accessible, same pointers), so a step is
    # the launches and one stream synchronisation -- no copy enqueues, no per-step allocations
    def _io_buffers(self):
        if self._io is None:
            torch = _torch()
            n = self.num_servers * NF
            host = torch.zeros(2 * n + 2, dtype=torch.float32, pin_memory=True)
            act_dt = torch.int64 if self.action_type == "discrete" else torch.float32
            act_h = torch.zeros(self.num_servers, dtype=act_dt, pin_memory=True)
            done_h = torch.zeros(8, dtype=torch.uint8, pin_memory=True)
            # the step's completion word (lbsim_step_outputs_t::done_word): polled instead of a
            # stream synchronisation
            flag_h = torch.zeros(1, dtype=torch.int32, pin_memory=True)
            self._flag = (flag_h, flag_h.numpy().view(np.uint32))
            out = _lib.StepOutputs()
            base = host.data_ptr()
            out.obs, out.raw_obs, out.reward = base, base + 4 * n, base + 8 * n
            out.done = done_h.data_ptr()
            out.done_word = flag_h.data_ptr()
            stream = torch.cuda.current_stream(self._vec.device)
            dt = _lib.DTYPE_I64 if self.action_type == "discrete" else _lib.DTYPE_F32
            self._io = (host, host.numpy(), act_h, act_h.numpy(), done_h, out, stream,
                        ctypes.c_void_p(stream.cuda_stream), dt, n,
                        ctypes.c_void_p(act_h.data_ptr()), ctypes.byref(out))
        return self._io

    def _sim_reset(self) -> np.ndarray:
        """Reset the simulator; returns the (possibly normalised) first observation."""
        obs = self._vec.reset()[0].cpu().numpy()
        self._last_raw = obs
        if self._host_norm:
            obs = self._normalize_host(obs)
        return obs

    def _sim_step(self, idx_or_w: np.ndarray):
        """One simulator step -> (obs, raw obs, reward), zero-copy through pinned host memory."""
        v = self._vec
        if not v._reset_done:  # e.g. SHM mode whose reset came from a frame
            v.reset()
        io = self._io if self._io is not None else self._io_buffers()
        cur = _torch().cuda.current_stream(v.device)
        if cur.cuda_stream != (io[7].value or 0):  # c_void_p(0).value is None
            # the caller switched streams since the buffers were made: launch on the current one,
            # so the step stays ordered after a reset() / _upstream issued on it
            io = self._io = io[:6] + (cur, ctypes.c_void_p(cur.cuda_stream)) + io[8:]
        hview, aview, stream, sptr, dt, n, aptr, outref = (io[1], io[3], io[6], io[7], io[8],
                                                           io[9], io[10], io[11])
        aview[:] = idx_or_w
        # the launch stores this step's sequence number into the pinned completion word after
        # every other output (system-scope release): spin on it instead of a stream sync, whose
        # wake-up costs several us; past _POLL_S a plain synchronisation (which reports faults)
        seq = self._seq = (self._seq + 1) & 0xFFFFFFFF or 1
        io[5].done_value = seq
        rc = v.handle.lib.lbsim_step_ex(v.handle.h, aptr, dt, outref, sptr)
        if rc != _lib.OK:
            v.handle.check(rc)
        v._step_bound += 1
        fv = self._flag[1]
        t0 = None
        while fv[0] != seq:
            if t0 is None:
                t0 = time.perf_counter()
            elif time.perf_counter() - t0 > _POLL_S:
                stream.synchronize()
                if fv[0] != seq:
                    raise RuntimeError("lbsim step finished without its completion word")
                break
        S = self.num_servers
        obs = hview[:n].reshape(S, NF).copy()
        raw = hview[n:2 * n].reshape(S, NF).copy()
        if self._host_norm:
            obs = self._normalize_host(raw)
        return obs, raw, float(hview[2 * n])

    # ---- gym API
    def reset(self) -> np.ndarray:
        self.current_step = 0
        self.episode_rewards = []
        self.episode_return = 0.0
        if self._plumb is not None:  # env.py:206-213
            obs = self._plumb.simulate()
            self._last_raw = obs
            return self._plumb.normalize(obs) if self.normalize_obs else obs
        if self.use_shm and self.shm is not None:  # env.py:197-205
            try:
                obs_dict = self.shm.read_observation()
            except Exception as e:
                obs_dict = None
                print(f"Warning: Failed to read from SHM: {e}")
            if obs_dict is not None:
                self.last_observation = obs_dict
                # the simulator starts a fresh episode lazily, at the first step that falls back
                # to it (_sim_step), so it is reset once per episode either way
                self._vec._reset_done = False
                return self._shm_obs(obs_dict)
            print("Warning: Failed to read from SHM: no observation published")
        return self._sim_reset()

    # ---- SHM path (env.py:235-254): frames in problem-02's wire format (marllb_amd/shm.py)
    def _shm_obs(self, obs_dict: dict) -> np.ndarray:
        """A msg_out frame's rows -> (S, 11): n_flow_on and the 10 reservoir features in wire
        order (problem-02 names them duration_*, problem-03 flow_duration_*; the wire order is
        the same, so the columns are taken positionally), normalised like the simulation path."""
        obs = np.zeros((self.num_servers, NF), np.float32)
        for sid, st in obs_dict.get("server_stats", {}).items():
            if sid < self.num_servers:
                obs[sid, 0] = st.get("n_flow_on", 0)
                obs[sid, 1:] = st.get("reservoir_features", [0.0] * 10)[:10]
        self._last_raw = obs
        if self.normalize_obs:
            obs = self._normalize_host(obs)
        return obs

    def _normalize_host(self, obs: np.ndarray) -> np.ndarray:
        """env.py:450-470 in float64 (the device kernel does the same for simulated envs)."""
        if self._norm is None:
            self._norm = [0, np.zeros(obs.shape), np.ones(obs.shape)]
        n, mean, std = self._norm
        n += 1
        o = obs.astype(np.float64)
        delta = o - mean
        mean = mean + delta / n
        var = (std ** 2 * (n - 1) + delta * (o - mean)) / n
        std = np.sqrt(np.maximum(var, 1e-8))
        self._norm = [n, mean, std]
        return ((o - mean) / (std + 1e-8)).astype(np.float32)

    def _shm_reward(self, raw: np.ndarray) -> float:
        """RewardFunction.compute on the frame (rewards.py:329-381) by the lbsim_reward kernel."""
        torch = _torch()
        lib = _lib.load()
        o = torch.from_numpy(np.ascontiguousarray(raw[None])).to(self._vec.device)
        out = torch.empty(1, dtype=torch.float32, device=self._vec.device)
        stream = torch.cuda.current_stream(self._vec.device).cuda_stream
        _lib.check(lib.lbsim_reward(ctypes.byref(self._vec.cfg), ctypes.c_void_p(o.data_ptr()), 1,
                                    ctypes.c_void_p(out.data_ptr()), ctypes.c_void_p(stream)))
        return float(out.item())

    def _shm_step(self, weights: np.ndarray):
        """env.py:235-254: write the weights, wait, read the next frame.  Write and read errors
        are reported and tolerated as the reference does; None = no new frame (the caller falls
        back to the simulator)."""
        try:
            seq = (self.last_observation or {}).get("sequence_id", self.current_step)
            self.shm.write_action(sequence_id=seq, weights=[float(x) for x in weights])
        except Exception as e:
            print(f"Warning: Failed to write action to SHM: {e}")
        time.sleep(self.step_interval)  # the live LB runs in wall-clock time
        try:
            obs_dict = self.shm.read_observation()
        except Exception as e:
            print(f"Warning: Failed to read from SHM: {e}")
            return None
        if obs_dict is None:
            print("Warning: Failed to read from SHM: no new observation")
            return None
        self.last_observation = obs_dict
        obs = self._shm_obs(obs_dict)
        return obs, self._last_raw, self._shm_reward(self._last_raw), obs_dict

    def step(self, action) -> Tuple[np.ndarray, float, bool, Dict[str, Any]]:
        if self._plumb is None and not (self.use_shm and self.shm is not None):
            return self._step_sim(action)
        self.current_step += 1
        weights = self._action_to_weights(action)  # IndexError on a bad index, as env.py:346
        if self._plumb is not None:  # env.py:255-286, simulation mode
            raw = self._plumb.simulate()
            obs_dict = self._array_to_dict(raw)
            reward = self._plumb.reward(obs_dict)
            next_obs = self._plumb.normalize(raw) if self.normalize_obs else raw
        else:
            a = np.asarray(action).reshape(-1)
            # int(x) truncation = astype (indices past the weights already raised above)
            act = a.astype(np.int64) if self.action_type == "discrete" else a.astype(np.float32)
            shm_res = self._shm_step(weights) if (self.use_shm and self.shm is not None) else None
            if shm_res is not None:
                next_obs, raw, reward, _ = shm_res
            else:
                next_obs, raw, reward = self._sim_step(act)
            obs_dict = None  # the per-server dict (env.py:391-423) is built when render asks
        self._last_raw = raw
        # the reference sets last_observation only in SHM mode (env.py:201,249); problem-05's
        # get_state() relies on it staying None in simulation (multi_agent_env.py:249-254)
        self._last_obs_dict = obs_dict
        self._last_obs_step = self.current_step
        self.episode_rewards.append(reward)
        self.episode_return += reward
        done = self.current_step >= self.max_steps
        active = (obs_dict["active_servers"] if obs_dict is not None
                  else np.flatnonzero((raw > 0).any(axis=1)).tolist())  # env.py:410-413
        info = {
            "step": self.current_step,
            "weights": weights.tolist(),
            "active_servers": active,
            "episode_return": self.episode_return,
        }
        if done:
            info["episode"] = {"r": self.episode_return, "l": self.current_step}
        return next_obs, reward, done, info

    def _step_sim(self, action) -> Tuple[np.ndarray, float, bool, Dict[str, Any]]:
        """step() on the GPU simulator (no SHM, no plumbing): the same results and info as the
        general path, with its host bookkeeping in list form (the problem-04 Trainer calls this
        once per simulated step and waits for it)."""
        self.current_step += 1
        if self.action_type == "discrete":
            # env.py:346: discrete_weights[int(a)] (IndexError on a bad index, negative indices as
            # Python's), reported as the float32 values the reference's np.array holds
            idx = np.asarray(action).reshape(-1)
            il = idx.tolist()
            dw = self.discrete_weights
            key = tuple(dw)
            if self._dw32 is None or self._dw32[0] != key:
                self._dw32 = (key, np.asarray(dw, dtype=np.float32).tolist())
            w32 = self._dw32[1]
            weights = [w32[int(a)] for a in il]
            act = idx if idx.dtype == np.int64 else idx.astype(np.int64)
        else:
            wa = action_to_weights(action, self.action_type, self.discrete_weights,
                                   self.min_weight, self.max_weight)
            weights = wa.tolist()
            act = np.asarray(action).reshape(-1).astype(np.float32)
        next_obs, raw, reward = self._sim_step(act)
        self._last_raw = raw
        self._last_obs_dict = None  # built when render asks (env.py:391-423)
        self._last_obs_step = self.current_step
        self.episode_rewards.append(reward)
        self.episode_return += reward
        done = self.current_step >= self.max_steps
        # env.py:410-413 (active = any feature > 0), one lookup per activity pattern
        pat = (raw > 0).any(1).tobytes()
        act_l = self._active_lut.get(pat)
        if act_l is None:
            act_l = self._active_lut[pat] = np.flatnonzero(np.frombuffer(pat, np.bool_)).tolist()
        info = {
            "step": self.current_step,
            "weights": weights,
            "active_servers": list(act_l),
            "episode_return": self.episode_return,
        }
        if done:
            info["episode"] = {"r": self.episode_return, "l": self.current_step}
        return next_obs, reward, done, info

    def render(self, mode: str = "human"):
        if mode == "human":
            print(f"\n{'=' * 60}")
            print(f"Step: {self.current_step}/{self.max_steps}")
            print(f"Episode Return: {self.episode_return:.4f}")
            obs_dict = self.last_observation or getattr(self, "_last_obs_dict", None)
            if obs_dict is None and getattr(self, "_last_raw", None) is not None:
                obs_dict = array_to_dict(self._last_raw, getattr(self, "_last_obs_step", 0))
            if obs_dict:
                active = obs_dict.get("active_servers", [])
                stats = obs_dict.get("server_stats", {})
                print(f"Active Servers: {active}")
                print(f"\n{'Server':<10} {'n_flows':<10} {'fct_mean':<12} {'fct_p90':<12} "
                      f"{'dur_decay':<12}")
                print("-" * 60)
                for sid in active:
                    st = stats.get(sid, {})
                    print(f"{sid:<10} {st.get('n_flow_on', 0):<10.0f} "
                          f"{st.get('fct_mean', 0):<12.4f} {st.get('fct_p90', 0):<12.4f} "
                          f"{st.get('flow_duration_avg_decay', 0):<12.4f}")
            print("=" * 60)

    def close(self):
        if self.shm is not None:
            self.shm.close()
            self.shm = None
        if self._vec is not None:
            self._vec.close()

    def seed(self, seed: Optional[int] = None):  # env.py:327-330
        if self._plumb is not None:
            self._plumb.seed(seed)
        else:
            self._vec.seed(seed)
        return [seed]

    # ---- reference helpers (host plumbing, env.py:334-423)
    def _action_to_weights(self, action) -> np.ndarray:
        return action_to_weights(action, self.action_type, self.discrete_weights,
                                 self.min_weight, self.max_weight)

    def _dict_to_array(self, obs_dict: dict) -> np.ndarray:
        return dict_to_array(obs_dict, self.num_servers)

    def _array_to_dict(self, obs: np.ndarray) -> dict:
        return array_to_dict(obs, self.current_step)


class LoadBalanceEnvGym(LoadBalanceEnv):
    """env.py:474-481 alias (gym.Env mixin not needed: no gym dependency)."""

    metadata = {"render.modes": ["human"]}
