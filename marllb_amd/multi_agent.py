"""problem-05 multi-agent facade over the GPU simulator (config C5).

`MultiAgentLoadBalanceEnv` mirrors `simulation-mode/problem-05-qmix/src/multi_agent_env.py:22-282`
over `marllb_amd.LoadBalanceEnv`; `VecMultiAgentLoadBalanceEnv` is its batched GPU form.

Contract (SURVEY §0.6 -- the reference wrapper does not compose with QMIXAgent as written; this
facade reproduces its actual I/O and fixes only what crashes):
  * per-agent observation = the wrapper's 4-value slices of the flattened (S, 11) obs for the
    agent's servers, then flat[4 S:] -> 4 k + 7 S values (128 at 4 agents x 4 servers; the
    wrapper's declared obs_dim of 4 k + 4 is kept as `declared_obs_dim`, `obs_dim` is the real one)
    (multi_agent_env.py:152-188); float64 in the single-env facade as in the reference;
  * get_state() = zeros(4 S) ++ [0, 0, 0, 0, 0, 0, 0, 0, step / max_steps, A] -> 4 S + 10 (74):
    the reference's simulation-mode value (last_observation stays None, no request counters;
    multi_agent_env.py:228-272);
  * global reward replicated per agent (multi_agent_env.py:143-147);
  * FIX 1: an agent action may be a scalar (QMIXAgent.select_actions returns one int per agent,
    qmix_agent.py:164): it is broadcast to the agent's k servers, where the reference raises
    TypeError on len(int) (multi_agent_env.py:205);
  * FIX 2: info['server_loads'] (n_flow_on per server) is emitted, so global_reward=False computes
    the wrapper's local Jain index instead of raising KeyError (multi_agent_env.py:226).
"""
from __future__ import annotations

import ctypes
from typing import Any, Dict, List

import numpy as np

from . import _lib
from .env import LoadBalanceEnv, VecLoadBalanceEnv, _torch


def agent_obs_dim(num_agents: int, servers_per_agent: int) -> int:
    return 4 * servers_per_agent + 7 * num_agents * servers_per_agent


class MultiAgentLoadBalanceEnv:
    """multi_agent_env.py:22-282 over the GPU simulator (one env)."""

    def __init__(self, num_agents: int = 4, servers_per_agent: int = 4,
                 action_type: str = "continuous", reward_metric: str = "jain",
                 max_steps: int = 100, use_shm: bool = False, global_reward: bool = True,
                 **sim_kwargs):
        self.num_agents = num_agents
        self.servers_per_agent = servers_per_agent
        self.total_servers = num_agents * servers_per_agent
        self.global_reward = global_reward
        self.env = LoadBalanceEnv(num_servers=self.total_servers, action_type=action_type,
                                  reward_metric=reward_metric, max_steps=max_steps,
                                  use_shm=use_shm, **sim_kwargs)
        self.agent_servers = {i: list(range(i * servers_per_agent, (i + 1) * servers_per_agent))
                              for i in range(num_agents)}
        self.observation_space = self.env.observation_space
        self.action_space = self.env.action_space
        self.declared_obs_dim = servers_per_agent * 4 + 4  # multi_agent_env.py:86-93
        self.obs_dim = agent_obs_dim(num_agents, servers_per_agent)
        self.state_dim = self.total_servers * 4 + 10      # multi_agent_env.py:95-98
        self._server_loads = [0.0] * self.total_servers

    def reset(self) -> List[np.ndarray]:
        g = self.env.reset()
        self._server_loads = [float(x) for x in self.env._last_raw[:, 0]]
        return [self._get_agent_observation(g, i) for i in range(self.num_agents)]

    def step(self, actions):
        g, reward, done, info = self.env.step(self._combine_actions(actions))
        # raw n_flow_on (not the normalised column) of this step
        self._server_loads = [float(x) for x in self.env._last_raw[:, 0]]
        info = dict(info)
        info["server_loads"] = list(self._server_loads)  # FIX 2
        obs = [self._get_agent_observation(g, i) for i in range(self.num_agents)]
        rewards = ([reward] * self.num_agents if self.global_reward
                   else self._compute_local_rewards(info))
        return obs, rewards, done, info

    def _get_agent_observation(self, global_obs: np.ndarray, agent_id: int) -> np.ndarray:
        flat = np.asarray(global_obs).flatten()
        own = []
        for s in self.agent_servers[agent_id]:
            own.extend(flat[4 * s:4 * s + 4].tolist())
        return np.concatenate([np.array(own).flatten(), flat[self.total_servers * 4:].flatten()])

    def _combine_actions(self, actions) -> np.ndarray:
        out = np.zeros(self.total_servers)
        for agent_id, action in enumerate(actions):
            a = np.asarray(action)
            if a.ndim == 0:  # FIX 1: one value per agent
                a = np.full(self.servers_per_agent, a.item())
            for i, s in enumerate(self.agent_servers[agent_id]):
                if i < len(a):
                    out[s] = a[i]
        return out

    def _compute_local_rewards(self, info: Dict[str, Any]) -> List[float]:
        rewards = []
        for agent_id in range(self.num_agents):
            loads = [info["server_loads"][i] for i in self.agent_servers[agent_id]]
            s = sum(loads)
            if s == 0:
                rewards.append(0.0)
            else:
                sq = sum(x ** 2 for x in loads)
                rewards.append((s ** 2) / (self.servers_per_agent * sq + 1e-8))
        return rewards

    def get_state(self) -> np.ndarray:
        loads = np.zeros(self.total_servers)
        metrics = [0, 0, 0, 0, 0, np.std(loads), np.max(loads), np.min(loads),
                   self.env.current_step / self.env.max_steps, self.num_agents]
        return np.concatenate([np.zeros(self.total_servers * 4), metrics])

    def render(self, mode: str = "human"):
        return self.env.render(mode)

    def close(self):
        self.env.close()


class VecMultiAgentLoadBalanceEnv:
    """B problem-05 multi-agent envs on one GPU.

    reset(mask=None)  -> obs (B, A, 4k + 7S) f32
    step(actions)     -> obs (B, A, D), rewards (B, A), done (B,), info
    get_state()       -> (B, 4S + 10) f32 (the wrapper's simulation-mode state)
    actions: (B, A) one value per agent (broadcast to its k servers), (B, A, k) or (B, S).
    """

    def __init__(self, num_envs: int, num_agents: int = 4, servers_per_agent: int = 4, *,
                 device=None, action_type: str = "continuous", max_steps: int = 100,
                 global_reward: bool = True, **kwargs):
        torch = _torch()
        self.num_envs, self.num_agents, self.k = int(num_envs), num_agents, servers_per_agent
        self.S = num_agents * servers_per_agent
        self.global_reward = global_reward
        self.vec = VecLoadBalanceEnv(num_envs, self.S, device=device, action_type=action_type,
                                     max_steps=max_steps, **kwargs)
        self.device = self.vec.device
        self.max_steps = max_steps
        self.obs_dim = agent_obs_dim(num_agents, servers_per_agent)
        self.state_dim = self.S * 4 + 10
        self.lib = _lib.load()
        self._state = None  # the state the last step / reset launch wrote (get_state)

    def agent_obs(self, obs, out=None):
        """(B, S, 11) -> (B, A, 4k + 7S) by lbsim_agent_obs (into `out` when given)."""
        torch = _torch()
        obs = obs.contiguous()
        if out is None:
            out = torch.empty((obs.shape[0], self.num_agents, self.obs_dim), dtype=torch.float32,
                              device=self.device)
        stream = torch.cuda.current_stream(self.device).cuda_stream
        self.vec.handle.check(self.lib.lbsim_agent_obs(
            ctypes.c_void_p(obs.data_ptr()), obs.shape[0], self.S, self.num_agents, self.k,
            ctypes.c_void_p(out.data_ptr()), ctypes.c_void_p(stream)))
        return out

    def expand_actions(self, actions):
        torch = _torch()
        a = actions if isinstance(actions, torch.Tensor) else torch.as_tensor(np.asarray(actions))
        a = a.to(self.device)
        if a.dim() == 2 and a.shape[1] == self.num_agents and self.num_agents != self.S:
            return a.repeat_interleave(self.k, dim=1)
        if a.dim() == 3:
            return a.reshape(a.shape[0], self.S)
        return a

    def _facade(self, masked: bool):
        """Fresh per-call output tensors for the launch to fill (callers may keep them: value
        semantics without a copy kernel); a masked reset starts from the previous state.  In the
        inner env's graph_mode: the same two buffers every call (rewritten in place)."""
        torch = _torch()
        v = self.vec
        ao = v._buf("agent_obs", (self.num_envs, self.num_agents, self.obs_dim), torch.float32)
        if masked and self._state is not None and not v.graph_mode:
            st = self._state.clone()
        else:
            st = v._buf("state", (self.num_envs, self.state_dim), torch.float32)
        return (self.num_agents, self.k, ao, st)

    def reset(self, mask=None):
        """The per-agent observations and the state come from the reset launch itself."""
        f = self._facade(mask is not None)
        obs = self.vec.reset(mask=mask, facade=f)
        ao = f[2]
        if self.vec.feature_mode == "upstream":
            # the launch wrote agent_obs from problem-01 rows; _upstream then replaced columns
            # 1-10 of obs: the agent observations follow the returned rows
            ao = self.agent_obs(obs, out=ao)
        elif mask is not None and not self.vec.graph_mode:  # rows of envs not reset: their last
            ao = self.agent_obs(obs)                         # agent observations
        self._state = f[3]
        return ao

    def step(self, actions):
        torch = _torch()
        v = self.vec
        # server loads are this step's raw n_flow_on: the un-normalised column, and for envs the
        # masked auto-reset restarts, the terminal step's value (not the next episode's first
        # obs, which step() writes over `obs`).  raw_obs is requested only when they can differ.
        need_raw = bool(v.cfg.normalize_obs) or v.graph_mode or (
            v.autoreset and v._step_bound + 1 >= v.cfg.max_steps)
        f = self._facade(False)
        obs, rew, done, info = v.step(self.expand_actions(actions), raw_obs=need_raw, facade=f)
        self._state = f[3]  # written by the step launch (and the auto-reset launch's rows)
        ao = f[2]
        if v.feature_mode == "upstream":  # as in reset(): the rows step() returns
            ao = self.agent_obs(obs, out=ao)
        loads = (info["raw_obs"] if need_raw else obs)[:, :, 0]
        info = dict(info)
        info["server_loads"] = loads
        if self.global_reward:
            rewards = rew.unsqueeze(1).expand(-1, self.num_agents)
        else:  # the wrapper's local Jain index per agent (multi_agent_env.py:212-236)
            l = loads.double().view(-1, self.num_agents, self.k)
            s, sq = l.sum(2), (l * l).sum(2)
            rewards = torch.where(s == 0, torch.zeros_like(s),
                                  s * s / (self.k * sq + 1e-8)).float()
        return ao, rewards, done, info

    def get_state(self):
        """(B, 4S + 10): written by the last step / reset launch into a tensor of its own, never
        written again (value semantics without a copy)."""
        if self._state is None:
            raise RuntimeError("call reset() before get_state()")
        return self._state

    def close(self):
        self.vec.close()
