"""Policy-in-the-loop rollouts on one GPU: the networks of problem-04 / problem-05 drive the batched
simulator with no host round trip (BASELINE configs[3] and configs[4]).

SACGRURollout  problem-04 Trainer's acting loop (trainer.py:96-126): flattened (S*11) state ->
               PolicyNetwork.sample (GRU hidden state resident, (1, B, 128)) -> continuous weights
               -> env.step; hidden state of finished envs zeroed (init_hidden at episode start,
               folded into the next policy launch).
QMIXRollout    problem-05 QMIXAgent.select_actions (qmix_agent.py:138-178) over the multi-agent
               facade: per-agent GRU Q-networks, epsilon-greedy argmax, one int per agent, then
               the mixing network on the chosen Q-values and the global state (qmix_agent.py:110).
"""
from __future__ import annotations

from typing import List, Optional

import torch

from .env import VecLoadBalanceEnv
from .multi_agent import VecMultiAgentLoadBalanceEnv
from .policies import (AgentQNet, FusedAgentQNets, FusedGRUPolicy, FusedQMIXPolicy, FusedQMixer,
                       GRUPolicy, QMixer)


class SACGRURollout:
    def __init__(self, env: VecLoadBalanceEnv, policy: Optional[GRUPolicy] = None,
                 deterministic: bool = False, seed: int = 0, fused: bool = True):
        self.env = env
        S = env.num_servers
        self.policy = (policy or GRUPolicy(S * 11, S, 256, 128)).to(env.device).eval()
        # fused: one lbsim_sac_actor_step launch per step at the reference widths (else hipBLASLt
        # GEMMs + lbsim_gru_gates / lbsim_sac_head), noise from Philox; unfused: the torch module
        # (noise from torch's generator)
        self.fused = FusedGRUPolicy(self.policy, seed=seed) if fused else None
        self.deterministic = deterministic
        self.gen = torch.Generator(device=env.device)
        self.gen.manual_seed(seed)
        self._h = torch.zeros(1, env.num_envs, self.policy.gru_dim, device=env.device)
        self._reset = None  # done of the last step: those envs start the next one from h = 0
        self.obs = env.reset()

    @property
    def hidden(self):
        """The GRU state the next step starts from, (1, B, gru): init_hidden (zeros) for envs whose
        episode just ended (trainer.py:96-98)."""
        if self._reset is None:
            return self._h
        return self._h * (~self._reset).view(1, -1, 1).to(self._h.dtype)

    def capture(self, warmup: int = 2, steps: int = 1) -> "torch.cuda.CUDAGraph":
        """`steps` step()s captured into one torch.cuda.CUDAGraph (as QMIXRollout.capture): needs
        the one-launch actor kernel and an env in graph_mode; `warmup` eager steps first on a side
        stream, then g.replay() == `steps` step()s on the same static buffers (self.obs,
        self.last: the last step's outputs).  Several steps per graph amortise the replay's own
        launch cost."""
        if self.fused is None or self.fused.kernel is None or not self.env.graph_mode:
            raise ValueError("capture needs the fused SAC actor kernel and graph_mode=True")
        self.fused.use_device_step()
        side = torch.cuda.Stream(self.env.device)
        side.wait_stream(torch.cuda.current_stream(self.env.device))
        with torch.cuda.stream(side):
            for _ in range(max(1, warmup)):
                self.step()
        torch.cuda.current_stream(self.env.device).wait_stream(side)
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            for _ in range(max(1, steps)):
                self.last = self.step()
        return g

    @torch.no_grad()
    def step(self):
        B = self.env.num_envs
        state = self.obs.reshape(B, -1)
        if self.fused is not None:  # hidden updated in place, finished envs zeroed in the launch
            action, _, _ = self.fused(state, self._h[0], self.deterministic,
                                      reset_mask=self._reset, inplace=True)
        else:
            mean, log_std, self._h = self.policy(state, self.hidden)
            if self.deterministic:
                action = self.policy.squash(mean)
            else:
                eps = torch.randn(mean.shape, device=mean.device, generator=self.gen)
                action = self.policy.squash(mean + log_std.exp() * eps)
        obs, rew, done, info = self.env.step(action)
        self._reset = done
        self.obs = obs
        return rew, done, info


class QMIXRollout:
    def __init__(self, env: VecMultiAgentLoadBalanceEnv, agents: Optional[List[AgentQNet]] = None,
                 mixer: Optional[QMixer] = None, n_actions: int = 3, epsilon: float = 0.05,
                 seed: int = 0, fused: bool = True):
        self.env = env
        A, dev = env.num_agents, env.device
        self.agents = [(agents[a] if agents else AgentQNet(env.obs_dim, n_actions, 128, 64))
                       .to(dev).eval() for a in range(A)]
        self.mixer = (mixer or QMixer(A, env.state_dim, 32, 64)).to(dev).eval()
        self.epsilon = epsilon
        self.n_actions = n_actions
        self.gen = torch.Generator(device=dev)
        self.gen.manual_seed(seed)
        H = self.agents[0].gru_dim
        # fused: one lbsim_qmix_policy_step launch per step at the reference widths (agents,
        # epsilon-greedy with Philox noise, mixer; hidden (B, A, gru)), else hipBLASLt GEMMs + HIP
        # epilogues (hidden (A, B, gru)); unfused: the torch modules (a (1, B, gru) list)
        self.kernel = self.fused = None
        self._reset = None
        if fused and FusedQMIXPolicy.supported(self.agents, self.mixer, n_actions):
            self.kernel = FusedQMIXPolicy(self.agents, self.mixer, n_actions, epsilon, seed,
                                          env.k)
            self.hidden = torch.zeros(env.num_envs, A, H, device=dev)
        elif fused:
            self.fused = (FusedAgentQNets(self.agents), FusedQMixer(self.mixer))
            self.hidden = torch.zeros(A, env.num_envs, H, device=dev)
        else:
            self.hidden = [torch.zeros(1, env.num_envs, H, device=dev) for _ in self.agents]
        self.obs = env.reset()

    def capture(self, warmup: int = 2, steps: int = 1) -> "torch.cuda.CUDAGraph":
        """`steps` step()s captured into one torch.cuda.CUDAGraph: needs the fused kernel and an
        env in graph_mode (static buffers, auto-reset launched every step); the Philox step
        counter moves to the device.  `warmup` eager steps first (on a side stream, as torch
        requires), then g.replay() == `steps` step()s on the same static buffers (self.obs,
        self.hidden, ...)."""
        if self.kernel is None or not self.env.vec.graph_mode:
            raise ValueError("capture needs the fused QMIX kernel and graph_mode=True")
        self.kernel.use_device_step()
        side = torch.cuda.Stream(self.env.device)
        side.wait_stream(torch.cuda.current_stream(self.env.device))
        with torch.cuda.stream(side):
            for _ in range(max(1, warmup)):
                self.step()
        torch.cuda.current_stream(self.env.device).wait_stream(side)
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            for _ in range(max(1, steps)):
                self.last = self.step()
        return g

    @torch.no_grad()
    def step(self):
        B, A = self.env.num_envs, self.env.num_agents
        state = self.env.get_state()
        if self.kernel is not None:  # envs that finished last step restart from h = 0
            _, server_actions, q_tot, _ = self.kernel(self.obs, self.hidden, state,
                                                      reset_mask=self._reset)
            obs, rewards, done, info = self.env.step(server_actions)
            self._reset = done
            self.obs = obs
            return q_tot, rewards, done, info
        if self.fused is not None:
            nets, mixer = self.fused
            q, self.hidden = nets(self.obs.transpose(0, 1).contiguous(), self.hidden)  # (A, B, n)
            greedy = q.argmax(dim=2)
            rnd = torch.randint(0, self.n_actions, (A, B), device=q.device, generator=self.gen)
            explore = torch.rand((A, B), device=q.device, generator=self.gen) < self.epsilon
            act = torch.where(explore, rnd, greedy)
            chosen = q.gather(2, act.unsqueeze(2)).squeeze(2).t().contiguous()  # (B, A)
            q_tot = mixer(chosen, state)
            obs, rewards, done, info = self.env.step(act.t())
            self.hidden = self.hidden * (~done).view(1, B, 1).float()
            self.obs = obs
            return q_tot, rewards, done, info
        qs, acts = [], []
        for a, net in enumerate(self.agents):
            q, self.hidden[a] = net(self.obs[:, a], self.hidden[a])
            greedy = q.argmax(dim=1)
            rnd = torch.randint(0, self.n_actions, (B,), device=q.device, generator=self.gen)
            explore = torch.rand(B, device=q.device, generator=self.gen) < self.epsilon
            act = torch.where(explore, rnd, greedy)
            qs.append(q.gather(1, act.unsqueeze(1)))
            acts.append(act)
        actions = torch.stack(acts, dim=1)
        q_tot = self.mixer(torch.cat(qs, dim=1), state)
        obs, rewards, done, info = self.env.step(actions)
        keep = (~done).view(1, B, 1).float()
        self.hidden = [h * keep for h in self.hidden]
        self.obs = obs
        return q_tot, rewards, done, info
