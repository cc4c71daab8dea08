"""On-GPU policy and mixing networks that drive the batched env.

Module mirrors of the reference networks with identical parameter names and shapes, so a
reference checkpoint's state_dict loads unchanged (`load_state_dict(torch.load(...))`):

  GRUPolicy   problem-04 PolicyNetwork (src/networks.py:19-151): GRU(state -> 128), fc1 -> 256,
              ReLU, fc_mean / fc_logstd -> action_dim, log_std clamped to [-20, 2]; actions
              tanh(N(mean, std)) * scale + bias.
  AgentQNet   problem-05 AgentQNetwork (src/agent_network.py:13-92): GRU(obs -> 64), fc1 -> 128,
              fc2 -> 128 (ReLU), fc3 -> action_dim Q-values.
  QMixer      problem-05 QMixingNetwork (src/mixing_network.py:15-117): hypernetworks of the
              global state give |W1| (A x 32), b1, |W2| (32), b2; Q_tot = elu(q W1 + b1) W2 + b2.

These modules run on the GPU as torch fp32 (GEMMs through hipBLASLt); they are also the fp32
reference for the fused inference forms below (one MFMA kernel per step at the reference widths).  Rollout harnesses (marllb_amd/rollout.py) keep the GRU
hidden state resident on the device and feed actions to lbsim_step without a host round trip.
"""
from __future__ import annotations

import ctypes
from typing import Optional

import torch
import torch.nn as nn
import torch.nn.functional as F


class GRUPolicy(nn.Module):
    """PolicyNetwork (networks.py:19-151) with identical parameters."""

    def __init__(self, state_dim: int, action_dim: int, hidden_dim: int = 256, gru_dim: int = 128,
                 action_scale: float = 1.0, action_bias: float = 0.0, log_std_min: float = -20,
                 log_std_max: float = 2):
        super().__init__()
        self.state_dim, self.action_dim = state_dim, action_dim
        self.hidden_dim, self.gru_dim = hidden_dim, gru_dim
        self.action_scale, self.action_bias = action_scale, action_bias
        self.log_std_min, self.log_std_max = log_std_min, log_std_max
        self.gru = nn.GRU(state_dim, gru_dim, batch_first=True)
        self.fc1 = nn.Linear(gru_dim, hidden_dim)
        self.fc_mean = nn.Linear(hidden_dim, action_dim)
        self.fc_logstd = nn.Linear(hidden_dim, action_dim)
        self.apply(_init_weights)

    def forward(self, state: torch.Tensor, hidden: torch.Tensor):
        """state (B, state_dim), hidden (1, B, gru_dim) -> mean, log_std, hidden_new."""
        out, h1 = self.gru(state.unsqueeze(1), hidden)
        x = F.relu(self.fc1(out.squeeze(1)))
        mean = self.fc_mean(x)
        log_std = torch.clamp(self.fc_logstd(x), self.log_std_min, self.log_std_max)
        return mean, log_std, h1

    def init_hidden(self, batch_size: int = 1) -> torch.Tensor:
        return torch.zeros(1, batch_size, self.gru_dim)

    def squash(self, x: torch.Tensor) -> torch.Tensor:
        return torch.tanh(x) * self.action_scale + self.action_bias

    def sample(self, state, hidden):
        """networks.py:113-146: (action, log_prob, deterministic action, hidden_new)."""
        mean, log_std, h1 = self.forward(state, hidden)
        std = log_std.exp()
        x = mean + std * torch.randn_like(mean)
        y = torch.tanh(x)
        action = y * self.action_scale + self.action_bias
        log_prob = (-((x - mean) ** 2) / (2 * std ** 2) - log_std
                    - 0.5 * torch.log(torch.tensor(2 * torch.pi, device=x.device)))
        log_prob = log_prob - torch.log(self.action_scale * (1 - y.pow(2)) + 1e-6)
        return action, log_prob.sum(1, keepdim=True), self.squash(mean), h1


class AgentQNet(nn.Module):
    """AgentQNetwork (agent_network.py:13-92) with identical parameters."""

    def __init__(self, obs_dim: int, action_dim: int, hidden_dim: int = 128, gru_dim: int = 64):
        super().__init__()
        self.obs_dim, self.action_dim = obs_dim, action_dim
        self.hidden_dim, self.gru_dim = hidden_dim, gru_dim
        self.gru = nn.GRU(obs_dim, gru_dim, batch_first=True)
        self.fc1 = nn.Linear(gru_dim, hidden_dim)
        self.fc2 = nn.Linear(hidden_dim, hidden_dim)
        self.fc3 = nn.Linear(hidden_dim, action_dim)
        self.apply(_init_weights)

    def forward(self, obs: torch.Tensor, hidden: torch.Tensor):
        out, h1 = self.gru(obs.unsqueeze(1), hidden)
        x = F.relu(self.fc1(out.squeeze(1)))
        x = F.relu(self.fc2(x))
        return self.fc3(x), h1

    def init_hidden(self, batch_size: int = 1) -> torch.Tensor:
        return torch.zeros(1, batch_size, self.gru_dim)


class QMixer(nn.Module):
    """QMixingNetwork (mixing_network.py:15-117) with identical parameters."""

    def __init__(self, num_agents: int, state_dim: int, mixing_embed_dim: int = 32,
                 hypernet_embed_dim: int = 64):
        super().__init__()
        self.num_agents, self.state_dim = num_agents, state_dim
        self.mixing_embed_dim, self.hypernet_embed_dim = mixing_embed_dim, hypernet_embed_dim
        e, he = mixing_embed_dim, hypernet_embed_dim
        self.hyper_w1 = nn.Sequential(nn.Linear(state_dim, he), nn.ReLU(),
                                      nn.Linear(he, num_agents * e))
        self.hyper_b1 = nn.Sequential(nn.Linear(state_dim, e))
        self.hyper_w2 = nn.Sequential(nn.Linear(state_dim, he), nn.ReLU(), nn.Linear(he, e))
        self.hyper_b2 = nn.Sequential(nn.Linear(state_dim, he), nn.ReLU(), nn.Linear(he, 1))

    def forward(self, agent_qs: torch.Tensor, state: torch.Tensor) -> torch.Tensor:
        """agent_qs (B, A), state (B, state_dim) -> Q_tot (B, 1)."""
        b = agent_qs.size(0)
        w1 = torch.abs(self.hyper_w1(state)).view(b, self.num_agents, self.mixing_embed_dim)
        b1 = self.hyper_b1(state).view(b, 1, self.mixing_embed_dim)
        w2 = torch.abs(self.hyper_w2(state)).view(b, self.mixing_embed_dim, 1)
        b2 = self.hyper_b2(state)
        hidden = F.elu(torch.bmm(agent_qs.view(b, 1, self.num_agents), w1) + b1)
        return torch.bmm(hidden, w2).squeeze(1) + b2


def _init_weights(m: nn.Module) -> None:
    """Xavier-uniform linear weights, orthogonal GRU weights, zero biases (networks.py:70-80)."""
    if isinstance(m, nn.Linear):
        nn.init.xavier_uniform_(m.weight)
        nn.init.constant_(m.bias, 0.0)
    elif isinstance(m, nn.GRU):
        for name, p in m.named_parameters():
            if "weight" in name:
                nn.init.orthogonal_(p)
            else:
                nn.init.constant_(p, 0.0)


def load_prefixed(module: nn.Module, arrays, prefix: str) -> nn.Module:
    """Load a state_dict stored as `<prefix>.<name>` arrays (tests/golden/nets.npz)."""
    sd = {k[len(prefix) + 1:]: torch.from_numpy(arrays[k]) for k in arrays.files
          if k.startswith(prefix + ".")}
    module.load_state_dict(sd)
    return module


# ---------------------------------------------------------------------------- fused inference
# Two forms.  One kernel per step (lbsim_sac_actor_step / lbsim_qmix_policy_step, csrc/lbsim_fused.h:
# the whole network of a tile of envs on the f32 MFMA, activations in LDS) at the reference's
# layer widths; otherwise hipBLASLt GEMMs (torch.addmm / baddbmm, ReLU as the GEMM epilogue) with
# every elementwise stage in our HIP kernels (csrc/lbsim_nets.h).  Inference only (no autograd);
# the torch modules above are the fp32 reference both are tested against.

def _lib_and_stream(device):
    from . import _lib
    lib = _lib.load()
    return lib, ctypes.c_void_p(torch.cuda.current_stream(device).cuda_stream)


def _ptr(t: Optional[torch.Tensor]):
    return None if t is None else ctypes.c_void_p(t.data_ptr())


def _linear_relu(x, w, b):
    """x @ w.T + b with ReLU fused into the GEMM epilogue when torch exposes it."""
    f = getattr(torch, "_addmm_activation", None)
    if f is not None:
        return f(b, x, w.t())
    return torch.relu_(torch.addmm(b, x, w.t()))


def pack_linear(w: torch.Tensor, n_pad: Optional[int] = None) -> torch.Tensor:
    """A Linear weight [N, K] in the MFMA-fragment order of csrc/lbsim_fused.h: zero-padded to
    [16 NT, 16 KB] (N to n_pad if given), P[nt][kb][l][s] = W[16 nt + (l & 15)][16 kb + 4 (l >> 4)
    + s], flat float32."""
    n, k = w.shape
    npd = n_pad if n_pad is not None else -(-n // 16) * 16
    kpd = -(-k // 16) * 16
    p = torch.zeros(npd, kpd, dtype=torch.float32, device=w.device)
    p[:n, :k] = w.detach()
    return p.view(npd // 16, 16, kpd // 16, 4, 4).permute(0, 2, 3, 1, 4).contiguous().view(-1)


def _pad_vec(v: torch.Tensor, n: int) -> torch.Tensor:
    out = torch.zeros(n, dtype=torch.float32, device=v.device)
    out[:v.numel()] = v.detach().reshape(-1)
    return out


# bench.py sets this to a list to collect (start, end) CUDA events around each fused launch
profile_events: Optional[list] = None


class _ParamWatch:
    """Notices when the torch modules behind a fused form change their weights: every in-place
    update (optimizer.step, load_state_dict, copy_) bumps a parameter's version counter, and a
    re-registered parameter changes identity.  The fused forms keep packed COPIES of the weights,
    so they check this before each launch and repack in place (same device pointers) when needed.
    Assigning `param.data = ...` bypasses the counter: call sync_weights() after that."""

    def __init__(self, modules):
        self.params = [p for m in modules for p in m.parameters()]
        self.sig = self._sig()

    def _sig(self):
        return [(id(p), p._version) for p in self.params]

    def changed(self) -> bool:
        s = self._sig()
        if s == self.sig:
            return False
        self.sig = s
        return True


def _copy_into(dst, src):
    for d, x in zip(dst, src):
        d.copy_(x)


def _timed(launch):
    if profile_events is None:
        return launch()
    # fence-free HIP events (_lib.TimingEvent) on the stream the policy kernel is launched on
    from . import _lib
    stream = torch.cuda.current_stream().cuda_stream
    e0, e1 = _lib.TimingEvent(), _lib.TimingEvent()
    e0.record(stream)
    rc = launch()
    e1.record(stream)
    profile_events.append((e0, e1))
    return rc


class FusedGRUPolicy:
    """GRUPolicy.forward + sample for inference on the GPU (networks.py:82-146).

    kernel=True (default) and the reference widths (gru 128, hidden 256, action_dim <= 16): one
    launch per step, lbsim_sac_actor_step; otherwise the GEMM form (hipBLASLt + lbsim_gru_gates +
    lbsim_sac_head).  Both draw the exploration noise from the same Philox counters.
    """

    def __init__(self, policy: GRUPolicy, seed: int = 0, kernel: bool = True):
        g = policy.gru
        self.p = policy
        # views of the module's parameters (the GEMM form follows in-place updates by itself)
        self.w_ih, self.b_ih = g.weight_ih_l0.detach(), g.bias_ih_l0.detach()
        self.w_hh, self.b_hh = g.weight_hh_l0.detach(), g.bias_hh_l0.detach()
        self.w1, self.b1 = policy.fc1.weight.detach(), policy.fc1.bias.detach()
        self.wh, self.bh = self._heads()
        self.seed = int(seed) & 0xFFFFFFFFFFFFFFFF
        self.step_no = 0
        self.step_dev = None
        self.kernel = None
        if (kernel and self.w_ih.is_cuda and policy.gru_dim == 128 and policy.hidden_dim == 256
                and policy.action_dim <= 16 and policy.state_dim <= 512):
            self.kernel = self._pack()
        self._watch = _ParamWatch([policy])

    def use_device_step(self) -> None:
        """Keep the Philox step counter on the device (lbsim_sac_actor_t.step_dev), advanced by a
        tiny kernel after each launch: a captured call replays with a new step each time, drawing
        exactly what the eager calls would.  Needs the one-launch kernel form."""
        if self.kernel is None:
            raise ValueError("use_device_step needs the lbsim_sac_actor_step kernel form")
        if self.step_dev is None:
            self.step_dev = torch.tensor([self.step_no & 0x7FFFFFFF], dtype=torch.int32,
                                         device=self.w_ih.device)
            self.kernel.step_dev = self.step_dev.data_ptr()

    def _heads(self):
        p = self.p
        return (torch.cat([p.fc_mean.weight, p.fc_logstd.weight]).detach().contiguous(),
                torch.cat([p.fc_mean.bias, p.fc_logstd.bias]).detach().contiguous())

    def _pack_tensors(self):
        return [pack_linear(self.w_ih), pack_linear(self.w_hh), self.b_ih.contiguous(),
                self.b_hh.contiguous(), pack_linear(self.w1), self.b1.contiguous(),
                pack_linear(self.wh), _pad_vec(self.bh, -(-2 * self.p.action_dim // 16) * 16)]

    def _pack(self):
        from . import _lib
        p = self.p
        self._packed = [t.clone() for t in self._pack_tensors()]  # own storage: stable pointers
        return _lib.SacActor(p.state_dim, p.gru_dim, p.hidden_dim, p.action_dim,
                             *[t.data_ptr() for t in self._packed], float(p.log_std_min),
                             float(p.log_std_max), float(p.action_scale), float(p.action_bias))

    @torch.no_grad()
    def sync_weights(self) -> None:
        """Re-read the module's weights into the concatenated heads and the packed buffers, in
        place (the kernel keeps its device pointers).  Called automatically before a launch when
        a parameter changed (optimizer step, load_state_dict)."""
        _copy_into((self.wh, self.bh), self._heads())
        if self.kernel is not None:
            _copy_into(self._packed, self._pack_tensors())

    @torch.no_grad()
    def __call__(self, state: torch.Tensor, hidden: torch.Tensor, deterministic: bool = False,
                 reset_mask: Optional[torch.Tensor] = None, inplace: bool = False):
        """state (B, I), hidden (B, H) -> action (B, A), hidden_new (B, H), log_std (B, A).

        reset_mask (B,) bool: envs whose hidden state starts from zeros (a new episode).
        inplace: hidden_new is `hidden` itself, updated in place."""
        from . import _lib
        B, A = state.shape[0], self.p.action_dim
        if self._watch.changed():
            self.sync_weights()
        lib, stream = _lib_and_stream(state.device)
        action = torch.empty((B, A), dtype=torch.float32, device=state.device)
        log_std = torch.empty_like(action)
        mask = None if reset_mask is None else reset_mask.contiguous()
        if self.kernel is not None:
            h = hidden if inplace else hidden.clone()
            x = state.contiguous()
            _lib.check(_timed(lambda: lib.lbsim_sac_actor_step(
                ctypes.byref(self.kernel), _ptr(x), _ptr(h), _ptr(mask), B, int(deterministic),
                self.seed, self.step_no & 0xFFFFFFFF, _ptr(action), _ptr(log_std), stream)))
            self.step_no += 1
            if self.step_dev is not None:
                self.step_dev.add_(1)
            return action, h, log_std
        h0 = hidden if mask is None else hidden * (~mask.bool()).unsqueeze(1).to(hidden.dtype)
        gi = torch.addmm(self.b_ih, state, self.w_ih.t())
        gh = torch.addmm(self.b_hh, h0, self.w_hh.t())
        h1 = torch.empty_like(hidden)
        _lib.check(lib.lbsim_gru_gates(_ptr(gi), _ptr(gh), _ptr(h0), _ptr(h1), B, h1.shape[1],
                                       stream))
        y = torch.addmm(self.bh, _linear_relu(h1, self.w1, self.b1), self.wh.t())
        _lib.check(lib.lbsim_sac_head(
            _ptr(y), B, A, float(self.p.log_std_min), float(self.p.log_std_max),
            float(self.p.action_scale), float(self.p.action_bias), int(deterministic), self.seed,
            self.step_no & 0xFFFFFFFF, _ptr(action), _ptr(log_std), stream))
        self.step_no += 1
        if inplace:
            hidden.copy_(h1)
            h1 = hidden
        return action, h1, log_std


class FusedQMIXPolicy:
    """problem-05 QMIXAgent.select_actions for every agent (qmix_agent.py:138-178) and
    QMixingNetwork.forward (mixing_network.py:78-117) in ONE launch per step
    (lbsim_qmix_policy_step): per tile of envs each agent's GRU + three linear layers,
    epsilon-greedy with Philox noise (counter (env, step, agent)), the chosen Q-values and the
    mixer on the global state.  Reference widths: gru 64, hidden 128, embed 32, hypernet 64."""

    @staticmethod
    def supported(agents, mixer: QMixer, n_actions: int) -> bool:
        a0 = agents[0]
        A, E, he = len(agents), mixer.mixing_embed_dim, mixer.hypernet_embed_dim
        return (all(a.gru_dim == 64 and a.hidden_dim == 128 and a.obs_dim == a0.obs_dim
                    for a in agents)
                and 1 <= n_actions <= 16 and A <= 16 and a0.obs_dim <= 512
                and mixer.state_dim <= 512 and E % 16 == 0 and he % 16 == 0
                and 3 * he + E <= 256 and A * E // 16 + E // 16 + 1 <= 16
                and A * E + E + 16 <= 3 * he and next(mixer.parameters()).is_cuda)

    def __init__(self, agents, mixer: QMixer, n_actions: int = 3, epsilon: float = 0.05,
                 seed: int = 0, servers_per_agent: int = 1):
        from . import _lib
        if not self.supported(agents, mixer, n_actions):
            raise ValueError("FusedQMIXPolicy: layer widths not built into lbsim_qmix_policy_step")
        self.A, self.n_actions, self.k = len(agents), n_actions, servers_per_agent
        self.H = agents[0].gru_dim
        self.agents, self.mixer = list(agents), mixer
        self._packed = [t.clone() for t in self._pack_tensors()]  # own storage: stable pointers
        m = mixer
        self.net = _lib.QmixPolicy(self.A, agents[0].obs_dim, self.H, agents[0].hidden_dim,
                                   n_actions, m.state_dim, m.mixing_embed_dim,
                                   m.hypernet_embed_dim, servers_per_agent, float(epsilon),
                                   *[t.data_ptr() for t in self._packed])
        self.seed = int(seed) & 0xFFFFFFFFFFFFFFFF
        self.step_no = 0
        self.step_dev = None
        self._watch = _ParamWatch(self.agents + [mixer])

    def use_device_step(self) -> None:
        """Keep the Philox step counter on the device (lbsim_qmix_policy_t.step_dev), advanced
        by a tiny kernel after each launch: a captured call replays with a new step each time,
        drawing exactly what the eager calls would."""
        if self.step_dev is None:
            dev = self._packed[0].device
            self.step_dev = torch.tensor([self.step_no & 0x7FFFFFFF], dtype=torch.int32, device=dev)
            self.net.step_dev = self.step_dev.data_ptr()

    def _pack_tensors(self):
        agents, m = self.agents, self.mixer
        cat = lambda f: torch.cat([f(a).reshape(-1) for a in agents]).contiguous()  # noqa: E731
        first = [m.hyper_w1[0], m.hyper_w2[0], m.hyper_b2[0], m.hyper_b1[0]]
        return [
            cat(lambda a: pack_linear(a.gru.weight_ih_l0)),
            cat(lambda a: pack_linear(a.gru.weight_hh_l0)),
            cat(lambda a: a.gru.bias_ih_l0.detach()), cat(lambda a: a.gru.bias_hh_l0.detach()),
            cat(lambda a: pack_linear(a.fc1.weight)), cat(lambda a: a.fc1.bias.detach()),
            cat(lambda a: pack_linear(a.fc2.weight)), cat(lambda a: a.fc2.bias.detach()),
            cat(lambda a: pack_linear(a.fc3.weight, 16)), cat(lambda a: _pad_vec(a.fc3.bias, 16)),
            pack_linear(torch.cat([l.weight for l in first])),
            torch.cat([l.bias for l in first]).detach().contiguous(),
            pack_linear(m.hyper_w1[2].weight), m.hyper_w1[2].bias.detach().contiguous(),
            pack_linear(m.hyper_w2[2].weight), m.hyper_w2[2].bias.detach().contiguous(),
            pack_linear(m.hyper_b2[2].weight, 16), _pad_vec(m.hyper_b2[2].bias, 16)]

    @torch.no_grad()
    def sync_weights(self) -> None:
        """Repack the agents' and mixer's weights in place (automatic when they change)."""
        _copy_into(self._packed, self._pack_tensors())

    @torch.no_grad()
    def __call__(self, obs: torch.Tensor, hidden: torch.Tensor, state: torch.Tensor,
                 reset_mask: Optional[torch.Tensor] = None, q_values: bool = False):
        """obs (B, A, I), hidden (B, A, H) f32 contiguous, updated in place, state (B, Ds) ->
        actions (B, A) int64, server_actions (B, A k) int32, q_tot (B, 1), q (B, A, n) or None."""
        from . import _lib
        B, dev = obs.shape[0], obs.device
        if not (hidden.is_contiguous() and hidden.shape == (B, self.A, self.H)):
            raise ValueError("hidden must be a contiguous (B, A, gru) tensor")
        if self._watch.changed():
            self.sync_weights()
        lib, stream = _lib_and_stream(dev)
        acts = torch.empty((B, self.A), dtype=torch.int64, device=dev)
        sacts = torch.empty((B, self.A * self.k), dtype=torch.int32, device=dev)
        q_tot = torch.empty((B, 1), dtype=torch.float32, device=dev)
        q = torch.empty((B, self.A, self.n_actions), dtype=torch.float32, device=dev) \
            if q_values else None
        o, s = obs.contiguous(), state.contiguous()
        mask = None if reset_mask is None else reset_mask.contiguous()
        _lib.check(_timed(lambda: lib.lbsim_qmix_policy_step(
            ctypes.byref(self.net), _ptr(o), _ptr(hidden), _ptr(mask), _ptr(s), B, self.seed,
            self.step_no & 0xFFFFFFFF, _ptr(acts), _ptr(sacts), _ptr(q), None, _ptr(q_tot),
            stream)))
        self.step_no += 1
        if self.step_dev is not None:
            self.step_dev.add_(1)
        return acts, sacts, q_tot, q


class FusedAgentQNets:
    """A problem-05 AgentQNetworks (one per agent) evaluated together: per layer one batched GEMM
    over the stacked agent weights, GRU gates in lbsim_gru_gates."""

    def __init__(self, agents):
        self.agents = list(agents)
        self.A = len(agents)
        self.H = agents[0].gru_dim
        (self.w_ih, self.b_ih, self.w_hh, self.b_hh, self.w1, self.b1, self.w2, self.b2,
         self.w3, self.b3) = self._stacked()
        self._watch = _ParamWatch(self.agents)

    def _stacked(self):
        st = lambda f: torch.stack([f(a).detach() for a in self.agents]).contiguous()  # noqa: E731
        return (st(lambda a: a.gru.weight_ih_l0.t()),  # (A, I, 3H)
                st(lambda a: a.gru.bias_ih_l0).unsqueeze(1),
                st(lambda a: a.gru.weight_hh_l0.t()), st(lambda a: a.gru.bias_hh_l0).unsqueeze(1),
                st(lambda a: a.fc1.weight.t()), st(lambda a: a.fc1.bias).unsqueeze(1),
                st(lambda a: a.fc2.weight.t()), st(lambda a: a.fc2.bias).unsqueeze(1),
                st(lambda a: a.fc3.weight.t()), st(lambda a: a.fc3.bias).unsqueeze(1))

    @torch.no_grad()
    def sync_weights(self) -> None:
        _copy_into((self.w_ih, self.b_ih, self.w_hh, self.b_hh, self.w1, self.b1, self.w2,
                    self.b2, self.w3, self.b3), self._stacked())

    @torch.no_grad()
    def __call__(self, obs: torch.Tensor, hidden: torch.Tensor):
        """obs (A, B, I), hidden (A, B, H) -> q (A, B, n_actions), hidden_new (A, B, H)."""
        from . import _lib
        A, B, H = obs.shape[0], obs.shape[1], self.H
        if self._watch.changed():
            self.sync_weights()
        lib, stream = _lib_and_stream(obs.device)
        gi = torch.baddbmm(self.b_ih, obs, self.w_ih)
        gh = torch.baddbmm(self.b_hh, hidden, self.w_hh)
        h1 = torch.empty_like(hidden)
        _lib.check(lib.lbsim_gru_gates(_ptr(gi), _ptr(gh), _ptr(hidden), _ptr(h1), A * B, H,
                                       stream))
        x = torch.relu_(torch.baddbmm(self.b1, h1, self.w1))
        x = torch.relu_(torch.baddbmm(self.b2, x, self.w2))
        return torch.baddbmm(self.b3, x, self.w3), h1


class FusedQMixer:
    """QMixer.forward: the four hypernetwork first layers as one GEMM on the state, the second
    layers as GEMMs, then abs / bmm / elu / bmm per env in lbsim_qmix_tail."""

    def __init__(self, mixer: QMixer):
        m = mixer
        self.m = m
        self.A, self.E = m.num_agents, m.mixing_embed_dim
        self.w0, self.b0 = self._firsts()
        he = m.hypernet_embed_dim
        self.cuts = [he, he + self.E, 2 * he + self.E, 3 * he + self.E]
        self.w1, self.bw1 = m.hyper_w1[2].weight.detach(), m.hyper_w1[2].bias.detach()
        self.w2, self.bw2 = m.hyper_w2[2].weight.detach(), m.hyper_w2[2].bias.detach()
        self.wb2, self.bb2 = m.hyper_b2[2].weight.detach(), m.hyper_b2[2].bias.detach()
        self._watch = _ParamWatch([m])

    def _firsts(self):
        m = self.m
        firsts = [m.hyper_w1[0], m.hyper_b1[0], m.hyper_w2[0], m.hyper_b2[0]]
        return (torch.cat([l.weight for l in firsts]).detach().contiguous(),
                torch.cat([l.bias for l in firsts]).detach().contiguous())

    @torch.no_grad()
    def sync_weights(self) -> None:
        _copy_into((self.w0, self.b0), self._firsts())  # the other layers are views

    @torch.no_grad()
    def __call__(self, agent_qs: torch.Tensor, state: torch.Tensor) -> torch.Tensor:
        from . import _lib
        B = agent_qs.shape[0]
        if self._watch.changed():
            self.sync_weights()
        lib, stream = _lib_and_stream(state.device)
        z = torch.addmm(self.b0, state, self.w0.t())  # [hw1 | b1 | hw2 | hb2] pre-activation
        c0, c1, c2, c3 = self.cuts
        b1 = z[:, c0:c1]                               # hyper_b1 has no ReLU
        w1 = torch.addmm(self.bw1, torch.relu(z[:, :c0]), self.w1.t())
        w2 = torch.addmm(self.bw2, torch.relu(z[:, c1:c2]), self.w2.t())
        b2 = torch.addmm(self.bb2, torch.relu(z[:, c2:c3]), self.wb2.t())
        q_tot = torch.empty((B, 1), dtype=torch.float32, device=state.device)
        qs = agent_qs.contiguous()
        _lib.check(lib.lbsim_qmix_tail(_ptr(qs), _ptr(w1), w1.stride(0), _ptr(b1), b1.stride(0),
                                       _ptr(w2), w2.stride(0), _ptr(b2), b2.stride(0), B, self.A,
                                       self.E, _ptr(q_tot), stream))
        return q_tot
