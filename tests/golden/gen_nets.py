#!/usr/bin/env python3
"""Golden vectors for the on-GPU policy / mixer networks.

Imports the reference modules in place (this container only; they never travel) and records
their OUTPUTS on seeded weights and inputs as data:
  PolicyNetwork.forward / sample(mean)   simulation-mode/problem-04-sac-gru/src/networks.py:19-151
  AgentQNetwork.forward                  simulation-mode/problem-05-qmix/src/agent_network.py:13-92
  QMixingNetwork.forward                 simulation-mode/problem-05-qmix/src/mixing_network.py:15-117

    python tests/golden/gen_nets.py [--reference /root/reference]
-> tests/golden/nets.npz: for each net, its state_dict tensors (prefixed), inputs and outputs.
"""
import argparse
import importlib.util
import os

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))


def load_module(path, name):
    spec = importlib.util.spec_from_file_location(name, path)
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reference", default="/root/reference")
    a = ap.parse_args()
    sm = os.path.join(a.reference, "simulation-mode")
    nets = load_module(os.path.join(sm, "problem-04-sac-gru/src/networks.py"), "ref_networks")
    agent = load_module(os.path.join(sm, "problem-05-qmix/src/agent_network.py"), "ref_agent_net")
    mixer = load_module(os.path.join(sm, "problem-05-qmix/src/mixing_network.py"), "ref_mixer")
    torch.manual_seed(20260109)
    out = {}

    def put(prefix, module):
        for k, v in module.state_dict().items():
            out[f"{prefix}.{k}"] = v.detach().cpu().numpy()

    # ---- SAC-GRU actor at configs[3]: S = 8, state = S * 11 = 88, gru 128, hidden 256
    S, B = 8, 64
    pol = nets.PolicyNetwork(state_dim=S * 11, action_dim=S, hidden_dim=256, gru_dim=128)
    with torch.no_grad():  # non-zero biases so every term is exercised
        for p in pol.parameters():
            if p.dim() == 1:
                p.uniform_(-0.1, 0.1)
    put("policy", pol)
    x = torch.randn(B, S * 11) * 3.0
    h = torch.randn(1, B, 128) * 0.5
    with torch.no_grad():
        mean, log_std, h1 = pol(x, h)
        _, _, det, _ = pol.sample(x, h)
    out.update({"policy_x": x.numpy(), "policy_h": h.numpy(), "policy_mean": mean.numpy(),
                "policy_log_std": log_std.numpy(), "policy_h1": h1.numpy(),
                "policy_det_action": det.numpy()})

    # ---- QMIX agent Q-network: per-agent obs as the problem-05 wrapper emits it (128-dim at
    #      4 agents x 4 servers), 3 actions
    A, k = 4, 4
    obs_dim = 4 * k + (A * k * 11 - A * k * 4)
    q = agent.AgentQNetwork(obs_dim=obs_dim, action_dim=3, hidden_dim=128, gru_dim=64)
    with torch.no_grad():
        for p in q.parameters():
            if p.dim() == 1:
                p.uniform_(-0.1, 0.1)
    put("agentq", q)
    o = torch.randn(B, obs_dim)
    hq = torch.randn(1, B, 64) * 0.5
    with torch.no_grad():
        qv, hq1 = q(o, hq)
    out.update({"agentq_obs": o.numpy(), "agentq_h": hq.numpy(), "agentq_q": qv.numpy(),
                "agentq_h1": hq1.numpy()})

    # ---- QMIX mixer: 4 agents, state_dim = 4 * 16 + 10 = 74 (the wrapper's get_state)
    mix = mixer.QMixingNetwork(num_agents=A, state_dim=A * k * 4 + 10, mixing_embed_dim=32,
                               hypernet_embed_dim=64)
    put("mixer", mix)
    qs = torch.randn(B, A)
    st = torch.randn(B, A * k * 4 + 10)
    with torch.no_grad():
        qtot = mix(qs, st)
    out.update({"mixer_qs": qs.numpy(), "mixer_state": st.numpy(), "mixer_qtot": qtot.numpy()})

    np.savez_compressed(os.path.join(HERE, "nets.npz"), **out)
    print(f"wrote nets.npz ({len(out)} arrays)")


if __name__ == "__main__":
    main()
