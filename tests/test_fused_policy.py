"""One-kernel policy inference (csrc/lbsim_fused.h: lbsim_sac_actor_step, lbsim_qmix_policy_step)
against the torch modules of the reference networks (problem-04 networks.py, problem-05
agent_network.py / mixing_network.py; the modules themselves are pinned to the reference outputs
in tests/test_policies.py).  fp32, tolerance 1e-5 (abs + rel).  CPU part: the packed-weight
layout the kernels assume and the ABI's argument checks."""
import ctypes
import os

import numpy as np
import pytest

torch = pytest.importorskip("torch")

from marllb_amd import _lib  # noqa: E402
from marllb_amd.policies import (AgentQNet, FusedGRUPolicy, FusedQMIXPolicy, GRUPolicy,  # noqa: E402
                                 QMixer, load_prefixed, pack_linear)

TOL = dict(rtol=1e-5, atol=1e-5)


def close(a, b, **kw):
    np.testing.assert_allclose(a.detach().cpu().numpy(), b.detach().cpu().numpy(), **(kw or TOL))


def test_pack_linear_is_the_mfma_fragment_order():
    """Replay what the kernel does with a packed weight: lane l of k-step s of block kb multiplies
    X[row][16 kb + 4 (l >> 4) + s] by P[nt][kb][l][s] into output column 16 nt + (l & 15)."""
    g = torch.Generator().manual_seed(0)
    W = torch.randn(40, 37, generator=g)  # ragged N and K: padded to 48 x 48
    X = torch.randn(5, 37, generator=g, dtype=torch.float64)
    P = pack_linear(W).double().view(3, 3, 64, 4)
    Xp = torch.zeros(5, 48, dtype=torch.float64)
    Xp[:, :37] = X
    Y = torch.zeros(5, 48, dtype=torch.float64)
    lane = torch.arange(64)
    for nt in range(3):
        for kb in range(3):
            for s in range(4):
                k = 16 * kb + 4 * (lane >> 4) + s  # (64,)
                contrib = Xp[:, k] * P[nt, kb, :, s]  # (5, 64)
                Y[:, 16 * nt:16 * nt + 16] += contrib.view(5, 4, 16).sum(1)
    torch.testing.assert_close(Y[:, :40], X @ W.double().T)
    assert torch.all(Y[:, 40:] == 0)
    assert pack_linear(W, 64).numel() == 64 * 48


def test_fused_abi_layout_and_argument_checks():
    """Struct sizes match the header; NULL / unsupported widths are rejected before any launch."""
    lib = _lib.load()
    assert lib.lbsim_sac_actor_size() == ctypes.sizeof(_lib.SacActor)
    assert lib.lbsim_qmix_policy_size() == ctypes.sizeof(_lib.QmixPolicy)

    def sac(net, B):
        return lib.lbsim_sac_actor_step(ctypes.byref(net), None, None, None, B, 1, 0, 0, None,
                                        None, None)

    assert lib.lbsim_sac_actor_step(None, None, None, None, 4, 1, 0, 0, None, None, None) \
        == _lib.EINVAL
    assert sac(_lib.SacActor(88, 128, 256, 8), 0) == _lib.OK       # nothing to do
    assert sac(_lib.SacActor(88, 128, 256, 8), 4) == _lib.EINVAL   # NULL buffers
    assert sac(_lib.SacActor(88, 128, 256, 17), 4) == _lib.EINVAL  # action_dim > 16
    assert sac(_lib.SacActor(88, 64, 256, 8), 4) == _lib.ENOTSUP   # width not built

    def qmix(net, B):
        return lib.lbsim_qmix_policy_step(ctypes.byref(net), None, None, None, None, B, 0, 0,
                                          None, None, None, None, None, None)

    ok = (4, 128, 64, 128, 3, 74, 32, 64, 4, 0.05)
    assert qmix(_lib.QmixPolicy(*ok), 0) == _lib.OK
    assert qmix(_lib.QmixPolicy(*ok), 4) == _lib.EINVAL
    assert qmix(_lib.QmixPolicy(*ok[:9], 1.5), 4) == _lib.EINVAL                 # epsilon > 1
    assert qmix(_lib.QmixPolicy(4, 128, 64, 96, 3, 74, 32, 64, 4, 0.05), 4) == _lib.ENOTSUP
    assert qmix(_lib.QmixPolicy(8, 128, 64, 128, 3, 74, 32, 64, 4, 0.05), 4) == _lib.ENOTSUP


@pytest.fixture(scope="module")
def g(golden_dir):
    return np.load(os.path.join(golden_dir, "nets.npz"))


@pytest.mark.gpu
def test_sac_actor_kernel_matches_module(g):
    dev = "cuda:0"
    pol = load_prefixed(GRUPolicy(88, 8, 256, 128), g, "policy").to(dev)
    t = lambda k: torch.from_numpy(g[k]).to(dev)  # noqa: E731
    x, h = t("policy_x"), t("policy_h")[0].contiguous()
    f = FusedGRUPolicy(pol)
    assert f.kernel is not None
    act, h1, ls = f(x, h, deterministic=True)
    np.testing.assert_allclose(act.cpu().numpy(), g["policy_det_action"], **TOL)
    np.testing.assert_allclose(h1.cpu().numpy(), g["policy_h1"][0], **TOL)
    np.testing.assert_allclose(ls.cpu().numpy(), g["policy_log_std"], **TOL)
    assert h1.data_ptr() != h.data_ptr()
    np.testing.assert_array_equal(h.cpu().numpy(), g["policy_h"][0])  # input untouched
    # a ragged batch (1000: not a multiple of the 16, 32 or 64-env tile) with reset rows, hidden
    # updated in place
    gen = torch.Generator(device=dev).manual_seed(1)
    B = 1000
    xb = torch.randn(B, 88, device=dev, generator=gen) * 3
    hb = torch.randn(B, 128, device=dev, generator=gen) * 0.5
    mask = torch.rand(B, device=dev, generator=gen) < 0.3
    with torch.no_grad():
        mean, log_std, rh = pol(xb, (hb * (~mask).unsqueeze(1)).unsqueeze(0))
    hk = hb.clone()
    a, hh, lsk = FusedGRUPolicy(pol)(xb, hk, deterministic=True, reset_mask=mask, inplace=True)
    assert hh.data_ptr() == hk.data_ptr()
    close(a, torch.tanh(mean))
    close(hh, rh[0])
    close(lsk, log_std)
    # stochastic: the kernel and the GEMM form draw the same Philox noise
    ak, hk2, _ = FusedGRUPolicy(pol, seed=7)(xb, hb, reset_mask=mask)
    ag, hg2, _ = FusedGRUPolicy(pol, seed=7, kernel=False)(xb, hb, reset_mask=mask)
    assert FusedGRUPolicy(pol, kernel=False).kernel is None
    close(hk2, hg2)
    close(ak, ag, rtol=1e-4, atol=5e-5)
    assert bool((ak.abs() <= 1).all()) and not torch.equal(ak, a)


@pytest.mark.gpu
def test_qmix_policy_kernel_matches_modules(g):
    dev = "cuda:0"
    agents = [load_prefixed(AgentQNet(128, 3, 128, 64), g, "agentq").to(dev) for _ in range(4)]
    with torch.no_grad():
        for k, a in enumerate(agents[1:], 1):
            for p in a.parameters():
                p.mul_(1.0 + 0.1 * k)
    mix = load_prefixed(QMixer(4, 74, 32, 64), g, "mixer").to(dev)
    gen = torch.Generator(device=dev).manual_seed(3)
    B = 300  # ragged: not a multiple of the tile
    obs = torch.randn(B, 4, 128, device=dev, generator=gen)
    hid = torch.randn(B, 4, 64, device=dev, generator=gen) * 0.5
    state = torch.randn(B, 74, device=dev, generator=gen)
    mask = torch.zeros(B, dtype=torch.bool, device=dev)
    mask[::7] = True
    pol = FusedQMIXPolicy(agents, mix, 3, epsilon=0.0, seed=1, servers_per_agent=4)
    hk = hid.clone()
    acts, sacts, q_tot, q = pol(obs, hk, state, reset_mask=mask, q_values=True)
    h0 = hid * (~mask).view(B, 1, 1).float()
    with torch.no_grad():
        for a, net in enumerate(agents):
            rq, rh = net(obs[:, a], h0[:, a].unsqueeze(0).contiguous())
            close(q[:, a], rq)
            close(hk[:, a], rh[0])
            top2 = rq.topk(2, dim=1).values
            clear = (top2[:, 0] - top2[:, 1]) > 1e-4  # greedy = argmax where it is well defined
            assert torch.equal(acts[clear, a], rq.argmax(1)[clear])
        chosen = q.gather(2, acts.unsqueeze(2)).squeeze(2)
        close(q_tot, mix(chosen, state))
    assert torch.equal(sacts.long(), acts.repeat_interleave(4, dim=1))
    # epsilon = 1: uniform actions; Q_tot is still the mixer of the chosen Q-values
    pol1 = FusedQMIXPolicy(agents, mix, 3, epsilon=1.0, seed=2, servers_per_agent=4)
    a1, _, qt1, q1 = pol1(obs, hid.clone(), state, q_values=True)
    counts = torch.bincount(a1.flatten(), minlength=3)
    assert counts.numel() == 3 and int(counts.min()) > 0.25 * a1.numel()
    with torch.no_grad():
        close(qt1, mix(q1.gather(2, a1.unsqueeze(2)).squeeze(2), state))
    # the same seed and step reproduce; the next step draws new noise
    pol2 = FusedQMIXPolicy(agents, mix, 3, epsilon=1.0, seed=2, servers_per_agent=4)
    a2, _, _, _ = pol2(obs, hid.clone(), state)
    a3, _, _, _ = pol2(obs, hid.clone(), state)
    assert torch.equal(a1, a2) and not torch.equal(a2, a3)


@pytest.mark.gpu
def test_qmix_policy_kernel_wide_obs_matches_modules():
    """configs[4] literal: 4 agents x 16 servers (agent obs 4 k + 7 S = 512, state 4 S + 10 =
    266): the pair kernel's LDS is too full there to also hold the mixer's state rows at the
    start, so the mixer stages them itself -- same results as the torch modules."""
    dev = "cuda:0"
    torch.manual_seed(11)
    agents = [AgentQNet(512, 3, 128, 64).to(dev) for _ in range(4)]
    mix = QMixer(4, 266, 32, 64).to(dev)
    gen = torch.Generator(device=dev).manual_seed(4)
    B = 70
    obs = torch.randn(B, 4, 512, device=dev, generator=gen) * 0.3
    hid = torch.randn(B, 4, 64, device=dev, generator=gen) * 0.5
    state = torch.randn(B, 266, device=dev, generator=gen)
    pol = FusedQMIXPolicy(agents, mix, 3, epsilon=0.0, seed=1, servers_per_agent=16)
    hk = hid.clone()
    acts, _, q_tot, q = pol(obs, hk, state, q_values=True)
    with torch.no_grad():
        for a, net in enumerate(agents):
            rq, rh = net(obs[:, a], hid[:, a].unsqueeze(0).contiguous())
            close(q[:, a], rq)
            close(hk[:, a], rh[0])
        close(q_tot, mix(q.gather(2, acts.unsqueeze(2)).squeeze(2), state))


@pytest.mark.gpu
@pytest.mark.parametrize("env", [{"LBSIM_QMIX_KERNEL": "wave"},
                                 {"LBSIM_QMIX_KERNEL": "tile"},
                                 {"LBSIM_FUSED_MT": "1"},
                                 {"LBSIM_FUSED_MT": "2", "LBSIM_QMIX_KERNEL": "tile"},
                                 {"LBSIM_FUSED_MT": "4", "LBSIM_QMIX_KERNEL": "tile"}])
def test_other_tile_forms_match_modules(env):
    """The one-wave-per-agent and layer-split QMIX kernels, the 16 / 32 / 64-env tiles (SAC's
    default is 32 since round 6, the QMIX tile kernel's 16; selected once per process by the
    environment, so checked in a child process) pass the same parity tests as the defaults."""
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    r = subprocess.run([sys.executable, "-m", "pytest", "-q", "-x", "-m", "gpu", "-p",
                        "no:cacheprovider", os.path.join(root, "tests", "test_fused_policy.py"),
                        "-k", "matches_module"],
                       cwd=root, env={**os.environ, **env}, capture_output=True, text=True,
                       timeout=300)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]


@pytest.mark.gpu
def test_fused_forms_follow_weight_updates(g):
    """An optimizer step or load_state_dict on the torch modules reaches the packed copies the
    fused kernels read (version-counter check before each launch; sync_weights() by hand)."""
    dev = "cuda:0"
    gen = torch.Generator(device=dev).manual_seed(5)
    x = torch.randn(64, 88, device=dev, generator=gen) * 0.1
    h = torch.randn(64, 128, device=dev, generator=gen) * 0.1
    for kernel in (True, False):
        pol = load_prefixed(GRUPolicy(88, 8, 256, 128), g, "policy").to(dev)
        f = FusedGRUPolicy(pol, kernel=kernel)
        a0, _, _ = f(x, h, deterministic=True)
        opt = torch.optim.SGD(pol.parameters(), lr=1e-2)
        mean, _, _ = pol(x, h.unsqueeze(0))
        mean.sum().backward()
        opt.step()
        opt.zero_grad()
        a1, h1, ls1 = f(x, h, deterministic=True)
        with torch.no_grad():
            m1, l1, rh1 = pol(x, h.unsqueeze(0))
        assert not torch.equal(a0, a1)
        close(a1, torch.tanh(m1))
        close(h1, rh1[0])
        close(ls1, l1)
    agents = [load_prefixed(AgentQNet(128, 3, 128, 64), g, "agentq").to(dev) for _ in range(4)]
    mix = load_prefixed(QMixer(4, 74, 32, 64), g, "mixer").to(dev)
    B = 48
    obs = torch.randn(B, 4, 128, device=dev, generator=gen)
    hid = torch.randn(B, 4, 64, device=dev, generator=gen) * 0.5
    state = torch.randn(B, 74, device=dev, generator=gen)
    qp = FusedQMIXPolicy(agents, mix, 3, epsilon=0.0, seed=1, servers_per_agent=4)
    _, _, qt0, q0 = qp(obs, hid.clone(), state, q_values=True)
    new = QMixer(4, 74, 32, 64).to(dev)
    mix.load_state_dict(new.state_dict())
    with torch.no_grad():
        agents[2].fc3.weight.mul_(-2.0)
    acts, _, qt1, q1 = qp(obs, hid.clone(), state, q_values=True)
    with torch.no_grad():
        rq, _ = agents[2](obs[:, 2], hid[:, 2].unsqueeze(0).contiguous())
        close(q1[:, 2], rq)
        close(qt1, mix(q1.gather(2, acts.unsqueeze(2)).squeeze(2), state))
    assert not torch.allclose(qt0, qt1)


@pytest.mark.gpu
def test_fused_kernels_full_shard_vs_modules(g):
    """Full per-GPU shards of configs[3] and configs[4] (SAC-GRU 65536 x 8; QMIX 8192 envs x 4
    agents over 16 servers) against the torch modules, every row, within 1e-5 (greedy actions;
    argmax compared where the top two Q-values are 1e-4 apart)."""
    dev = "cuda:0"
    gen = torch.Generator(device=dev).manual_seed(11)
    pol = load_prefixed(GRUPolicy(88, 8, 256, 128), g, "policy").to(dev)
    B = 65536
    x = torch.randn(B, 88, device=dev, generator=gen) * 2
    h = torch.randn(B, 128, device=dev, generator=gen) * 0.5
    mask = torch.rand(B, device=dev, generator=gen) < 0.1
    with torch.no_grad():
        mean, log_std, rh = pol(x, (h * (~mask).unsqueeze(1)).unsqueeze(0))
    a, h1, ls = FusedGRUPolicy(pol)(x, h, deterministic=True, reset_mask=mask)
    close(a, torch.tanh(mean))
    close(h1, rh[0])
    close(ls, log_std)
    del x, h, mean, log_std, rh, a, h1, ls
    agents = [load_prefixed(AgentQNet(128, 3, 128, 64), g, "agentq").to(dev) for _ in range(4)]
    with torch.no_grad():
        for k, ag in enumerate(agents[1:], 1):
            for p in ag.parameters():
                p.mul_(1.0 - 0.07 * k)
    mix = load_prefixed(QMixer(4, 74, 32, 64), g, "mixer").to(dev)
    B = 8192
    obs = torch.randn(B, 4, 128, device=dev, generator=gen)
    hid = torch.randn(B, 4, 64, device=dev, generator=gen) * 0.5
    state = torch.randn(B, 74, device=dev, generator=gen)
    qp = FusedQMIXPolicy(agents, mix, 3, epsilon=0.0, seed=3, servers_per_agent=4)
    hk = hid.clone()
    acts, _, q_tot, q = qp(obs, hk, state, q_values=True)
    with torch.no_grad():
        for ai, net in enumerate(agents):
            rq, rh = net(obs[:, ai], hid[:, ai].unsqueeze(0).contiguous())
            close(q[:, ai], rq)
            close(hk[:, ai], rh[0])
            top2 = rq.topk(2, dim=1).values
            clear = (top2[:, 0] - top2[:, 1]) > 1e-4
            assert torch.equal(acts[clear, ai], rq.argmax(1)[clear])
        close(q_tot, mix(q.gather(2, acts.unsqueeze(2)).squeeze(2), state))
