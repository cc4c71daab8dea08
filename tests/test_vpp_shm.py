"""The VPP shared-memory bridge (marllb_amd/vpp_shm.py) against the reference's own agent side.

tests/golden/vpp_shm.npz comes from src/lb/shm_proxy.py imported in place (gen_vpp_shm.py): its
Shm_Manager's field offsets, the frames it reads (written with its own offsets and struct formats,
as VPP's stats.c does), the features its process_reservoir computes from them, and the msg_in
bytes its register_as_weights / register_as_alias write.

CPU: layout offsets, byte-exact frame publication (stats.c order) and msg_in packing, the ring
walks of both sides, and the oracle's restatement of process_reservoir.  GPU: the features
kernel on those frames (1e-5, in practice <= 1 ulp: only the f64 pow differs) and the simulator
as a live VPP LB (lbsim_vpp_export) read back by the agent side.
"""
import os
from unittest import mock

import numpy as np
import pytest

from marllb_amd import vpp_shm as vs

CASES = ("seven", "sparse", "wrap")


@pytest.fixture(scope="module")
def gold(golden_dir):
    return np.load(os.path.join(golden_dir, "vpp_shm.npz"))


@pytest.fixture
def region(tmp_path):
    # /dev/shm when present (the reference's location), else a tmp file: same bytes either way
    d = "/dev/shm" if os.path.isdir("/dev/shm") else str(tmp_path)
    path = os.path.join(d, f"lbsim_test_vpp_{os.getpid()}_{np.random.randint(1 << 30)}")
    shm = vs.VipShm.create(path=path)
    yield shm
    shm.close()
    shm.unlink()


def test_layout_matches_reference(gold):
    names = [str(n) for n in gold["layout_names"]]
    assert names == [n for n, _, _ in vs.LAYOUT]
    for (start, size, count), (name, dt, n) in zip(gold["layout"], vs.LAYOUT):
        assert (vs.OFFSETS[name], dt.itemsize, n) == (start, size, count), name
    assert [str(f) for f in gold["feature_as_all"]] == vs.FEATURE_AS_ALL


def _publish_case(dp, gold, name):
    """Frames of one fixture case published as VPP would (older frames: other ts / header)."""
    active, seqs = list(gold[f"{name}_active"]), list(gold[f"{name}_seqs"])
    ts, nflow = float(gold[f"{name}_ts"]), gold[f"{name}_nflow"]
    res = np.zeros((64, 2, 128, 2), np.float32)
    res[active] = gold[f"{name}_res"]
    dp.shm.res_as[:] = res.reshape(-1).view(vs.RESERVOIR_AS)
    dp.shm.msg_out_cache["body"][0] = [(a, int(nflow[a])) for a in range(64)]
    hdr = vs.header_from_active(active)
    for k, sid in enumerate(seqs):
        dp.id_out = sid - 1  # the fixture skips ids (VPP's counter is private to the plugin)
        last = k == len(seqs) - 1
        dp.shm.msg_out_cache["b_header"][0] = hdr if last else hdr ^ 1
        assert dp.publish(np.float32(ts if last else ts - 0.2 * (len(seqs) - 1 - k))) == sid
    return res


def test_frames_byte_exact_and_agent_ring_walk(gold, region):
    """VppDataPlane.publish writes the frames VPP writes (the reference read them back); the
    agent's walk finds the newest sequence id and its active list, as Shm_Manager did."""
    dp = vs.VppDataPlane(region)
    mgr = vs.ShmManager(shm=region, device="cpu")
    assert region.n_as[0] == 64
    for name in CASES:
        res = _publish_case(dp, gold, name)
        ring = np.frombuffer(region.msg_out_frames.tobytes(), np.uint8)
        np.testing.assert_array_equal(ring, gold[f"{name}_ring"], err_msg=name)
        assert region.res_as.tobytes() == res.tobytes()
        mgr.id_out = int(gold[f"{name}_seqs"][0]) - 1
        assert mgr.get_latest_sid_out() == int(gold[f"{name}_id_out"])
        fid = mgr.id_out & vs.SHM_FRAME_MASK
        assert mgr.get_active_as(fid) == list(gold[f"{name}_active_got"])
        assert mgr.get_field_from_frame(fid, "ts") == float(gold[f"{name}_ts"])


def test_msg_in_bytes_match_register_as_weights(gold, region, oracle_mod):
    """register_as_weights's bytes (shm_proxy.py:635-669) with the fixture's fixed time.time():
    scores, gen_alias of the weights > 0 scattered to their ASes (the oracle's gen_alias here;
    the GPU test runs the product's lbsim_alias_tables), id last."""
    mgr = vs.ShmManager(shm=region, device="cpu")
    for w, seq, want in zip(gold["weights_cases"], gold["weights_seqs"], gold["msg_in_weights"]):
        table = [(1.0, 0)] * 64
        ids = [i for i, x in enumerate(w) if x > 0]
        if ids:
            odd, ali = oracle_mod.gen_alias(np.asarray(w[ids], np.float32))
            for k, a in enumerate(ids):
                table[a] = (float(odd[k]), int(ali[k]))
        with mock.patch.object(vs.time, "time", return_value=float(gold["fixed_time"])):
            mgr._write_in(int(seq), w, table)
        got = np.frombuffer(region.msg_in_frames[int(seq) & 3].tobytes(), np.uint8)
        np.testing.assert_array_equal(got, want, err_msg=str(seq))


def test_msg_in_alias_bytes_and_vpp_pickup(gold, region):
    """register_as_alias bytes; then the VPP side's walk of the agent's ring (stats.c:159-180)
    copies the newest frame (id 40) into msg_in_cache, once."""
    mgr = vs.ShmManager(shm=region, device="cpu")
    tab = [(float(o), int(a)) for o, a in gold["alias_table"]]
    with mock.patch.object(vs.time, "time", return_value=float(gold["fixed_time"])):
        mgr.register_as_alias(40, tab)
    np.testing.assert_array_equal(np.frombuffer(region.msg_in_frames[0].tobytes(), np.uint8),
                                  gold["msg_in_alias"])
    region.msg_in_frames[:] = gold["msg_in_ring"].view(vs.MSG_IN)
    dp = vs.VppDataPlane(region)
    assert dp.pull_frame_in()
    assert int(region.msg_in_cache["id"][0]) == 40
    np.testing.assert_array_equal(np.frombuffer(region.msg_in_cache.tobytes(), np.uint8),
                                  gold["msg_in_alias"])
    assert not dp.pull_frame_in()  # nothing newer


def test_oracle_process_reservoir_matches_reference(gold, oracle_mod):
    """The oracle restatement (oracle_vpp_features) equals the reference's features up to the
    last bit of the f64 pow (numpy's vs glibc's): <= 2e-16 relative."""
    for name in CASES:
        act = gold[f"{name}_active"]
        res = gold[f"{name}_res"].reshape(-1, 128, 2)
        o = oracle_mod.vpp_features(res, np.array([gold[f"{name}_ts"]]), res_per_ts=10 ** 9)
        ref = gold[f"{name}_feature_as"][act][:, 1:].reshape(-1, 5)
        np.testing.assert_allclose(o, ref, rtol=4e-16, atol=0, err_msg=name)
        # every column but the two decayed ones is bit-exact
        np.testing.assert_array_equal(o[:, [0, 1, 2]], ref[:, [0, 1, 2]])


# ---------------------------------------------------------------------------------------- GPU
@pytest.mark.gpu
def test_gpu_features_on_reference_frames(gold, region):
    """ShmManager.get_latest_frame on the reference's frames: feature_as equals the reference's
    process_reservoir output within 1e-5 (observed: <= 1 ulp, the pow)."""
    dp = vs.VppDataPlane(region)
    mgr = vs.ShmManager(shm=region, device="cuda:0")
    for name in CASES:
        _publish_case(dp, gold, name)
        mgr.id_out = int(gold[f"{name}_seqs"][0]) - 1
        mgr.stat_last = {a: {"as_index": 0, "n_flow_on": 0, "ts": 0} for a in range(64)}
        active, feat, gt = mgr.get_latest_frame()
        ref = gold[f"{name}_feature_as"]
        assert active == list(gold[f"{name}_active_got"]) and gt is None
        np.testing.assert_allclose(feat, ref, rtol=1e-5, atol=1e-12, err_msg=name)
        np.testing.assert_allclose(feat, ref, rtol=1e-14, atol=0, err_msg=name)
        np.testing.assert_array_equal(feat[:, :4], ref[:, :4])  # n_flow_on, avg, 90, std exact


@pytest.mark.gpu
def test_gpu_register_as_weights_bytes(gold, region):
    """register_as_weights end to end on the product path (lbsim_alias_tables for gen_alias)."""
    mgr = vs.ShmManager(shm=region, device="cuda:0")
    for w, seq, want in zip(gold["weights_cases"], gold["weights_seqs"], gold["msg_in_weights"]):
        with mock.patch.object(vs.time, "time", return_value=float(gold["fixed_time"])):
            mgr.register_as_weights(int(seq), w)
        got = np.frombuffer(region.msg_in_frames[int(seq) & 3].tobytes(), np.uint8)
        np.testing.assert_array_equal(got, want, err_msg=str(seq))


@pytest.mark.gpu
def test_gpu_simulator_as_live_vpp(oracle_mod, tmp_path):
    """VppPublisher: the simulator's raw reservoirs (lbsim_vpp_export) equal the oracle's state
    seen the VPP way; the agent side reads the frame and computes process_reservoir on the GPU
    (= the oracle's restatement on the same bytes, up to the pow's last bit); the agent's
    register_as_weights scores come back as the envs' next weights."""
    import torch

    from marllb_amd.env import VecLoadBalanceEnv, make_config
    from tests import statelayout
    B, S, n = 6, 4, 3
    kw = dict(seed=77, action_type="continuous")
    env = VecLoadBalanceEnv(B, S, device="cuda:0", autoreset=False, **kw)
    ora = oracle_mod.OracleEnv(make_config(B, S, **kw), threads=2)
    env.reset()
    ora.reset()
    rng = np.random.default_rng(3)
    for _ in range(5):
        a = rng.uniform(0.1, 3.0, (B, S)).astype(np.float32)
        obs_g = env.step(torch.from_numpy(a))[0]
        ora.step(a)
    d = tmp_path.as_posix()
    pub = vs.VppPublisher(env, path_fmt=os.path.join("/dev/shm" if os.path.isdir("/dev/shm")
                                                      else d, f"lbsim_t{os.getpid()}_{{}}"), n=n)
    try:
        tv, nf, ts = pub.export()
        st = statelayout.parse(ora.state_bytes(), B, S, env.cfg.queue_capacity, False)
        cnt = np.minimum(st["res_count"].reshape(B, S), 128)
        words = {0: st["res_fct"].reshape(B, S, 128), 1: st["res_dur"].reshape(B, S, 128)}
        tsw = st["res_ts"].reshape(B, S, 128)
        clock = st["clock"]
        for b in range(n):
            assert ts[b] == np.float32(clock[b] * 0.25)
            np.testing.assert_array_equal(nf[b], obs_g[b, :, 0].cpu().numpy().astype(np.int32))
            for s in range(S):
                m = np.arange(128) < cnt[b, s]
                t = np.where(m, (tsw[b, s].astype(np.float64) * 1e-3).astype(np.float32), 0)
                for r in range(2):
                    v = np.where(m, words[r][b, s].view(np.int32).astype(np.float32) * np.float32(1e-6), 0)
                    np.testing.assert_array_equal(tv[b, s, r, :, 0], t)
                    np.testing.assert_array_equal(tv[b, s, r, :, 1], v.astype(np.float32))
        seqs = pub.publish()
        assert seqs == [1] * n
        for b in range(n):
            mgr = vs.ShmManager(path=pub.paths[b], device="cuda:0")
            active, feat, _ = mgr.get_latest_frame()
            assert active == list(range(S)) and mgr.id_out == 1
            want = oracle_mod.vpp_features(tv[b].reshape(-1, 128, 2), ts[b:b + 1],
                                           res_per_ts=10 ** 9).reshape(S, 10)
            np.testing.assert_allclose(feat[:S, 1:], want, rtol=1e-14, atol=0)
            np.testing.assert_array_equal(feat[:S, 0], nf[b])
            w = np.zeros(64)
            w[:S] = [1.0, 2.0, 0.5, 1.5]
            mgr.register_as_weights(1, w)
            mgr.close()
        acts = pub.poll_actions()
        np.testing.assert_array_equal(acts, np.tile(np.float32([1.0, 2.0, 0.5, 1.5]), (n, 1)))
        assert np.isnan(pub.poll_actions()).all()  # nothing new
    finally:
        pub.close()
        env.close()


def _tv_from_oracle_state(st, B, S, vpp=False):
    """The VPP view (lbsim_vpp_export's contract) of an oracle state snapshot: [B, S, 2, 128, 2]
    (t, v) f32 and the frame times [B].  vpp (reservoir_mode "vpp"): every bin as stored, else the
    first min(count, 128); a split (lost-FIN) snapshot's duration reservoir has its own count and
    timestamps."""
    cnts = (st["res_count"], st.get("res_count_dur", st["res_count"]))
    words = (st["res_fct"].reshape(B, S, 128), st["res_dur"].reshape(B, S, 128))
    tss = (st["res_ts"].reshape(B, S, 128), st.get("res_dur_ts", st["res_ts"]).reshape(B, S, 128))
    tv = np.zeros((B, S, 2, 128, 2), np.float32)
    for r in range(2):
        cnt = np.minimum(cnts[r].reshape(B, S), 128)
        m = np.arange(128)[None, None, :] < (128 if vpp else cnt[:, :, None])
        tv[:, :, r, :, 0] = np.where(m, (tss[r].astype(np.float64) * 1e-3).astype(np.float32),
                                     np.float32(0))
        tv[:, :, r, :, 1] = np.where(m, words[r].view(np.int32).astype(np.float32) * np.float32(1e-6),
                                     np.float32(0))
    ts = (st["clock"].astype(np.float64) * 0.25).astype(np.float32)
    return tv, ts


@pytest.mark.gpu
@pytest.mark.parametrize("kw", [dict(reservoir_mode="vpp"),
                                dict(lost_fin_prob=0.4, flow_timeout=0.5, flow_buckets=32),
                                dict(reservoir_mode="vpp", lost_fin_prob=0.4, flow_timeout=0.5,
                                     flow_buckets=32, duration_mode="service")])
def test_gpu_vpp_export_reservoir_modes(oracle_mod, kw):
    """lbsim_vpp_export under reservoir_mode "vpp" (every sample to bin rand() % 128 of a zeroed
    reservoir, lbhash.h:108,179: the agent's process_reservoir reads all 128 bins, shm_proxy.py:
    518-543) and under lost-FIN deferral (the duration reservoir's own count and timestamps):
    the GPU's wire view equals the oracle state's, bin for bin, after a reset and steps; under
    "vpp" never-written bins stay (0, 0) at first and fill as samples land."""
    import torch

    from marllb_amd.env import VecLoadBalanceEnv, make_config
    from tests import statelayout
    B, S = 24, 4
    kw = dict(seed=4242, **kw)
    env = VecLoadBalanceEnv(B, S, device="cuda:0", autoreset=False, **kw)
    cfg = make_config(B, S, **kw)
    ora = oracle_mod.OracleEnv(cfg, threads=2)
    vpp = kw.get("reservoir_mode") == "vpp"
    env.reset()
    ora.reset()
    rng = np.random.default_rng(1)
    zero_bins = []
    for k in range(6):
        a = rng.integers(0, 3, (B, S)).astype(np.int64)
        env.step(torch.from_numpy(a))
        ora.step(a)
        st = statelayout.parse(ora.state_bytes(), B, S, cfg.queue_capacity, False,
                               split_P=statelayout.split_p(cfg))
        want, ts_w = _tv_from_oracle_state(st, B, S, vpp)
        pub = vs.VppPublisher(env, path_fmt=os.path.join("/dev/shm", f"lbsim_m{os.getpid()}_{{}}"),
                              n=B)
        try:
            tv, _, ts = pub.export()
        finally:
            pub.close()
        np.testing.assert_array_equal(tv, want, err_msg=f"step {k}")
        np.testing.assert_array_equal(ts, ts_w)
        zero_bins.append(float((tv[..., 0] == 0).mean()))
    if vpp:  # bins stay zero until a sample lands in them: fewer with every step
        assert zero_bins[0] > zero_bins[-1] and zero_bins[0] > 0.05
    env.close()
    ora.close()


@pytest.mark.gpu
def test_gpu_upstream_feature_mode(oracle_mod):
    """VecLoadBalanceEnv(feature_mode='upstream'): columns 1-10 are process_reservoir's features
    of the simulator's reservoirs (oracle restatement on the oracle's state: 1e-5, observed within
    a float32 rounding of the f64 features), column 0 and the dynamics unchanged, the reward the
    reference reward on those rows, episode returns their running sum."""
    import torch

    from marllb_amd.env import VecLoadBalanceEnv, make_config
    from tests import statelayout
    B, S = 40, 4
    kw = dict(seed=5150, reward_metric="variance")
    env = VecLoadBalanceEnv(B, S, device="cuda:0", autoreset=False, feature_mode="upstream", **kw)
    ora = oracle_mod.OracleEnv(make_config(B, S, **kw), threads=2)
    Q = env.cfg.queue_capacity

    def expect(o_obs):
        st = statelayout.parse(ora.state_bytes(), B, S, Q, False)
        tv, ts = _tv_from_oracle_state(st, B, S)
        f = oracle_mod.vpp_features(tv.reshape(-1, 128, 2), ts, res_per_ts=2 * S)
        obs = o_obs.copy()
        obs[:, :, 1:] = f.reshape(B, S, 10).astype(np.float32)
        return obs, oracle_mod.rewards(obs, env.cfg.reward_metric, env.cfg.reward_field)

    og = env.reset().cpu().numpy()
    oo, _ = expect(ora.reset())
    np.testing.assert_allclose(og, oo, rtol=1e-6, atol=0)
    rng = np.random.default_rng(9)
    ret = np.zeros(B)
    for k in range(6):
        a = rng.integers(0, 3, (B, S)).astype(np.int64)
        og, rg, _, info = env.step(torch.from_numpy(a))
        o2, _, _, _ = ora.step(a)
        eo, er = expect(o2)
        np.testing.assert_allclose(og.cpu().numpy(), eo, rtol=1e-6, atol=0, err_msg=f"step {k}")
        np.testing.assert_array_equal(og.cpu().numpy()[:, :, 0], o2[:, :, 0])
        np.testing.assert_allclose(rg.cpu().numpy(), er, rtol=1e-5, atol=1e-7)
        ret += rg.cpu().numpy().astype(np.float64)
        np.testing.assert_allclose(info["episode_return"].cpu().numpy(), ret, rtol=1e-12)
    env.close()


@pytest.mark.gpu
def test_gpu_gen_alias_matches_reference_tables(golden_dir):
    """vpp_shm.gen_alias (lbsim_alias_tables) equals the reference gen_alias tables recorded by
    tests/golden/gen_golden.py (odd to float32, alias index exact)."""
    import json
    cases = json.load(open(os.path.join(golden_dir, "alias.json")))["cases"]
    for c in cases[:40]:
        w = c["weights"]
        if not all(x > 0 for x in w):
            continue
        got = vs.gen_alias(w, device="cuda:0")
        want = [(float(np.float32(o)), int(a)) for o, a in zip(c["odd"], c["alias"])]
        assert got == want, w
