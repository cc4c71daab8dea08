"""The CPU oracle against the reference's own outputs (tests/golden/, made by gen_golden.py).

Pins oracle/lbsim_oracle.c to the reference Python before the oracle is trusted as the GPU
checker:
  reservoir.py:105-196 features   -> bit-exact mean/p90/std/p90_decay, mean_decay <= 2e-6 rel
  rewards.py:21-381 (9 metrics)   -> <= 1e-12 rel in float64 (numpy's x**2 goes through libm pow)
  env.py:450-470 normalisation    -> float32 cast of the float64 reference
  Philox4x32-10                   -> Random123 known-answer vectors
  Algorithm R                     -> uniformity chi^2 as test_reservoir.py:243-287
"""
import json
import math
import os

import numpy as np
import pytest

FIELD_COL = {"flow_duration_avg_decay": 10, "n_flow_on": 0, "fct_mean": 1, "no_such_field": -1}


def test_philox_known_answers(oracle_mod):
    kat = [((0, 0, 0, 0), (0, 0), (0x6627E8D5, 0xE169C58D, 0xBC57AC4C, 0x9B00DBD8)),
           ((0xFFFFFFFF,) * 4, (0xFFFFFFFF,) * 2, (0x408F276D, 0x41C83B0E, 0xA20BC7C6, 0x6D5451FD)),
           ((0x243F6A88, 0x85A308D3, 0x13198A2E, 0x03707344), (0xA4093822, 0x299F31D0),
            (0xD16CFE09, 0x94FDCCEB, 0x5001E420, 0x24126EA1))]
    for ctr, key, exp in kat:
        assert list(oracle_mod.philox(ctr, key)) == list(exp)


def test_log_exp2_accuracy(oracle_mod):
    lib = oracle_mod.load()
    xs = np.linspace(-59.9, 0.0, 20001, dtype=np.float32)
    rel = max(abs(lib.oracle_exp2f(float(x)) / 2.0 ** float(x) - 1.0) for x in xs)
    assert rel < 2e-7
    us = (np.arange(1, 2 ** 24, 997) * 2.0 ** -24).astype(np.float32)
    err = max(abs(lib.oracle_logf(float(u)) - math.log(float(u))) for u in us)
    assert err < 1e-6


def test_reservoir_features_match_reference(oracle_mod, golden_dir):
    g = np.load(os.path.join(golden_dir, "reservoir_features.npz"))
    out = oracle_mod.features(g["values"], g["ts_ms"], g["counts"], float(g["decay"]))
    exp = g["expected"]
    for f in (0, 1, 2, 4):  # mean, p90, std, p90_decay: bit-exact float32
        np.testing.assert_array_equal(out[:, f], exp[:, f].astype(np.float32), err_msg=f"col {f}")
    rel = np.abs(out[:, 3] - exp[:, 3]) / np.maximum(np.abs(exp[:, 3]), 1e-30)
    assert rel.max() < 2e-6, rel.max()
    # known answers of test_reservoir.py:80-131
    assert out[0].tolist() == [0.0] * 5
    assert abs(out[1, 0] - 3.0) < 1e-6 and abs(out[1, 2] - np.std([1, 2, 3, 4, 5])) < 1e-6
    assert 85 < out[2, 1] < 95
    assert abs(out[3, 0] - 5.5) < 0.5 and 7.0 < out[3, 3] < 10.0


@pytest.mark.parametrize("S", [1, 2, 3, 4, 8, 16])
def test_rewards_match_reference(oracle_mod, golden_dir, S):
    g = np.load(os.path.join(golden_dir, "rewards.npz"))
    metrics, fields = list(g["metrics"]), list(g["fields"])
    obs, exp = g[f"obs_S{S}"], g[f"expected_S{S}"]
    for m in range(len(metrics)):
        for fi, fname in enumerate(fields):
            got = oracle_mod.rewards(obs, m, FIELD_COL[str(fname)], f64=True)
            want = exp[:, m, fi]
            np.testing.assert_allclose(got, want, rtol=1e-12, atol=1e-300,
                                       err_msg=f"{metrics[m]} {fname}")


def test_metric_known_answers(oracle_mod, golden_dir):
    """rewards.py docstring / test_rewards.py values through the obs path (all servers active)."""
    plumb = json.load(open(os.path.join(golden_dir, "env_plumbing.json")))
    names = ["jain", "variance", "std", "cv", "max", "min", "product", "range", "gini"]
    for case in plumb["metric_kat"]:
        vals = case["values"]
        obs = np.ones((1, len(vals), 11), np.float32)
        obs[0, :, 10] = vals
        for m, name in enumerate(names):
            got = oracle_mod.rewards(obs, m, 10, f64=True)[0]
            assert got == pytest.approx(case[name], rel=1e-12, abs=1e-15), name


def test_normalisation_matches_reference(oracle_mod, golden_dir):
    """env.py:450-470 through a 1-env oracle whose raw obs are injected via the state snapshot."""
    plumb = json.load(open(os.path.join(golden_dir, "env_plumbing.json")))
    seq = [np.array(x, np.float32) for x in plumb["normalize"]["inputs"]]
    want = [np.array(x) for x in plumb["normalize"]["outputs"]]
    lib = oracle_mod.load()
    mean = np.zeros(44, np.float64)
    std = np.ones(44, np.float64)
    count = np.zeros(1, np.int32)
    for raw, w in zip(seq, want):
        out = np.zeros(44, np.float32)
        lib.oracle_normalize(oracle_mod.ptr(np.ascontiguousarray(raw.reshape(-1))), 44,
                             oracle_mod.ptr(count), oracle_mod.ptr(mean), oracle_mod.ptr(std),
                             oracle_mod.ptr(out))
        np.testing.assert_array_equal(out, w.reshape(-1).astype(np.float32))


def test_algorithm_r_uniformity(oracle_mod):
    """Every stream element is kept with probability K/N (chi^2 as test_reservoir.py:243-287)."""
    import ctypes
    lib = oracle_mod.load()
    K, N, trials = 128, 1000, 500
    counts = np.zeros(N)
    key = np.array([12345, 678], np.uint32)
    for t in range(trials):
        slots = np.arange(K)  # slot -> stream index
        for c in range(K, N):
            j = lib.oracle_algr_slot(c, t, 1, 0, oracle_mod.ptr(key))
            if j >= 0:
                slots[j] = c
        counts[slots] += 1
    expected = trials * K / N
    chi2 = np.sum((counts - expected) ** 2 / expected)
    assert chi2 < 1100, chi2


def test_algorithm_r_acceptance_rate(oracle_mod):
    lib = oracle_mod.load()
    key = np.array([1, 2], np.uint32)
    for count in (128, 1000, 100000, 2 ** 31 - 5):
        acc = sum(lib.oracle_algr_slot(count, e, 7, 3, oracle_mod.ptr(key)) >= 0
                  for e in range(20000))
        p = 128 / (count + 1)
        assert abs(acc / 20000 - p) < 5 * math.sqrt(p * (1 - p) / 20000) + 1e-4


def test_algorithm_r_arrival_draw_rule(oracle_mod):
    """The in-step rule (a flow that arrives and completes in one step): j = floor(r (c + 1) /
    2^32) from its arrival's Philox word 3: exact edges, then every stream
    element kept with probability K/N and the acceptance rate K/(c + 1)."""
    lib = oracle_mod.load()
    K = 128
    assert lib.oracle_algr_slot_r32(5, 0xFFFFFFFF) == 5          # filling: slot = count
    assert lib.oracle_algr_slot_r32(K, 0) == 0
    assert lib.oracle_algr_slot_r32(K, 0xFFFFFFFF) == -1         # j = count = 128: not kept
    assert lib.oracle_algr_slot_r32(2 ** 32 - 1, 127) == 127     # c + 1 = 2^32: j = r
    key = np.array([12345, 678], np.uint32)
    N, trials = 1000, 500
    counts = np.zeros(N)
    for t in range(trials):
        slots = np.arange(K)
        for c in range(K, N):  # the arrival block of arrival c of "env" t
            r = int(oracle_mod.philox(np.array([c, t, 1, 1 << 24], np.uint32), key)[3])
            j = lib.oracle_algr_slot_r32(c, r)
            if j >= 0:
                slots[j] = c
        counts[slots] += 1
    expected = trials * K / N
    chi2 = np.sum((counts - expected) ** 2 / expected)
    assert chi2 < 1100, chi2
    for count in (128, 1000, 100000, 2 ** 31 - 5):
        acc = sum(lib.oracle_algr_slot_r32(
            count, int(oracle_mod.philox(np.array([e, 7, 3, 1 << 24], np.uint32), key)[3])) >= 0
            for e in range(20000))
        p = 128 / (count + 1)
        assert abs(acc / 20000 - p) < 5 * math.sqrt(p * (1 - p) / 20000) + 1e-4


def test_gen_alias_matches_reference(oracle_mod, golden_dir):
    """oracle_gen_alias == the reference gen_alias (src/lb/shm_proxy.py:127-146) bit for bit in
    float64, on 137 weight vectors (n = 1..16, ties with the mean, the SURVEY §8a example)."""
    import json
    cases = json.load(open(os.path.join(golden_dir, "alias.json")))["cases"]
    assert len(cases) > 100
    for c in cases:
        odd, alias = oracle_mod.gen_alias(np.array(c["weights"], np.float32))
        np.testing.assert_array_equal(odd, np.array(c["odd"], np.float64))
        np.testing.assert_array_equal(alias, np.array(c["alias"], np.int32))


def test_alias_pick_frequencies(oracle_mod):
    """The ALIAS rule (node.c:449-460) over a gen_alias table picks server i with probability
    ~ w_i / sum(w) (gen_alias's 1e-6 epsilons aside)."""
    w = np.array([1.0, 1.0, 1.0, 1.0, 2.0, 2.0, 2.0], np.float32)
    odd, alias = oracle_mod.gen_alias(w)
    odd = odd.astype(np.float32)
    u = np.random.default_rng(0).integers(0, 2**32, 400000, dtype=np.uint64).astype(np.uint32)
    rn = (u >> 8).astype(np.float32) * np.float32(5.9604644775390625e-8) * np.float32(len(w))
    bucket = np.minimum(rn.astype(np.int32), len(w) - 1)
    pick = np.where(rn - bucket.astype(np.float32) > odd[bucket], alias[bucket], bucket)
    freq = np.bincount(pick, minlength=len(w)) / len(u)
    np.testing.assert_allclose(freq, w / w.sum(), atol=3e-3)


def vose_rows(seed=5):
    """Weight rows for the Vose tests: ragged S (1..64), zeros, ties, one dominant weight,
    all-zero and negative-sum rows (the identity table), huge dynamic range."""
    rng = np.random.default_rng(seed)
    rows = [np.array([1, 2, 3, 2], np.float32), np.ones(4, np.float32), np.zeros(6, np.float32),
            np.array([5.0], np.float32), np.array([0, 0, 7, 0], np.float32),
            np.array([-1.0, 0.5, 0.25], np.float32), np.array([1e-6, 1e6, 1.0, 3.0], np.float32),
            np.array([0.1] * 10 + [10.0], np.float32)]
    for S in (2, 3, 4, 8, 16, 20, 33, 64):
        for _ in range(12):
            w = rng.choice([0.1, 1.0, 1.5, 2.0, 10.0], S).astype(np.float32)
            if rng.random() < 0.5:
                w = rng.uniform(0, 10, S).astype(np.float32)
            w[rng.random(S) < 0.2] = 0.0
            rows.append(w)
    return rows


def test_vose_known_answers(oracle_mod):
    """Hand-traced alias_table_build (problem-07 vpp-plugin/alias_table.h:82-158) and the
    xorshift32 of alias_table_random (:163-172)."""
    # w = [1,2,3,2]: prob_scaled [0.5,1,1.5,1]; small [0], large [1,2,3]; (0 <- 3) leaves 3 at
    # 0.5 -> small; (3 <- 2) leaves 2 at 1.0 -> large; leftovers 2, 1 are (1, self)
    prob, alias = oracle_mod.vose_build([1, 2, 3, 2])
    assert prob.tolist() == [0.5, 1.0, 1.0, 0.5] and alias.tolist() == [3, 1, 2, 2]
    prob, alias = oracle_mod.vose_build([0, 0, 0])  # sum <= 0: identity (:95-102)
    assert prob.tolist() == [1.0] * 3 and alias.tolist() == [0, 1, 2]
    # xorshift32 from state 1: 270369, then 67634689 (13/17/5 triple)
    idx, hist, st = oracle_mod.vose_sample(np.ones(4, np.float32), np.arange(4), 1, 1)
    assert st == 67634689 and idx.tolist() == [270369 % 4] and hist.tolist() == [0, 1, 0, 0]


def test_vose_tables_represent_weights(oracle_mod):
    """Every Vose table's implied distribution (prob[i] + sum over j aliased to i of
    1 - prob[j], over n) equals w / sum(w) within float32 rounding; the sampler's frequencies
    follow it."""
    for w in vose_rows():
        prob, alias = oracle_mod.vose_build(w)
        n = len(w)
        assert ((prob >= 0) & (prob <= 1.0 + 1e-6)).all() and (alias < n).all()
        implied = prob.astype(np.float64).copy()
        np.add.at(implied, alias, 1.0 - prob.astype(np.float64))
        implied /= n
        s = float(np.sum(w, dtype=np.float32))
        want = w / s if s > 0 else np.full(n, 1.0 / n)
        np.testing.assert_allclose(implied, want, atol=2e-6 * max(1, n))
    w = np.array([1, 2, 3, 2, 0, 8], np.float32)
    prob, alias = oracle_mod.vose_build(w)
    _, hist, _ = oracle_mod.vose_sample(prob, alias, 12345, 400000)
    np.testing.assert_allclose(hist / 400000, w / w.sum(), atol=3e-3)
