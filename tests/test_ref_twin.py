"""The reference's own C reservoir twin (simulation-mode/problem-01-reservoir-sampling/src/
reservoir.h, compiled where it lies by oracle/ref_build.py into oracle/_ref/, CPU) against our
oracle -- test infrastructure checking test infrastructure.

* Algorithm R (reservoir.h:118-143): the twin's reservoir after every add equals a replay of the
  oracle's rule (count < K -> slot count, else slot j = draw mod (count + 1), kept if j < K) fed
  with the twin's own xorshift128+ draws (reservoir.h:80-106), predicted here.  The oracle
  applies the same rule to a Philox draw, so only the draw differs.
* Statistics (reservoir.h:179-268) vs the oracle's, which follows the Python reference
  (reservoir.py:105-196, pinned by tests/golden): mean, mean_decay and p90_decay agree within
  float32 summation-order tolerance; p90 differs by design -- the C twin takes the nearest index
  sorted[(int)(0.9f n)], the Python reference and the oracle numpy's linear interpolation -- so the
  twin's p90 is checked against that index of the sorted values.
"""
import ctypes
import os

import numpy as np
import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(os.path.dirname(HERE), "oracle", "_ref", "libref_reservoir.so")
K = 128
M64 = (1 << 64) - 1


@pytest.fixture(scope="module")
def twin():
    if not os.path.exists(LIB):
        pytest.skip("oracle/_ref/libref_reservoir.so not built (needs /root/reference)")
    lib = ctypes.CDLL(LIB)
    lib.ref_reservoir_sizeof.restype = ctypes.c_size_t
    lib.ref_reservoir_init.argtypes = [ctypes.c_void_p, ctypes.c_uint64]
    lib.ref_reservoir_add.argtypes = [ctypes.c_void_p, ctypes.c_float, ctypes.c_uint64]
    lib.ref_reservoir_add.restype = ctypes.c_int
    lib.ref_reservoir_count.argtypes = [ctypes.c_void_p]
    lib.ref_reservoir_count.restype = ctypes.c_uint64
    lib.ref_reservoir_values.argtypes = [ctypes.c_void_p]
    lib.ref_reservoir_values.restype = ctypes.POINTER(ctypes.c_float)
    lib.ref_reservoir_stats.argtypes = [ctypes.c_void_p, ctypes.c_float, ctypes.c_uint64,
                                        ctypes.c_void_p]
    return lib


def new_reservoir(lib, seed):
    buf = ctypes.create_string_buffer(lib.ref_reservoir_sizeof())
    lib.ref_reservoir_init(buf, seed)
    return buf


def xorshift_state(seed):  # reservoir.h:55-74 reservoir_init
    if seed == 0:
        return [0x123456789ABCDEF0, 0xFEDCBA9876543210]
    return [seed & M64, (seed ^ M64) & M64]


def xorshift128plus(st):  # reservoir.h:80-89
    x, y = st[0], st[1]
    st[0] = y
    x = (x ^ (x << 23)) & M64
    st[1] = x ^ y ^ (x >> 17) ^ (y >> 26)
    return (st[1] + y) & M64


def algorithm_r_slot(count, draw):
    """The oracle's rule (oracle/lbsim_oracle.c reservoir_add, reservoir.py:64-85) given a draw
    in [0, count] for a full reservoir; -1 = not stored."""
    if count < K:
        return count
    return draw if draw < K else -1


@pytest.mark.parametrize("seed", [0, 1, 20260109])
def test_algorithm_r_rule_matches_the_c_twin(twin, seed):
    r = new_reservoir(twin, seed)
    st = xorshift_state(seed)
    mine = np.zeros(K, np.float32)
    rng = np.random.default_rng(seed)
    vals = rng.uniform(0.0, 100.0, 3000).astype(np.float32)
    stored = 0
    for i, v in enumerate(vals):
        draw = xorshift128plus(st) % (i + 1) if i >= K else 0  # random_range(count + 1)
        slot = algorithm_r_slot(i, draw)
        accepted = twin.ref_reservoir_add(r, float(v), i)
        assert bool(accepted) == (slot >= 0), f"add {i}"
        if slot >= 0:
            mine[slot] = v
            stored += 1
        assert twin.ref_reservoir_count(r) == i + 1
    got = np.ctypeslib.as_array(twin.ref_reservoir_values(r), shape=(K,))
    np.testing.assert_array_equal(got, mine)
    assert K < stored < len(vals)


def test_algorithm_r_inclusion_probability_twin_and_oracle(twin, oracle_mod):
    """Each of N items ends in the reservoir with probability K/N under both RNGs (the twin's
    xorshift128+ and the oracle's Philox Algorithm R draw, oracle_algr_slot)."""
    N, trials = 512, 300
    lib = oracle_mod.load()
    key = np.array([20260109, 0], np.uint32)
    hits_t = np.zeros(N)
    hits_o = np.zeros(N)
    for t in range(trials):
        r = new_reservoir(twin, 1000 + t)
        for i in range(N):
            twin.ref_reservoir_add(r, float(i), i)
        vals = np.ctypeslib.as_array(twin.ref_reservoir_values(r), shape=(K,)).astype(int)
        hits_t[vals] += 1
        res = np.arange(K)
        for c in range(K, N):
            s = lib.oracle_algr_slot(c, t, 1, 0, oracle_mod.ptr(key))
            if s >= 0:
                res[s] = c
        hits_o[res] += 1
    p = K / N
    sd = np.sqrt(trials * p * (1 - p))
    for hits in (hits_t, hits_o):
        z = (hits - trials * p) / sd
        assert abs(z.mean()) < 0.2 and z.std() < 1.3, (z.mean(), z.std())


def _stat_cases(rng):
    cases = []
    for n in (1, 5, 17, 64, 100, 128):
        for kind in range(3):
            if kind == 0:
                v = (rng.exponential(8e3, n).astype(np.int64) + 1).astype(np.float32) * np.float32(1e-6)
            elif kind == 1:
                v = rng.uniform(1.0, 50.0, n).astype(np.float32)
            else:
                v = rng.choice(np.float32([0.5, 1.0, 2.0, 4.0]), n)
            age_ms = rng.integers(0, 20000, n)
            cases.append((v.astype(np.float32), age_ms))
    return cases


def test_statistics_c_twin_vs_oracle(twin, oracle_mod):
    rng = np.random.default_rng(7)
    now_ms = 50_000
    for v, age_ms in _stat_cases(rng):
        n = len(v)
        r = new_reservoir(twin, 3)
        ts_ms = (now_ms - age_ms).astype(np.uint32)
        for i in range(n):
            twin.ref_reservoir_add(r, float(v[i]), int(ts_ms[i]) * 1000)  # us timestamps
        c_out = np.zeros(5, np.float32)
        twin.ref_reservoir_stats(r, 0.9, now_ms * 1000, c_out.ctypes.data)
        vv = np.zeros(K, np.float32)
        vv[:n] = v
        tt = np.zeros(K, np.uint32)
        tt[:n] = ts_ms
        o = oracle_mod.features(vv, tt, np.array([n], np.uint32))[0]
        mean, p90, std, md, p90d = c_out
        np.testing.assert_allclose(mean, o[0], rtol=2e-6)           # sequential vs pairwise f32
        np.testing.assert_allclose(std, o[2], rtol=2e-3, atol=1e-6)  # one-pass vs two-pass
        np.testing.assert_allclose(md, o[3], rtol=2e-5)              # f32 vs f64 weighted mean
        srt = np.sort(v)
        assert p90 == srt[min(int(np.float32(0.9) * np.float32(n)), n - 1)]  # nearest index
        if n > 1 and srt[0] != srt[-1]:
            lo = int(np.floor(np.float32(n - 1) * np.float32(0.9)))
            assert srt[lo] <= o[1] <= srt[min(lo + 1, n - 1)]  # the oracle interpolates
        # p90_decay: same crossing unless a cumulative weight sits at the 90% cut within float32
        # rounding of it (the C twin sums float32 sequentially, the oracle in exact fixed point)
        w = np.exp(np.log(np.float32(0.9)) * (age_ms / 1000.0))
        order = np.argsort(v, kind="stable")
        cs = np.cumsum(w[order])
        if np.min(np.abs(cs - 0.9 * cs[-1])) > 1e-4 * cs[-1]:
            assert p90d == o[4]
