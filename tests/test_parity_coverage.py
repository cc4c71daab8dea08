"""The GPU parity cases (tests/test_gpu_parity.py CONFIGS) reach the rare code paths of the
kernels -- checked here on the CPU with the oracle, which follows the same state layout:
  * reservoir samples >= 2^25 - 1 us  -> observe's two-pass (LSD) key sort;
  * queues longer than the dynamics kernel's LDS window -> HBM ring refills;
  * arrivals dropped because every queue is full;
  * observe's unchanged-reservoir skip: steps in which dynamics wrote no slot of any server of
    an env (observe reuses the cached features) next to steps that wrote many;
  * negative fct samples (lost-FIN flows with a flow timeout under 40 s) -> the signed sort;
  * servers down at the end of the failure cases;
  * observe's register-resident path (every reservoir of a 4-server chunk holding >= 8 samples,
    every slot below 2^25 - 1 us), both full (n = 128) and partly filled, next to its general path
    (a reservoir with fewer than 8 samples, or a large sample in the chunk).
"""
import numpy as np
import pytest

from tests import statelayout

pytest.importorskip("torch")
from tests.test_gpu_parity import CONFIGS, _actions, resolve_kw  # noqa: E402

PACK_LIMIT = (1 << 25) - 1


def window(S):
    return 8 if S <= 4 else (4 if S <= 8 else 2)


def run_case(oracle_mod, case, steps=12):
    from marllb_amd.env import make_config
    c = CONFIGS[case]
    B, S, kw = c["B"], c["S"], resolve_kw(c["kw"])
    kw.setdefault("seed", 1000 + case)
    cfg = make_config(B, S, **kw)
    ora = oracle_mod.OracleEnv(cfg, threads=4, trace=kw.get("trace"))
    ora.reset()
    rng = np.random.default_rng(case)
    max_q = 0
    written = []  # slots written per (env, server) by each step's dynamics
    paths = np.zeros(4, np.int64)  # recomputed chunks: register path full / register path partly
    #                                  filled / general path with a big sample / general with n < 8
    for _ in range(steps):
        ora.step(_actions(rng, B, S, c["kw"]))  # the GPU test's action stream
        st = statelayout.parse(ora.state_bytes(), B, S, cfg.queue_capacity, bool(cfg.normalize_obs),
                               cfg.fail_prob > 0, statelayout.has_leak(cfg),
                               split_P=statelayout.split_p(cfg))
        max_q = max(max_q, int((st["hc"] >> 16).max()))
        per_server = np.unpackbits(st["chg"].view(np.uint8)).reshape(B, S, 128).sum(2)
        written.append(per_server.sum(1))  # slots written per env (all its servers)
        nc = (S + 3) // 4
        pad = nc * 4 - S
        cnt = st["res_count"].reshape(B, S)
        full = np.pad(cnt >= 128, ((0, 0), (0, pad)), constant_values=True)
        ge8 = np.pad(cnt >= 8, ((0, 0), (0, pad)), constant_values=True)
        # the kernel decides by the sticky kHcBig flag of hc (bit 15): a record with a sample
        # >= 2^25 - 1 us (negative lost-FIN guesses: >= 2^31 as unsigned words) stored since the
        # reservoir was emptied
        big = ((st["hc"] >> 15) & 1).reshape(B, S).astype(bool)
        big = np.pad(big, ((0, 0), (0, pad)))
        chg = np.pad(per_server > 0, ((0, 0), (0, pad)))
        full, ge8, big, chg = (x.reshape(B, nc, 4) for x in (full, ge8, big, chg))
        cf, c8, cb, cc = full.all(2), ge8.all(2), big.any(2), chg.any(2)
        paths += [(cc & cf & ~cb).sum(), (cc & c8 & ~cf & ~cb).sum(), (cc & c8 & cb).sum(),
                  (cc & ~c8).sum()]
    run_case.written = np.concatenate(written)
    run_case.negative = bool((st["res_fct"].view(np.int32) < 0).any())
    run_case.down = int(st["down"].sum()) if "down" in st else 0
    run_case.paths = paths
    return st, max_q, S


def test_parity_cases_cover_rare_paths(oracle_mod):
    two_pass = overflow = dropped = negative = False
    down = 0
    written = []
    paths = np.zeros(4, np.int64)
    for case in range(len(CONFIGS)):
        st, max_q, S = run_case(oracle_mod, case)
        two_pass |= bool(max(st["res_fct"].max(), st["res_dur"].max()) >= PACK_LIMIT)
        overflow |= max_q > window(S)
        dropped |= bool(st["dropped"].sum() > 0)
        written.append(run_case.written)
        paths += run_case.paths
        negative |= run_case.negative
        down += run_case.down
    w = np.concatenate(written)
    assert (paths > 20).all(), f"observe paths (register full / register partial / general with a " \
                               f"big sample / general with n < 8): {paths}"
    assert (w == 0).sum() > 50, "too few env-steps leave every reservoir unchanged (the skip)"
    assert (w == 1).any() and (w >= 64).sum() > 100
    assert two_pass, "no parity case produces a sample >= 2^25 - 1 us"
    assert overflow, "no parity case queues more flows than the LDS window"
    assert dropped, "no parity case drops arrivals"
    assert negative, "no parity case records a negative (lost-FIN) fct sample"
    assert down > 20, "too few servers down at the end of the failure cases"
    assert any(c["kw"].get("_nan_actions") for c in CONFIGS), "no case with NaN SED scores"
