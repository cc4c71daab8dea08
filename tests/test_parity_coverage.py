"""The GPU parity cases (tests/test_gpu_parity.py CONFIGS) reach the rare code paths of the
kernels -- checked here on the CPU with the oracle, which follows the same state layout:
  * reservoir samples >= 2^25 - 1 us  -> observe's two-pass (LSD) key sort;
  * queues longer than the dynamics kernel's LDS window -> HBM ring refills;
  * arrivals dropped because every queue is full;
  * observe's unchanged-reservoir skip: steps in which dynamics wrote no slot of any server of
    an env (observe reuses the cached features) next to steps that wrote many.
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
    for _ in range(steps):
        ora.step(_actions(rng, B, S, c["kw"]))  # the GPU test's action stream
        st = statelayout.parse(ora.state_bytes(), B, S, cfg.queue_capacity, bool(cfg.normalize_obs))
        max_q = max(max_q, int((st["hc"] >> 16).max()))
        per_server = np.unpackbits(st["chg"].view(np.uint8)).reshape(B, S, 128).sum(2)
        written.append(per_server.sum(1))  # slots written per env (all its servers)
    run_case.written = np.concatenate(written)
    return st, max_q, S


def test_parity_cases_cover_rare_paths(oracle_mod):
    two_pass = overflow = dropped = False
    written = []
    for case in range(len(CONFIGS)):
        st, max_q, S = run_case(oracle_mod, case)
        two_pass |= bool(max(st["res_fct"].max(), st["res_dur"].max()) >= PACK_LIMIT)
        overflow |= max_q > window(S)
        dropped |= bool(st["dropped"].sum() > 0)
        written.append(run_case.written)
    w = np.concatenate(written)
    assert (w == 0).sum() > 50, "too few env-steps leave every reservoir unchanged (the skip)"
    assert (w == 1).any() and (w >= 64).sum() > 100
    assert two_pass, "no parity case produces a sample >= 2^25 - 1 us"
    assert overflow, "no parity case queues more flows than the LDS window"
    assert dropped, "no parity case drops arrivals"
    assert any(c["kw"].get("_nan_actions") for c in CONFIGS), "no case with NaN SED scores"
