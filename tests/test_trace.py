"""Trace arrival source: CSV/npz ingestion and the oracle's replay
rule (row (gid * 7919 + (episode - 1) * 1000003 + k) mod R for the k-th arrival)."""
import os

import numpy as np
import pytest

from marllb_amd import trace

REF_CSV = "/root/reference/data/trace/poisson_for_loop/rate_500.csv"


def test_builtin_trace_shape_and_rate():
    t = trace.builtin()
    assert t.rows == 77965 and t.gap_us.dtype == np.uint32 and t.work.dtype == np.float32
    assert abs(t.rate - 487.66) < 0.1                      # 487.7/s measured
    assert abs(float(t.work.astype(np.float64).mean()) - 1.0) < 1e-6
    assert t.gap_us[0] == round(int(t.gap_us[1:].sum()) / (t.rows - 1))  # wrap gap = mean gap


@pytest.mark.skipif(not os.path.exists(REF_CSV), reason="reference tree not present")
def test_builtin_npz_equals_reference_csv():
    a, b = trace.builtin(), trace.load_csv(REF_CSV)
    np.testing.assert_array_equal(a.gap_us, b.gap_us)
    np.testing.assert_array_equal(a.work, b.work)


def test_from_times_rules(tmp_path):
    t = trace.from_times(np.array([0.5, 0.5000014, 0.75, 2.0]), np.array([10, 20, 30, 40]))
    np.testing.assert_array_equal(t.gap_us, [500000, 1, 249999, 1250000])
    np.testing.assert_allclose(t.work, np.array([10, 20, 30, 40]) / 25.0, rtol=1e-7)
    p = tmp_path / "x.csv"
    p.write_text("time\tquery\n0.1\t/dummy.php/?n=5\n0.3\t/dummy.php/?n=15\n")
    c = trace.load_csv(str(p))
    np.testing.assert_array_equal(c.gap_us, [200000, 200000])
    with pytest.raises(ValueError):
        trace.from_times(np.array([1.0, 0.5]), np.array([1, 1]))
    with pytest.raises(ValueError):
        trace.from_times(np.array([1.0, 2.0]), np.array([1, 0]))


def test_oracle_replays_trace_rows(oracle_mod):
    """The oracle's arrivals follow the trace rows from each env's offset: per step, arrivals
    match the gaps cumulated from that offset, and work follows the rows' N."""
    from marllb_amd.env import make_config
    tr = trace.synthetic(500, 400.0, seed=2)
    B, S = 6, 4
    cfg = make_config(B, S, seed=5, trace=tr, warmup_steps=0, queue_capacity=64,
                      server_rates=[1e6] * S)
    assert cfg.arrival_source == 1 and abs(cfg.arrival_rate - tr.rate) < 1e-3
    ora = oracle_mod.OracleEnv(cfg, trace=tr)
    ora.reset()
    steps = 5
    tot = np.zeros((B, S), np.int64)
    for _ in range(steps):
        _, _, _, assign = ora.step(np.zeros((B, S), np.int64))
        tot += assign
    dt = 250000
    for b in range(B):
        r0 = (b * 7919) % tr.rows
        rows = (r0 + np.arange(4 * tr.rows)) % tr.rows
        t = np.cumsum(tr.gap_us[rows].astype(np.int64))
        assert tot[b].sum() == np.count_nonzero(t < steps * dt), b
