"""Arrival traces for the TRACE arrival source (BASELINE configs[2]).

The reference's traces are `time<TAB>query` CSVs (`data/trace/poisson_for_loop/rate_*.csv`, read by
`src/client/replay_fork_io.py:95-121`): a request time in seconds and a URL `/dummy.php/?n=<N>`
whose server runs an N-iteration loop.  The simulator consumes them as two device arrays, one entry
per row:

    gap_us[i]  integer us between row i-1 and row i (times rounded to us from the first row);
               gap_us[0] is the wrap-around gap, the trace's mean gap
    work[i]    float32 N_i / mean(N): service demand in mean-1 units, so a server of rate mu serves
               row i in max(1, int(work * 1e6 / mu)) us -- the same scale as the Poisson source's
               Exp(1) work

Env `gid` in episode `e` replays rows (gid * 7919 + (e - 1) * 1000003 + k) mod R for its k-th
arrival, wrapping around the end.  The hash words that break SED ties and pick SED2 / ALIAS
candidates still come from Philox.
"""
from __future__ import annotations

import os
from dataclasses import dataclass

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
DATA = os.path.join(os.path.dirname(HERE), "data", "traces")


@dataclass
class Trace:
    gap_us: np.ndarray   # uint32 [R]
    work: np.ndarray     # float32 [R]
    rate: float          # arrivals per second (rows / span)
    name: str = ""

    @property
    def rows(self) -> int:
        return int(self.gap_us.shape[0])


def from_times(t_s: np.ndarray, n: np.ndarray, name: str = "") -> Trace:
    """Build the device arrays from request times (s) and loop counts N."""
    t_s = np.asarray(t_s, np.float64)
    n = np.asarray(n, np.float64)
    if t_s.ndim != 1 or t_s.shape != n.shape or len(t_s) < 2:
        raise ValueError("trace needs >= 2 rows of (time, n)")
    if np.any(np.diff(t_s) < 0):
        raise ValueError("trace times must be non-decreasing")
    if np.any(n <= 0):
        raise ValueError("trace loop counts must be positive")
    t_us = np.rint((t_s - t_s[0]) * 1e6).astype(np.int64)
    span = int(t_us[-1])
    mean_gap = max(1, int(round(span / (len(t_us) - 1))))
    gap = np.empty(len(t_us), np.int64)
    gap[0] = mean_gap
    gap[1:] = np.diff(t_us)
    if gap.max() >= 2**31:
        raise ValueError("trace gaps must be < 2^31 us")
    work = (n / n.mean()).astype(np.float32)
    rate = (len(t_us) - 1) / (span * 1e-6) if span > 0 else float("inf")
    return Trace(gap.astype(np.uint32), work, float(rate), name)


def load_csv(path: str) -> Trace:
    """Parse a reference trace CSV (header `time<TAB>query`, query `...?n=<N>`)."""
    ts, ns = [], []
    with open(path) as fh:
        header = fh.readline().split()
        if header[:1] != ["time"]:
            raise ValueError(f"{path}: expected a 'time<TAB>query' header")
        for line in fh:
            parts = line.split()
            if len(parts) < 2:
                continue
            q = parts[1]
            i = q.rfind("n=")
            if i < 0:
                raise ValueError(f"{path}: query without n=: {q}")
            ts.append(float(parts[0]))
            ns.append(int(q[i + 2:]))
    return from_times(np.array(ts), np.array(ns), os.path.basename(path))


def save_npz(trace_times_s: np.ndarray, n: np.ndarray, path: str) -> None:
    """Compact form of a CSV (times in integer us from the first row, N as uint32)."""
    t = np.rint((np.asarray(trace_times_s, np.float64) - trace_times_s[0]) * 1e6).astype(np.uint32)
    np.savez_compressed(path, t_us=t, n=np.asarray(n, np.uint32))


def load_npz(path: str) -> Trace:
    d = np.load(path, allow_pickle=False)
    return from_times(d["t_us"].astype(np.float64) * 1e-6, d["n"].astype(np.float64),
                      os.path.basename(path))


def builtin(name: str = "poisson_for_loop_rate_500") -> Trace:
    """A trace converted into data/traces/ by tools/convert_trace.py."""
    return load_npz(os.path.join(DATA, name + ".npz"))


def synthetic(rows: int, rate: float, seed: int = 0) -> Trace:
    """Poisson-times, lognormal-N trace for tests (no file needed)."""
    rng = np.random.default_rng(seed)
    t = np.cumsum(rng.exponential(1.0 / rate, rows))
    n = np.maximum(1, rng.lognormal(14.8, 0.8, rows)).astype(np.int64)
    return from_times(t, n, f"synthetic-{rows}-{rate}")
