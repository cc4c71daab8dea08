#!/usr/bin/env python3
"""Convert a reference arrival-trace CSV into data/traces/<name>.npz (integer-us times + loop
counts), so the trace travels with the repo (the reference tree is not on the GPU box).

    python tools/convert_trace.py /root/reference/data/trace/poisson_for_loop/rate_500.csv \
        --name poisson_for_loop_rate_500

Runs in the build container only.  The .npz is data (request times and N), not code.
"""
import argparse
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from marllb_amd import trace  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("csv")
    ap.add_argument("--name", required=True)
    a = ap.parse_args()
    ts, ns = [], []
    with open(a.csv) as fh:
        fh.readline()
        for line in fh:
            p = line.split()
            if len(p) < 2:
                continue
            ts.append(float(p[0]))
            ns.append(int(p[1][p[1].rfind("n=") + 2:]))
    ts, ns = np.array(ts), np.array(ns)
    os.makedirs(trace.DATA, exist_ok=True)
    out = os.path.join(trace.DATA, a.name + ".npz")
    trace.save_npz(ts, ns, out)
    tr = trace.load_npz(out)
    ref = trace.load_csv(a.csv)
    assert np.array_equal(tr.gap_us, ref.gap_us) and np.array_equal(tr.work, ref.work)
    print(f"{out}: {tr.rows} rows, {tr.rate:.1f}/s, {os.path.getsize(out)} bytes")


if __name__ == "__main__":
    main()
