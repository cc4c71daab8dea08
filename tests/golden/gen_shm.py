#!/usr/bin/env python3
"""Golden wire-format bytes of problem-02's SHM messages (this container only).

Imports simulation-mode/problem-02-shared-memory-ipc/src/shm_layout.py in place and records the
bytes its packers produce (MessageOutLayout.pack, MessageInLayout.pack with a fixed timestamp) and
the layout sizes -> tests/golden/shm.json.  marllb_amd/shm.py must reproduce them byte for byte.
"""
import importlib.util
import io
import json
import os
import sys
from contextlib import redirect_stdout
from unittest import mock

HERE = os.path.dirname(os.path.abspath(__file__))


def main(root="/root/reference"):
    path = os.path.join(root, "simulation-mode/problem-02-shared-memory-ipc/src/shm_layout.py")
    spec = importlib.util.spec_from_file_location("ref_shm_layout", path)
    mod = importlib.util.module_from_spec(spec)
    with redirect_stdout(io.StringIO()):  # the module prints its sizes at import
        spec.loader.exec_module(mod)
    out = {"sizes": {"msg_out": mod.MessageOutLayout.MESSAGE_SIZE,
                     "msg_out_header": mod.MessageOutLayout.HEADER_SIZE,
                     "msg_out_server": mod.MessageOutLayout.SERVER_SIZE,
                     "msg_in": mod.MessageInLayout.MESSAGE_SIZE,
                     "ring_index": mod.RingBufferLayout.INDEX_SIZE,
                     "ring_total": mod.RingBufferLayout.TOTAL_SIZE,
                     "total": mod.TOTAL_SHM_SIZE, "max_as": mod.MAX_AS,
                     "ring_slots": mod.RING_BUFFER_SIZE}, "msg_out": [], "msg_in": []}
    cases = [
        (42, 1234567890123456, [0, 1], [{"n_flow_on": 10, "reservoir_features":
                                         [0.1, 0.2, 0.05, 0.11, 0.21, 1.0, 1.5, 0.3, 1.1, 1.6]},
                                        {"n_flow_on": 15, "reservoir_features":
                                         [0.15, 0.25, 0.06, 0.16, 0.26, 1.2, 1.7, 0.4, 1.3, 1.8]}]),
        (7, 99, [0, 2, 3], [{"n_flow_on": 3, "reservoir_features": [1.0] * 10},
                            {"n_flow_on": 0, "reservoir_features": [0.0] * 10},
                            {"n_flow_on": 5, "reservoir_features": [float(i) for i in range(10)]},
                            {"n_flow_on": 9, "reservoir_features": [0.5] * 10}]),
    ]
    for seq, ts, active, stats in cases:
        bitmap = sum(1 << s for s in active)
        b = mod.MessageOutLayout.pack(seq, ts, bitmap, len(active), stats)
        out["msg_out"].append({"sequence_id": seq, "timestamp_us": ts, "active": active,
                               "stats": stats, "hex": b.hex()})
    for seq, w, alias in ((42, [1.0, 1.5, 2.0, 1.2], None),
                          (8, [0.5, 2.0], [(0.7, 1), (1.0, 0)])):
        with mock.patch.object(mod.time, "time", return_value=1700000000.25):
            b = mod.MessageInLayout.pack(seq, w, alias)
        out["msg_in"].append({"sequence_id": seq, "weights": w, "alias": alias,
                              "timestamp_us": int(1700000000.25 * 1e6), "hex": b.hex()})
    with open(os.path.join(HERE, "shm.json"), "w") as fh:
        json.dump(out, fh)
    print("wrote shm.json", out["sizes"])


if __name__ == "__main__":
    main(*sys.argv[1:])
