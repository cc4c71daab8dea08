"""problem-02 SHM wire format (marllb_amd/shm.py) against the reference packers' bytes
(tests/golden/shm.json, tests/golden/gen_shm.py), and ring semantics through /dev/shm."""
import json
import os
import uuid

import numpy as np
import pytest

from marllb_amd import shm


@pytest.fixture(scope="module")
def g(golden_dir):
    return json.load(open(os.path.join(golden_dir, "shm.json")))


def test_sizes(g):
    s = g["sizes"]
    assert (shm.OUT_HEADER.itemsize, shm.OUT_SERVER.itemsize, shm.MSG_OUT.itemsize) == \
        (s["msg_out_header"], s["msg_out_server"], s["msg_out"])
    assert (shm.MSG_IN.itemsize, shm.RING_INDEX_SIZE, shm.RING_TOTAL, shm.TOTAL_SIZE) == \
        (s["msg_in"], s["ring_index"], s["ring_total"], s["total"])
    assert (shm.MAX_AS, shm.RING_SLOTS) == (s["max_as"], s["ring_slots"])


def test_msg_out_bytes_match_reference(g):
    for c in g["msg_out"]:
        rows = np.zeros((1, shm.MAX_AS, 11), np.float32)
        for i, st in enumerate(c["stats"]):
            rows[0, i, 0] = st["n_flow_on"]
            rows[0, i, 1:] = st["reservoir_features"]
        act = np.zeros((1, shm.MAX_AS), bool)
        act[0, c["active"]] = True
        f = shm.pack_observations(rows, c["sequence_id"], c["timestamp_us"], act)
        assert f.tobytes().hex() == c["hex"]
        d = shm.unpack_observation(np.frombuffer(bytes.fromhex(c["hex"]), shm.MSG_OUT)[0])
        assert d["active_servers"] == c["active"] and d["sequence_id"] == c["sequence_id"]


def test_msg_in_bytes_match_reference(g):
    for c in g["msg_in"]:
        m = shm.pack_action(c["sequence_id"], c["weights"], c["alias"], c["timestamp_us"])
        assert m.tobytes().hex() == c["hex"]


def test_region_ring_round_trip():
    name = f"lbsim_test_{uuid.uuid4().hex[:8]}"
    with shm.ShmRegion.create(name) as prod:
        cons = shm.ShmRegion.attach(name)
        assert cons.read_observation() is None
        for seq in range(1, 7):  # wraps the 4-slot ring
            prod.write_observation(seq, 1000 + seq, [0, 2],
                                   {0: {"n_flow_on": seq, "reservoir_features": [0.5] * 10},
                                    2: {"n_flow_on": 1, "reservoir_features": [1.0] * 10}})
        with pytest.warns(UserWarning, match="Missed 5 observations"):  # shm_region.py:131-134
            o = cons.read_observation()
        assert o["sequence_id"] == 6 and o["active_servers"] == [0, 2]
        assert o["server_stats"][0]["n_flow_on"] == 6 and o["server_stats"][0]["fct_p90"] == 0.5
        assert cons.read_observation() is None  # not newer
        cons.write_action(6, [1.0, 2.0, 0.5], [(0.7, 1), (1.0, 0), (1.0, 0)])
        a = prod.read_action()
        assert a["weights"] == [1.0, 2.0, 0.5] and a["alias_table"][0][1] == 1
        assert prod.read_action() is None
        cons.close()
    assert not os.path.exists(shm.shm_path(name))
