#!/usr/bin/env python3
"""Golden data of the VPP shared-memory bridge (this container only; the reference never travels).

Imports src/lb/shm_proxy.py IN PLACE (cwd src/lb: the module reads ./shm_layout.json at import)
with its FILE_FMT pointed at a temporary file in /dev/shm, and records -> tests/golden/vpp_shm.npz:

  layout      Shm_Manager.ptrs: start offset, element size and count of every layout field
              (shm.h:85-91 as the agent maps it) and the struct sizes
  frames      msg_out frames + raw res_as reservoirs written here with the reference's own
              offsets and struct formats (as VPP's stats.c would), several sequence ids in the
              4-frame ring; what Shm_Manager.get_latest_frame() returns for them: the newest
              sequence id, active_as and feature_as [64, 11] f64 (process_reservoir's features)
  msg_in      the bytes Shm_Manager.register_as_weights / register_as_alias write (time.time()
              fixed, so the f32 ts field is deterministic), for several weight vectors
"""
import importlib.util
import json
import os
import struct
import sys
from unittest import mock

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
FIXED_TIME = 1700000000.25


def load_shm_proxy(root):
    src = os.path.join(root, "src/lb")
    cwd = os.getcwd()
    os.chdir(src)
    try:
        spec = importlib.util.spec_from_file_location("ref_shm_proxy", os.path.join(src, "shm_proxy.py"))
        mod = importlib.util.module_from_spec(spec)
        spec.loader.exec_module(mod)
    finally:
        os.chdir(cwd)
    return mod


def reservoir_case(rng, kind, ts):
    """(2, 128, 2) f32 (t, v) pairs of one AS."""
    tv = np.zeros((2, 128, 2), np.float32)
    if kind == "full":
        n = 128
    elif kind == "partial":
        n = int(rng.integers(1, 128))
    else:  # "empty"
        return tv
    for r in range(2):
        slots = rng.permutation(128)[:n]  # VPP writes rand() % 128 slots
        t = ts - rng.exponential(3.0, n)
        v = rng.lognormal(-1.5, 1.0, n)
        if kind == "full" and r == 0:
            v[:3] = [-12.5, 0.0, 41.0]  # a timed-out flow's guessed fct can be negative
        tv[r, slots, 0] = t.astype(np.float32)
        tv[r, slots, 1] = v.astype(np.float32)
    return tv


def main(root="/root/reference"):
    sm = load_shm_proxy(root)
    path_fmt = "/dev/shm/lbsim_golden_vpp_{}"
    sm.GLOBAL_CONF["global"]["FILE_FMT"] = path_fmt
    path = path_fmt.format(sm.GLOBAL_CONF["global"]["VIP_ID"])
    with open(path, "wb") as f:
        f.write(b"\0" * sm.GLOBAL_CONF["global"]["SHM_SIZE"])
    try:
        mgr = sm.Shm_Manager(sm.CONF_FILE)
        out = {}
        names = [l[1] for l in mgr.layout]
        out["layout_names"] = np.array(names)
        out["layout"] = np.array([[mgr.ptrs[k][0]["mem"][0], mgr.ptrs[k][0]["mem"][1] -
                                   mgr.ptrs[k][0]["mem"][0], len(mgr.ptrs[k])] for k in names])
        out["struct_sizes"] = json.dumps(mgr.struct_sizes)
        out["feature_as_all"] = np.array(sm.FEATURE_AS_ALL)

        rng = np.random.default_rng(2026)
        mem = mgr._mem
        cases = [
            ("seven", [0, 1, 2, 3, 4, 5, 6], ["full"] * 5 + ["partial", "full"], [1, 2, 3, 5]),
            ("sparse", [1, 5, 17, 40, 63], ["full", "partial", "empty", "full", "partial"], [6, 7]),
            ("wrap", [2, 9, 11, 30], ["partial", "partial", "full", "full"], [8, 9, 10, 11, 12, 13]),
        ]
        for name, active, kinds, seqs in cases:
            ts = float(np.float32(100.0 + 37.5 * len(seqs)))
            res = np.zeros((64, 2, 128, 2), np.float32)
            for a, k in zip(active, kinds):
                res[a] = reservoir_case(rng, k, ts)
            # res_as: the reference's own element offsets and format
            for a in range(64):
                p = mgr.ptrs["res_as"][a]
                mem[p["mem"][0]:p["mem"][1]] = struct.pack(p["type"], *res[a].reshape(-1).tolist())
            b_header = 0
            for a in active:
                b_header |= 1 << (63 - a)
            nflow = np.zeros(64, np.int32)
            nflow[active] = rng.integers(0, 40, len(active))
            body = []
            for a in range(64):
                body += [a, int(nflow[a])]
            frames = []
            for k, sid in enumerate(seqs):  # VPP publishes in order: the last is the newest
                p = mgr.ptrs["msg_out_frames"][sid & 3]
                fts = ts if k == len(seqs) - 1 else ts - 0.2 * (len(seqs) - 1 - k)
                hdr = b_header if k == len(seqs) - 1 else b_header ^ (1 << 0)
                b = struct.pack(p["type"], sid, fts, hdr, *body)
                mem[p["mem"][0]:p["mem"][1]] = b
                frames.append(b)
            mgr.id_out = seqs[0] - 1  # the agent saw everything before this case's frames
            for a in range(64):
                mgr.stat_last[a]["ts"] = 0
            active_got, feature_as, gt = mgr.get_latest_frame()
            ring = bytes(mem[mgr.ptrs["msg_out_frames"][0]["mem"][0]:
                             mgr.ptrs["msg_out_frames"][3]["mem"][1]])
            out[f"{name}_res"] = res[active]
            out[f"{name}_active"] = np.array(active)
            out[f"{name}_seqs"] = np.array(seqs)
            out[f"{name}_ts"] = np.float32(ts)
            out[f"{name}_nflow"] = nflow
            out[f"{name}_ring"] = np.frombuffer(ring, np.uint8)
            out[f"{name}_id_out"] = np.int64(mgr.id_out)
            out[f"{name}_active_got"] = np.array(active_got)
            out[f"{name}_feature_as"] = feature_as

        # msg_in: register_as_weights / register_as_alias bytes, time.time() fixed
        weights_cases = [
            [1.0, 1.0, 1.0, 1.0, 2.0, 2.0, 2.0] + [0.0] * 57,  # shm_layout.json meta weights
            [0.0, 1.5, 0.0, 2.0, 1.0, 0.25] + [0.0] * 56 + [3.0, 0.5],
            list(np.round(rng.uniform(0.1, 10.0, 64), 3).astype(np.float32).astype(float)),
            [0.0] * 64,
        ]
        msg = []
        with mock.patch.object(sm.time, "time", return_value=FIXED_TIME):
            for i, w in enumerate(weights_cases):
                seq = 21 + i
                mgr.register_as_weights(seq, w)
                p = mgr.ptrs["msg_in_frames"][seq & 3]
                msg.append(bytes(mem[p["mem"][0]:p["mem"][1]]))
            alias = [(float(np.float32(0.25 * (j % 4))), (j * 7) % 64) for j in range(64)]
            seq = 40
            mgr.register_as_alias(seq, alias)
            p = mgr.ptrs["msg_in_frames"][seq & 3]
            alias_bytes = bytes(mem[p["mem"][0]:p["mem"][1]])
        out["weights_cases"] = np.array(weights_cases, np.float64)
        out["weights_seqs"] = np.arange(21, 21 + len(weights_cases))
        out["msg_in_weights"] = np.stack([np.frombuffer(b, np.uint8) for b in msg])
        out["alias_table"] = np.array(alias, np.float64)
        out["msg_in_alias"] = np.frombuffer(alias_bytes, np.uint8)
        out["fixed_time"] = np.float64(FIXED_TIME)
        # the whole msg_in ring after these writes (the VPP side must pick the newest, id 40)
        p0, p3 = mgr.ptrs["msg_in_frames"][0], mgr.ptrs["msg_in_frames"][3]
        out["msg_in_ring"] = np.frombuffer(bytes(mem[p0["mem"][0]:p3["mem"][1]]), np.uint8)
        np.savez_compressed(os.path.join(HERE, "vpp_shm.npz"), **out)
        print("wrote vpp_shm.npz:", {k: getattr(v, "shape", None) for k, v in out.items()})
    finally:
        os.unlink(path)


if __name__ == "__main__":
    main(*sys.argv[1:])
