"""Snapshot layout of lbsim device state — shared by liblbsim and the oracle."""
import numpy as np

K, NF = 128, 11


def sections(B, S, Q, normalize, failures=False, leak=False, dur_plane=False, split_P=0):
    """split_P > 0: a lost-FIN handle (split fct / duration reservoirs) with
    lost_fin_pending = split_P: {duration us, ts ms} records, the duration count, the pending
    guesses' ring words and entries {due us, guess us}, lf_over."""
    BS = B * S
    out = [("next_arr", np.int32, B), ("next_work", np.float32, B), ("next_u2", np.uint32, B),
           ("next_u3", np.uint32, B), ("arr_idx", np.uint32, B), ("episode", np.uint32, B),
           ("clock", np.uint32, B), ("ep_step", np.int32, B), ("dropped", np.uint32, B),
           ("norm_count", np.int32, B), ("ep_return", np.float64, B), ("hc", np.uint32, BS),
           ("last_tc", np.int32, BS), ("res_count", np.uint32, BS), ("ring", np.int32, BS * Q * 2),
           ("res", np.uint32, BS * K * 2), ("chg", np.uint32, BS * 4), ("fcache", np.float32, BS * 10)]
    if normalize:
        out += [("norm_mean", np.float64, BS * NF), ("norm_std", np.float64, BS * NF)]
    if failures:
        out += [("down", np.uint32, BS)]
    if leak:  # n_flow_on_mode "vpp" with lost-FIN: lost flows per server
        out += [("lost_on", np.uint32, BS)]
    if split_P:
        out += [("res_dur2", np.uint32, BS * K * 2), ("res_count_dur", np.uint32, BS),
                ("pend_hc", np.uint32, BS), ("pend", np.uint32, BS * split_P * 2),
                ("lf_over", np.uint32, B)]
    elif dur_plane:  # duration_mode "service": the duration of each slot
        out += [("res_dur", np.uint32, BS * K)]
    return out


def has_dur_plane(cfg) -> bool:
    return cfg.duration_mode == 1 or cfg.lost_fin_prob > 0


def split_p(cfg) -> int:
    """lost_fin_pending of a lost-FIN handle (split reservoirs), else 0."""
    return int(cfg.lost_fin_pending) if cfg.lost_fin_prob > 0 else 0


def has_leak(cfg) -> bool:
    return cfg.n_flow_on_mode == 1 and cfg.lost_fin_prob > 0


def parse(buf: bytes, B, S, Q, normalize, failures=False, leak=False, dur_plane=None, split_P=0):
    """dur_plane None: inferred from the snapshot's size (the plane is the last B*S*K words).
    split_P: see sections (a lost-FIN handle's snapshot)."""
    if dur_plane is None:
        base = sum(np.dtype(dt).itemsize * n for _, dt, n in sections(B, S, Q, normalize, failures, leak))
        dur_plane = len(buf) == base + 4 * B * S * K
    d, off = {}, 0
    for name, dt, n in sections(B, S, Q, normalize, failures, leak, dur_plane, split_P):
        nb = np.dtype(dt).itemsize * n
        d[name] = np.frombuffer(buf[off:off + nb], dtype=dt)
        off += nb
    assert off == len(buf), (off, len(buf))
    rec = d["res"].reshape(-1, 2)  # slot records {fct us, timestamp ms}
    d["res_fct"], d["res_ts"] = rec[:, 0], rec[:, 1]
    if "res_dur2" in d:  # split: the duration reservoir's own {us, ts} records
        r2 = d["res_dur2"].reshape(-1, 2)
        d["res_dur"], d["res_dur_ts"] = r2[:, 0], r2[:, 1]
    elif "res_dur" not in d:  # paired records: the duration reservoir is the fct reservoir
        d["res_dur"] = d["res_fct"]
    return d


def live_pend(d, B, S, P):
    """Pending guesses in their rings (entries past the count are not state), by position from
    the head."""
    hc = d["pend_hc"].reshape(B, S)
    ring = d["pend"].reshape(B, S, P, 2)
    out = np.zeros((B, S, P, 2), np.uint32)
    for b in range(B):
        for s in range(S):
            h, c = int(hc[b, s] & 0xFFFF), int(hc[b, s] >> 16)
            for i in range(c):
                out[b, s, i] = ring[b, s, (h + i) % P]
    return out


def live_ring(d, B, S, Q):
    """Ring entries that are in flight (stale slots beyond the count are not state)."""
    hc = d["hc"].reshape(B, S)
    ring = d["ring"].reshape(B, S, Q, 2)
    live = np.zeros((B, S, Q), bool)
    for b in range(B):
        for s in range(S):
            h, c = int(hc[b, s] & 0x7FFF), int(hc[b, s] >> 16)  # bit 15: the sticky big flag
            for i in range(c):
                live[b, s, (h + i) % Q] = True
    return np.where(live[..., None], ring, 0)
