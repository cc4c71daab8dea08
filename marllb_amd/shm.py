"""problem-02 shared-memory wire format: the GPU simulator as a stand-in for a
live VPP load balancer, and the facade's `use_shm=True` path.

Byte-compatible with `simulation-mode/problem-02-shared-memory-ipc/src/shm_layout.py` and
`shm_region.py` (pinned by tests/golden/shm.json, made from the reference packers):

    /dev/shm/<name>:  ring index   u64 write_index + 7 x u64 pad                    64 B
                      msg_out[4]   header '=QQQIIx' + 4 pad (37 B)                 4 x 2853 B
                                   + 64 x {u32 n_flow_on, f32 features[10]}
                      msg_in       '=QQII' + f32 weights[64] + 64 x {f32 prob, u32 alias}   792 B

A msg_out server record is exactly one (11,) observation row (n_flow_on, fct x5, duration x5), so
frames are packed for a whole batch at once with numpy structured arrays (no per-field struct).

ShmRegion      SharedMemoryRegion's API (create / attach / write_observation / read_observation /
               write_action / read_action / close / unlink), same ring semantics (latest slot,
               sequence check, "missed" warning).
ShmPublisher   publishes VecLoadBalanceEnv observations of envs [0, n) to regions <prefix><b> and
               reads their msg_in weights back as actions: the simulator driving any SHM consumer.
"""
from __future__ import annotations

import mmap
import os
import time
import warnings
from typing import Dict, List, Optional

import numpy as np

MAX_AS = 64
RING_SLOTS = 4
NF = 11

OUT_HEADER = np.dtype([("sequence_id", "<u8"), ("timestamp_us", "<u8"), ("active", "<u8"),
                       ("num_active", "<u4"), ("reserved", "<u4"), ("pad", "V5")])
OUT_SERVER = np.dtype([("n_flow_on", "<u4"), ("features", "<f4", (10,))])
MSG_OUT = np.dtype([("hdr", OUT_HEADER), ("srv", OUT_SERVER, (MAX_AS,))])
MSG_IN = np.dtype([("sequence_id", "<u8"), ("timestamp_us", "<u8"), ("num_servers", "<u4"),
                   ("reserved", "<u4"), ("weights", "<f4", (MAX_AS,)),
                   ("alias", [("prob", "<f4"), ("alias", "<u4")], (MAX_AS,))])
RING_INDEX_SIZE = 64
RING_TOTAL = RING_INDEX_SIZE + RING_SLOTS * MSG_OUT.itemsize
TOTAL_SIZE = RING_TOTAL + MSG_IN.itemsize
assert (OUT_HEADER.itemsize, MSG_OUT.itemsize, MSG_IN.itemsize, TOTAL_SIZE) == (37, 2853, 792, 12268)

# problem-02 unpack names (shm_layout.py:138-149); problem-03 reads 'flow_duration_*' (see
# LoadBalanceEnv's SHM path, which maps one onto the other)
FEATURE_KEYS = ["fct_mean", "fct_p90", "fct_std", "fct_mean_decay", "fct_p90_decay",
                "duration_mean", "duration_p90", "duration_std", "duration_mean_decay",
                "duration_p90_decay"]


def shm_path(name: str) -> str:
    return f"/dev/shm/{name}"


def pack_observations(obs: np.ndarray, sequence_id, timestamp_us=None,
                      active: Optional[np.ndarray] = None) -> np.ndarray:
    """(N, S, 11) observation rows -> N msg_out frames.  active: (N, S) bool, default every
    configured server (VPP's bitmap of live application servers)."""
    obs = np.asarray(obs, np.float32)
    n, S, _ = obs.shape
    out = np.zeros(n, MSG_OUT)
    if active is None:
        active = np.ones((n, S), bool)
    bits = (active.astype(np.uint64) << np.arange(S, dtype=np.uint64)[None, :]).sum(1)
    out["hdr"]["sequence_id"] = sequence_id
    out["hdr"]["timestamp_us"] = (int(time.time() * 1e6) if timestamp_us is None
                                  else timestamp_us)
    out["hdr"]["active"] = bits
    out["hdr"]["num_active"] = active.sum(1)
    out["srv"]["n_flow_on"][:, :S] = obs[:, :, 0].astype(np.uint32)
    out["srv"]["features"][:, :S] = obs[:, :, 1:]
    return out


def unpack_observation(frame: np.ndarray) -> Dict:
    """One msg_out frame -> the dict of MessageOutLayout.unpack (shm_layout.py:113-160)."""
    h = frame["hdr"]
    bitmap = int(h["active"])
    stats = {}
    for i in range(MAX_AS):
        if bitmap & (1 << i):
            feats = [float(x) for x in frame["srv"]["features"][i]]
            d = {"n_flow_on": int(frame["srv"]["n_flow_on"][i]), "reservoir_features": feats}
            d.update(zip(FEATURE_KEYS, feats))
            stats[i] = d
    ts = int(h["timestamp_us"])
    return {"sequence_id": int(h["sequence_id"]), "timestamp_us": ts, "timestamp": ts / 1e6,
            "active_as_bitmap": bitmap, "num_active_as": int(h["num_active"]),
            "active_servers": [i for i in range(MAX_AS) if bitmap & (1 << i)],
            "server_stats": stats}


def pack_action(sequence_id: int, weights, alias_table=None, timestamp_us=None) -> np.ndarray:
    """MessageInLayout.pack (shm_layout.py:192-237)."""
    m = np.zeros((), MSG_IN)
    w = list(weights)
    m["sequence_id"] = sequence_id
    m["timestamp_us"] = int(time.time() * 1e6) if timestamp_us is None else timestamp_us
    m["num_servers"] = len(w)
    m["weights"][:len(w)] = w
    for i, (p, a) in enumerate(alias_table or []):
        m["alias"][i] = (p, a)
    return m


class ShmRegion:
    """SharedMemoryRegion (shm_region.py:36-195) on the same bytes."""

    def __init__(self, name: str, mm: mmap.mmap, fd: int, owner: bool = False):
        self.name, self.mm, self.fd, self.owner = name, mm, fd, owner
        self.last_read_seq = 0
        self.last_write_seq = 0
        buf = memoryview(mm)
        self._index = np.frombuffer(buf, "<u8", 8, 0)
        self._ring = np.frombuffer(buf, MSG_OUT, RING_SLOTS, RING_INDEX_SIZE)
        self._msg_in = np.frombuffer(buf, MSG_IN, 1, RING_TOTAL)

    @classmethod
    def create(cls, name: str, size: int = TOTAL_SIZE) -> "ShmRegion":
        path = shm_path(name)
        if os.path.exists(path):
            warnings.warn(f"Shared memory {name} already exists, removing...")
            os.unlink(path)
        fd = os.open(path, os.O_CREAT | os.O_RDWR, 0o666)
        os.ftruncate(fd, size)
        return cls(name, mmap.mmap(fd, size, access=mmap.ACCESS_WRITE), fd, owner=True)

    @classmethod
    def attach(cls, name: str) -> "ShmRegion":
        path = shm_path(name)
        if not os.path.exists(path):
            raise FileNotFoundError(f"Shared memory {name} not found at {path}")
        fd = os.open(path, os.O_RDWR)
        size = os.fstat(fd).st_size
        if size < TOTAL_SIZE:
            os.close(fd)
            raise ValueError(f"{path}: {size} bytes, need {TOTAL_SIZE}")
        return cls(name, mmap.mmap(fd, size, access=mmap.ACCESS_WRITE), fd, owner=False)

    # -- VPP side (the producer) -------------------------------------------------------------
    def write_frame(self, frame: np.ndarray) -> int:
        w = int(self._index[0])
        slot = w % RING_SLOTS
        self._ring[slot] = frame
        self._index[0] = w + 1
        self.last_write_seq = int(frame["hdr"]["sequence_id"])
        return slot

    def write_observation(self, sequence_id: int, timestamp_us: Optional[int] = None,
                          active_servers: Optional[List[int]] = None,
                          server_stats: Optional[Dict] = None) -> int:
        active_servers = active_servers or []
        server_stats = server_stats or {}
        rows = np.zeros((1, MAX_AS, NF), np.float32)
        for i in range(MAX_AS):
            st = server_stats.get(i)
            if st is not None:
                rows[0, i, 0] = st.get("n_flow_on", 0)
                f = list(st.get("reservoir_features", [0.0] * 10))[:10]
                rows[0, i, 1:1 + len(f)] = f
        act = np.zeros((1, MAX_AS), bool)
        act[0, active_servers] = True
        return self.write_frame(pack_observations(rows, sequence_id, timestamp_us, act)[0])

    def read_action(self) -> Optional[Dict]:
        m = self._msg_in[0]
        seq = int(m["sequence_id"])
        if seq <= self.last_read_seq:
            return None
        self.last_read_seq = seq
        n = int(m["num_servers"])
        ts = int(m["timestamp_us"])
        return {"sequence_id": seq, "timestamp_us": ts, "timestamp": ts / 1e6, "num_servers": n,
                "weights": [float(x) for x in m["weights"][:n]],
                "alias_table": [(float(p), int(a)) for p, a in m["alias"][:n]]}

    # -- RL side (the consumer) --------------------------------------------------------------
    def latest_frame(self) -> Optional[np.ndarray]:
        w = int(self._index[0])
        return None if w == 0 else self._ring[(w - 1) % RING_SLOTS].copy()

    def read_observation(self, slot: Optional[int] = None) -> Optional[Dict]:
        w = int(self._index[0])
        if w == 0:
            return None
        frame = self._ring[(w - 1) % RING_SLOTS if slot is None else slot].copy()
        obs = unpack_observation(frame)
        if obs["sequence_id"] <= self.last_read_seq:
            return None
        if obs["sequence_id"] > self.last_read_seq + 1:
            warnings.warn(f"Missed {obs['sequence_id'] - self.last_read_seq - 1} observations")
        self.last_read_seq = obs["sequence_id"]
        return obs

    def write_action(self, sequence_id: int, weights, alias_table=None) -> None:
        self._msg_in[0] = pack_action(sequence_id, weights, alias_table)
        self.last_write_seq = sequence_id

    def close(self) -> None:
        if self.mm is not None:
            self._index = self._ring = self._msg_in = None
            self.mm.close()
            self.mm = None
        if self.fd >= 0:
            os.close(self.fd)
            self.fd = -1

    def unlink(self) -> None:
        if os.path.exists(shm_path(self.name)):
            os.unlink(shm_path(self.name))

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()
        if self.owner:
            self.unlink()

    def __del__(self):
        try:
            self.close()
            if self.owner:
                self.unlink()
        except Exception:
            pass


class ShmPublisher:
    """Serve the first `n` envs of a VecLoadBalanceEnv as SHM regions <prefix><b>: publish() writes
    each env's current observation as a msg_out frame; poll_actions() returns the msg_in weights
    written since the last poll (NaN rows where none arrived) for the env's next step."""

    def __init__(self, env, prefix: str, n: Optional[int] = None):
        self.env = env
        self.n = int(n if n is not None else env.num_envs)
        self.S = env.num_servers
        if self.S > MAX_AS:
            raise ValueError(f"at most {MAX_AS} servers per region")
        self.regions = [ShmRegion.create(f"{prefix}{b}") for b in range(self.n)]
        self.seq = 0

    def publish(self, obs) -> None:
        rows = obs[:self.n].detach().cpu().numpy() if hasattr(obs, "detach") else np.asarray(obs)
        self.seq += 1
        frames = pack_observations(rows, self.seq)
        for r, f in zip(self.regions, frames):
            r.write_frame(f)

    def poll_actions(self) -> np.ndarray:
        w = np.full((self.n, self.S), np.nan, np.float32)
        for b, r in enumerate(self.regions):
            a = r.read_action()
            if a is not None:
                k = min(self.S, len(a["weights"]))
                w[b, :k] = a["weights"][:k]
        return w

    def close(self) -> None:
        for r in self.regions:
            r.close()
            r.unlink()
        self.regions = []
