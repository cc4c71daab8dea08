"""The VPP load balancer's shared-memory bridge: the simulator in place of a
live VPP LB, and the agent side computing its features on the GPU.

Byte-compatible with the reference's data plane and agent:
  layout      src/vpp/lb/shm.h:5-91 (packed structs, stats.h:97-102), mapped as stats.c:67-114
  VPP side    stats.c:147-157 shm_memcpy_frame_out (frame copied with the cache's id 0, the new
              sequence id written LAST), stats.c:159-180 shm_memcpy_frame_in (newest msg_in frame
              by walking the 4-frame ring), stats.c:58-65 shm_as_clear_cache, the b_header bit of
              AS i = 1 << (63 - i) (stats.h:58-61)
  agent side  src/lb/shm_proxy.py:170-743 Shm_Manager: get_latest_frame / parse_frame_out ->
              (active_as, feature_as [64, 11] f64, gt), register_as_weights / register_as_alias
              (frame first, sequence id last), process_reservoir's features (lbsim_vpp_features)

/dev/shm/shm_vip_<id> (1 MiB), packed from SHM_OFFSET = 42 (offsets pinned against the reference's
own Shm_Manager.ptrs by tests/golden/vpp_shm.npz):

    u8               n_as                  @ 42
    msg_out_t        msg_out_cache         @ 43      {u32 id, f32 ts, u64 b_header, as_stat_t[64]}  528 B
    msg_out_t        msg_out_frames[4]     @ 571
    reservoir_as_t   res_as[64]            @ 2683    {tv_pair_f fct[128], flow_duration[128]}  2048 B
    msg_in_t         msg_in_cache          @ 133755  {u32 id, f32 ts, f32 score[64], alias_t[64]} 776 B
    msg_in_t         msg_in_frames[4]      @ 134531  (ends at 137635)

Classes:
  VipShm        the mapped region (create / attach / close / unlink) with numpy views of every field
  VppDataPlane  the VPP side of stats.c on a region: publish() a frame, pull_frame_in()
  ShmManager    the agent side, Shm_Manager's method names and return values; the reservoir
                features run on the GPU (lbsim_vpp_features), alias tables through lbsim_alias_tables
  VppPublisher  envs [0, n) of a VecLoadBalanceEnv as n live VPP LBs: each step the simulator's
                raw reservoirs (lbsim_vpp_export), n_flow_on and active bitmap go out as frames, and
                the agents' msg_in scores come back as the envs' next weights
"""
from __future__ import annotations

import ctypes
import mmap
import os
import time
from typing import List, Optional, Sequence, Tuple

import numpy as np

from . import _lib

SHM_SIZE = 1048576
SHM_OFFSET = 42
SHM_N_BIN = 64
SHM_N_FRAME = 4
SHM_FRAME_MASK = 3
VIP_ID = 1
SHM_UPT_DT = 0.2
RESERVOIR_N_BIN = 128
FILE_FMT = "/dev/shm/shm_vip_{}"
RES_DECAY = 0.9  # shm_proxy.py:150

AS_STAT = np.dtype([("as_index", "<u4"), ("n_flow_on", "<i4")])
TV_PAIR_F = np.dtype([("t", "<f4"), ("v", "<f4")])
RESERVOIR_AS = np.dtype([("fct", TV_PAIR_F, (RESERVOIR_N_BIN,)),
                         ("flow_duration", TV_PAIR_F, (RESERVOIR_N_BIN,))])
ALIAS = np.dtype([("odd", "<f4"), ("alias", "<u4")])
MSG_OUT = np.dtype([("id", "<u4"), ("ts", "<f4"), ("b_header", "<u8"),
                    ("body", AS_STAT, (SHM_N_BIN,))])
MSG_IN = np.dtype([("id", "<u4"), ("ts", "<f4"), ("score", "<f4", (SHM_N_BIN,)),
                   ("weights", ALIAS, (SHM_N_BIN,))])
assert (MSG_OUT.itemsize, RESERVOIR_AS.itemsize, MSG_IN.itemsize) == (528, 2048, 776)

# lb_foreach_layout (shm.h:85-91), in order
LAYOUT = [("n_as", np.dtype("u1"), 1), ("msg_out_cache", MSG_OUT, 1),
          ("msg_out_frames", MSG_OUT, SHM_N_FRAME), ("res_as", RESERVOIR_AS, SHM_N_BIN),
          ("msg_in_cache", MSG_IN, 1), ("msg_in_frames", MSG_IN, SHM_N_FRAME)]
OFFSETS = {}
_off = SHM_OFFSET
for _name, _dt, _n in LAYOUT:
    OFFSETS[_name] = _off
    _off += _dt.itemsize * _n
LAYOUT_END = _off
assert LAYOUT_END <= SHM_SIZE

# shm_proxy.py:22-23: the agent reads ./shm_layout.json; its "global" section is shm.h's defines
CONF_FILE = "./shm_layout.json"
GLOBAL_CONF = {"global": {"SHM_SIZE": SHM_SIZE, "SHM_OFFSET": SHM_OFFSET, "SHM_N_BIN": SHM_N_BIN,
                          "SHM_N_FRAME": SHM_N_FRAME, "SHM_FRAME_MASK": SHM_FRAME_MASK,
                          "VIP_ID": VIP_ID, "SHM_UPT_DT": SHM_UPT_DT,
                          "RESERVOIR_N_BIN": RESERVOIR_N_BIN, "FILE_FMT": "/dev/shm/shm_vip_{}"}}

# shm_proxy.py:151-155
FEATURE_AS_CNT = ["n_flow_on"]
FEATURE_AS_CNT_C: List[str] = []
FEATURE_AS_RES = ["fct", "flow_duration"]
RES_FEATURE_ENG = ["avg", "90", "std", "avg_decay", "90_decay"]
FEATURE_AS_ALL = FEATURE_AS_CNT + ["_".join((a, b)) for a in FEATURE_AS_RES for b in RES_FEATURE_ENG]


def as_bit(asid: int) -> int:
    """SetBit(var, asid) of stats.h:59: AS i is bit 63 - i of b_header."""
    return 1 << (SHM_N_BIN - asid - 1)


def active_from_header(b_header: int) -> List[int]:
    """get_active_as (shm_proxy.py:474-485): the '1' positions of b_header's 64-bit string."""
    bits = format(int(b_header), f"0{SHM_N_BIN}b")
    return [i for i, v in enumerate(bits) if v == "1"]


def header_from_active(active: Sequence[int]) -> int:
    h = 0
    for a in active:
        h |= as_bit(int(a))
    return h


def _torch():
    import torch
    return torch


def gen_alias(weights, device=None) -> List[Tuple[float, int]]:
    """gen_alias (shm_proxy.py:127-146) of a list of weights > 0 -- what register_as_weights
    hands it -- on the GPU (lbsim_alias_tables: the reference's float64 arithmetic on the float32
    weights): [(odd, alias)] per weight, odd rounded to the float32 the wire carries."""
    torch = _torch()
    w = np.asarray(weights, np.float32).reshape(1, -1)
    n = w.shape[1]
    if n == 0:
        return []
    if n > _lib.MAX_SERVERS:
        raise ValueError(f"at most {_lib.MAX_SERVERS} weights")
    dev = torch.device(device if device is not None else "cuda")
    wd = torch.from_numpy(w).to(dev)
    odd = torch.empty((1, n), dtype=torch.float32, device=dev)
    ali = torch.empty((1, n), dtype=torch.int32, device=dev)
    act = torch.empty((1, n), dtype=torch.int32, device=dev)
    stream = ctypes.c_void_p(torch.cuda.current_stream(dev).cuda_stream)
    _lib.check(_lib.load().lbsim_alias_tables(
        ctypes.c_void_p(wd.data_ptr()), 1, n, ctypes.c_void_p(odd.data_ptr()),
        ctypes.c_void_p(ali.data_ptr()), ctypes.c_void_p(act.data_ptr()), stream))
    return [(float(o), int(a)) for o, a in zip(odd.cpu().numpy()[0], ali.cpu().numpy()[0])]


class VipShm:
    """One mapped /dev/shm/shm_vip_<id> region (stats.c:67-114) with numpy views of its fields."""

    def __init__(self, path: str, mm: mmap.mmap, fd: int, owner: bool):
        self.path, self.mm, self.fd, self.owner = path, mm, fd, owner
        buf = memoryview(mm)
        for name, dt, n in LAYOUT:
            setattr(self, name, np.frombuffer(buf, dt, n, OFFSETS[name]))

    @classmethod
    def create(cls, vip_id: int = VIP_ID, path: Optional[str] = None) -> "VipShm":
        """shm_open(O_CREAT) + ftruncate(SHM_SIZE) + mmap (stats.c:72-87); a fresh file is zeros."""
        path = path or FILE_FMT.format(vip_id)
        fd = os.open(path, os.O_CREAT | os.O_RDWR, 0o666)
        os.ftruncate(fd, SHM_SIZE)
        return cls(path, mmap.mmap(fd, SHM_SIZE, mmap.MAP_SHARED,
                                   mmap.PROT_READ | mmap.PROT_WRITE), fd, owner=True)

    @classmethod
    def attach(cls, vip_id: int = VIP_ID, path: Optional[str] = None) -> "VipShm":
        path = path or FILE_FMT.format(vip_id)
        fd = os.open(path, os.O_RDWR)
        if os.fstat(fd).st_size < SHM_SIZE:
            os.close(fd)
            raise ValueError(f"{path}: smaller than SHM_SIZE = {SHM_SIZE}")
        return cls(path, mmap.mmap(fd, SHM_SIZE, mmap.MAP_SHARED,
                                   mmap.PROT_READ | mmap.PROT_WRITE), fd, owner=False)

    def close(self) -> None:
        if self.mm is not None:
            for name, _, _ in LAYOUT:
                setattr(self, name, None)
            self.mm.close()
            self.mm = None
        if self.fd >= 0:
            os.close(self.fd)
            self.fd = -1

    def unlink(self) -> None:
        if os.path.exists(self.path):
            os.unlink(self.path)

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()
        if self.owner:
            self.unlink()


class VppDataPlane:
    """The VPP plugin's side of a region (stats.c): init, frame publication, msg_in pickup."""

    def __init__(self, shm: VipShm):
        self.shm = shm
        # shm_vip_init_mem (stats.c:104-110)
        shm.n_as[0] = SHM_N_BIN
        shm.msg_in_cache["id"][0] = 0
        self.id_out = 0

    @property
    def cache(self):
        return self.shm.msg_out_cache[0]

    def set_active(self, asid: int, on: bool = True) -> None:
        h = int(self.shm.msg_out_cache["b_header"][0])
        h = (h | as_bit(asid)) if on else (h & ~as_bit(asid) & (2 ** 64 - 1))
        self.shm.msg_out_cache["b_header"][0] = h

    def clear_as(self, asid: int) -> None:
        """shm_as_clear_cache (stats.c:58-65): default as_stat and alias, score 0, bit muted."""
        self.shm.msg_out_cache["body"][0, asid] = (0, 0)
        self.shm.msg_in_cache["weights"][0, asid] = (1.0, 0)
        self.shm.msg_in_cache["score"][0, asid] = 0.0
        self.set_active(asid, False)

    def publish(self, time_now: float) -> int:
        """shm_memcpy_frame_out (stats.c:147-157): frame <- cache (id 0 = locked), then the
        sequence id last.  Returns the sequence id."""
        self.id_out += 1
        seq = self.id_out
        frame = self.shm.msg_out_frames[seq & SHM_FRAME_MASK:(seq & SHM_FRAME_MASK) + 1]
        self.shm.msg_out_cache["ts"][0] = np.float32(time_now)
        frame[:] = self.shm.msg_out_cache  # cache id is always 0
        frame["id"][0] = seq
        return seq

    def pull_frame_in(self) -> bool:
        """shm_memcpy_frame_in (stats.c:159-180): walk the msg_in ring from the cache's id to the
        newest frame; copy it into msg_in_cache if newer.  Returns whether the cache changed."""
        frames = self.shm.msg_in_frames
        base = int(self.shm.msg_in_cache["id"][0])
        cur = int(base)
        fid = (cur + 1) & SHM_FRAME_MASK
        best = fid
        sid = int(frames["id"][fid])
        while sid > cur:
            cur = sid
            best = fid
            fid = (sid + 1) & SHM_FRAME_MASK
            sid = int(frames["id"][fid])
        if cur > base:
            self.shm.msg_in_cache[:] = frames[best:best + 1]
            return True
        return False


class ShmManager:
    """Shm_Manager (src/lb/shm_proxy.py:170-743) on the GPU: same methods and return values, the
    reservoir features computed by lbsim_vpp_features.  A 'frame' is a msg_out_frames index."""

    def __init__(self, conf_file=None, verbose=False, verbose_debug=False, gt=False, *,
                 vip_id: int = VIP_ID, path: Optional[str] = None, device=None,
                 shm: Optional[VipShm] = None):
        if gt:
            raise NotImplementedError("gt=True queries the AS hosts over TCP (out of scope)")
        torch = _torch()
        self.device = torch.device(device if device is not None else "cuda")
        self.shm = shm if shm is not None else VipShm.attach(vip_id, path)
        self.id_out = 0
        self.id_in = 0
        self.frame_mask = SHM_FRAME_MASK
        self.shm_size, self.shm_offset = SHM_SIZE, SHM_OFFSET
        self.shm_n_bin, self.res_n_bin = SHM_N_BIN, RESERVOIR_N_BIN
        self.stat_last = {a: {"as_index": 0, "n_flow_on": 0, "ts": 0} for a in range(SHM_N_BIN)}
        self.active_ass: List[int] = []
        self.gt = False
        self.verbose, self.verbose_debug = verbose, verbose_debug
        self._lib = _lib.load()

    def _stream(self):
        return ctypes.c_void_p(_torch().cuda.current_stream(self.device).cuda_stream)

    # -- reading msg_out
    def clear_shm(self) -> None:
        self.shm.mm[:] = b"0" * SHM_SIZE  # shm_proxy.py:416-421 writes ASCII '0's

    def get_frame_sid_out(self, fid: int) -> int:
        assert 0 <= fid < SHM_N_FRAME
        return int(self.shm.msg_out_frames["id"][fid])

    def get_field_from_frame(self, frame: int, field: str, _id: int = 0):
        f = self.shm.msg_out_frames[frame]
        if field == "body":
            return {"as_index": int(f["body"][_id]["as_index"]),
                    "n_flow_on": int(f["body"][_id]["n_flow_on"])}
        if field == "ts":
            return float(f["ts"])
        return int(f[field])

    def get_active_as(self, frame: int, debug=False) -> List[int]:
        return active_from_header(self.shm.msg_out_frames["b_header"][frame])

    def get_active_as_all(self, frame: int) -> List[int]:
        return [int(c) for c in format(int(self.shm.msg_out_frames["b_header"][frame]),
                                       f"0{SHM_N_BIN}b")]

    def process_as_stat(self, frame: int, asid: int, ts: float) -> np.ndarray:
        """shm_proxy.py:497-516: the counter features (n_flow_on; no accumulated counters)."""
        st = self.get_field_from_frame(frame, "body", asid)
        assert ts >= self.stat_last[asid]["ts"]
        st["ts"] = ts
        res = np.array([st[f] - self.stat_last[asid][f] if f in FEATURE_AS_CNT_C else st[f]
                        for f in FEATURE_AS_CNT], np.float64)
        self.stat_last[asid] = st
        return res

    def reservoir_features(self, asids: Sequence[int], ts: float) -> np.ndarray:
        """process_reservoir of several ASes in one launch -> [len(asids), 10] f64."""
        torch = _torch()
        asids = list(asids)
        if not asids:
            return np.zeros((0, 10), np.float64)
        raw = np.ascontiguousarray(self.shm.res_as[asids]).view(np.float32)
        tv = torch.from_numpy(raw.reshape(-1)).to(self.device)
        tsd = torch.tensor([ts], dtype=torch.float32, device=self.device)
        out = torch.empty((2 * len(asids), 5), dtype=torch.float64, device=self.device)
        _lib.check(self._lib.lbsim_vpp_features(
            ctypes.c_void_p(tv.data_ptr()), ctypes.c_void_p(tsd.data_ptr()), 2 * len(asids),
            2 * len(asids), RES_DECAY, ctypes.c_void_p(out.data_ptr()), self._stream()))
        return out.cpu().numpy().reshape(len(asids), 10)

    def process_reservoir(self, asid: int, ts: float) -> np.ndarray:
        return self.reservoir_features([asid], ts)[0]

    def parse_frame_out(self, frame: int) -> Tuple[List[int], np.ndarray, None]:
        """shm_proxy.py:602-618 -> (active_as, feature_as [64, 11] f64, gt=None)."""
        self.active_ass = self.get_active_as(frame)
        ts = self.get_field_from_frame(frame, "ts")
        feature_as = np.zeros((SHM_N_BIN, len(FEATURE_AS_ALL)))
        feats = self.reservoir_features(self.active_ass, ts)
        for k, asid in enumerate(self.active_ass):
            feature_as[asid] = np.concatenate((self.process_as_stat(frame, asid, ts), feats[k]))
        return self.active_ass, feature_as, None

    def get_latest_sid_out(self) -> int:
        sid = self.get_frame_sid_out((self.id_out + 1) & self.frame_mask)
        while self.id_out < sid:
            self.id_out = sid
            sid = self.get_frame_sid_out((self.id_out + 1) & self.frame_mask)
        return self.id_out

    def get_current_active_as(self):
        sid = self.get_latest_sid_out()
        return self.get_active_as(sid & self.frame_mask), sid

    def get_latest_frame(self):
        """shm_proxy.py:691-714: walk the ring to the newest frame and parse it."""
        self.get_latest_sid_out()
        return self.parse_frame_out(self.id_out & self.frame_mask)

    # -- writing msg_in
    def _write_in(self, seq_id: int, score, alias) -> None:
        slot = seq_id & self.frame_mask
        m = np.zeros(1, MSG_IN)
        m["ts"] = time.time()
        m["score"][0] = np.asarray(score, np.float32)
        m["weights"][0]["odd"] = [a[0] for a in alias]
        m["weights"][0]["alias"] = [a[1] for a in alias]
        self.shm.msg_in_frames[slot:slot + 1] = m  # id 0 first ...
        self.shm.msg_in_frames["id"][slot] = seq_id  # ... then the lock: the sequence id

    def register_as_alias(self, seq_id: int, alias) -> None:
        """shm_proxy.py:620-633: scores 0, the given alias tuples."""
        self._write_in(seq_id, [0.0] * SHM_N_BIN, alias)

    def alias_of(self, weights) -> List[Tuple[float, int]]:
        """register_as_weights's table (shm_proxy.py:643-651): gen_alias over the weights > 0
        (lbsim_alias_tables, float32 weights as on the wire), scattered to their ASes."""
        torch = _torch()
        w = np.asarray(weights, np.float32).reshape(1, SHM_N_BIN)
        wd = torch.from_numpy(w).to(self.device)
        odd = torch.empty((1, SHM_N_BIN), dtype=torch.float32, device=self.device)
        ali = torch.empty((1, SHM_N_BIN), dtype=torch.int32, device=self.device)
        act = torch.empty((1, SHM_N_BIN), dtype=torch.int32, device=self.device)
        _lib.check(self._lib.lbsim_alias_tables(
            ctypes.c_void_p(wd.data_ptr()), 1, SHM_N_BIN, ctypes.c_void_p(odd.data_ptr()),
            ctypes.c_void_p(ali.data_ptr()), ctypes.c_void_p(act.data_ptr()), self._stream()))
        odd, ali, act = odd.cpu().numpy()[0], ali.cpu().numpy()[0], act.cpu().numpy()[0]
        table = [(1.0, 0)] * SHM_N_BIN
        for k in range(SHM_N_BIN):
            if act[k] >= 0:
                table[int(act[k])] = (float(odd[k]), int(ali[k]))
        return table

    def register_as_weights(self, seq_id: int, weights) -> None:
        """shm_proxy.py:635-669: scores = weights, alias = gen_alias of the weights > 0."""
        self._write_in(seq_id, weights, self.alias_of(weights))

    def close(self) -> None:
        self.shm.close()


class VppPublisher:
    """Envs [0, n) of a VecLoadBalanceEnv served as n VPP load balancers (one region each, path
    `path_fmt.format(b)`): publish() writes each env's raw reservoirs, n_flow_on and active bitmap
    and publishes a frame (stats.c:147-157); poll_actions() picks up the agents' msg_in frames
    (stats.c:159-180) and returns their scores as the envs' weights (NaN where none arrived), the
    SED weights node.c:393-404 reads."""

    def __init__(self, env, path_fmt: str = "/dev/shm/lbsim_vip_{}", n: Optional[int] = None):
        self.env = env
        self.n = int(n if n is not None else env.num_envs)
        self.S = env.num_servers
        if self.S > SHM_N_BIN:
            raise ValueError(f"at most {SHM_N_BIN} servers per VIP")
        self.paths = [path_fmt.format(b) for b in range(self.n)]
        self.planes = [VppDataPlane(VipShm.create(path=p)) for p in self.paths]
        hdr = header_from_active(range(self.S))
        for dp in self.planes:
            dp.shm.msg_out_cache["b_header"][0] = hdr
            dp.shm.msg_out_cache["body"][0, :self.S] = [(s, 0) for s in range(self.S)]
            dp.shm.msg_in_cache["score"][0, :self.S] = 1.0  # shm.h:52 default score

    def export(self):
        """lbsim_vpp_export of envs [0, n) -> (tv [n, S, 2, 128, 2] f32, n_flow_on [n, S], ts [n])."""
        torch = _torch()
        dev, h = self.env.device, self.env.handle
        tv = torch.empty((self.n, self.S, 2, RESERVOIR_N_BIN, 2), dtype=torch.float32, device=dev)
        nf = torch.empty((self.n, self.S), dtype=torch.int32, device=dev)
        ts = torch.empty(self.n, dtype=torch.float32, device=dev)
        stream = ctypes.c_void_p(torch.cuda.current_stream(dev).cuda_stream)
        h.check(h.lib.lbsim_vpp_export(h.h, 0, self.n, ctypes.c_void_p(tv.data_ptr()),
                                       ctypes.c_void_p(nf.data_ptr()),
                                       ctypes.c_void_p(ts.data_ptr()), stream))
        return tv.cpu().numpy(), nf.cpu().numpy(), ts.cpu().numpy()

    def publish(self) -> List[int]:
        tv, nf, ts = self.export()
        seqs = []
        for b, dp in enumerate(self.planes):
            dp.shm.res_as[:self.S] = tv[b].reshape(-1).view(RESERVOIR_AS)
            dp.shm.msg_out_cache["body"]["n_flow_on"][0, :self.S] = nf[b]
            seqs.append(dp.publish(float(ts[b])))
        return seqs

    def poll_actions(self) -> np.ndarray:
        w = np.full((self.n, self.S), np.nan, np.float32)
        for b, dp in enumerate(self.planes):
            if dp.pull_frame_in():
                w[b] = dp.shm.msg_in_cache["score"][0, :self.S]
        return w

    def close(self) -> None:
        for dp in self.planes:
            dp.shm.close()
            dp.shm.unlink()
        self.planes = []
