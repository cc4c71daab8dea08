// lbsim_dyn_wave.h — dynamics with one WAVE per env, for batches too small to fill the chip
// (BASELINE configs[0] 1 x 4, configs[1] at 4096 x 4): there the event loop is one env's dependent
// chain, so the instructions per arrival on that chain, not issue throughput, set the step time.
//
// The server-per-lane kernel (lbsim_dyn_group.h) spends ~150 instructions per event-loop
// iteration: a pop per iteration (extra iterations when two completions fall between arrivals), an
// LDS round trip for the next queue head and one for the next drawn arrival, two DPP reductions,
// the reservoir insert and the draw-ahead refill every G iterations.  Here the whole env is one
// wave and its state is laid out so that an arrival is a short straight-line block:
//   * ring lanes: servers 2g and 2g + 1 own the two 32-lane halves of ring register g (NG = 1, 2
//     or 4 registers each of {t_complete, t_arrival}); ring position pos of server s is register
//     s >> 1, lane 32 (s & 1) + pos, so the HBM ring loads and stores lane for
//     lane.  With FIFO service and arrival times that never decrease, a slot's flow is queued at
//     time t iff its t_complete > t (free slots hold kDead): the pops before an arrival at ta are
//     implicit, and a server's flow count at ta is the popcount of its half of one ballot per
//     register (the oracle's pop_until, lbsim_oracle.c sim_step, however many complete);
//   * the counts for the NEXT arrival are taken while the current one is chosen (its time is
//     known: arrivals are drawn ahead), and with them the keys of both outcomes of the push from a
//     per-step LDS key table (wave_event_loop), so the chain from one choice to the next is a
//     select, one DPP minimum, a ballot of the ties and a find-first-set;
//   * server lanes: lane s < S holds server s's fields (write position, tail, Algorithm R count,
//     SED denominator); the push is a select in ring lane 32 (c & 1) + wp_c and one in lane c;
//   * arrivals: 64 at a time (lane j: arrival base + j, its Philox block, gap and work or its
//     trace row, times by one wave prefix sum); consecutive batches overlap by one arrival (the
//     look-ahead), and the loop reads arrival k with v_readlane (SGPRs): no LDS on the chain;
//   * reservoir inserts are deferred to the end of each batch: every arrival logs its server and
//     completion time in its batch lane; the flush gives each completed flow its Algorithm R count
//     (the server's count + the earlier inserts of the batch into it, a masked bit count), its slot
//     from its arrival's draw word, keeps the LAST insert into each (server, slot) (an LDS
//     atomic max over arrival order) and stores the records in one pass.  Per server the inserts
//     happen in arrival order = FIFO completion order, after the carried-in flows, exactly as
//     the oracle's pops make them.
// Same event sequence, same arithmetic, same state layout as the other two
// mappings: interchangeable between launches, bit-identical to the oracle.  S <= 8 (NG = 1, 2, 4
// ring registers), Q <= 32 and the SED / SED2 / LSQ / LSQ2 policies (ALIAS and larger shapes use
// the group kernel: dyn_wave_ok in lbsim_internal.h).
#pragma once

#include "lbsim_dyn_group.h"

namespace lbk {

// Register g, lane l: ring position l & 31 of server 2g + (l >> 5).  FIFO service and arrival
// times that never decrease make a slot's flow queued at time t iff its t_complete > t: a popped
// flow completed no later than the arrival that popped it, and a free slot holds kDead.  So no
// queue bookkeeping survives between arrivals but the slots themselves.
constexpr int32_t kDead = kLastNone;
template <int NG>
struct WaveRing {
  int32_t tc[NG], ta[NG];
};

// Server lane s (s < S; the other lanes carry inactive copies).
struct WaveSrv {
  int32_t wp;        // ring position of the next push (= head + count mod Q)
  int32_t cnt0;      // flows queued at the start of the step
  int32_t pushed;    // pushes this step
  int32_t tail;      // t_complete of the last pushed flow
  int32_t last;      // t_complete of the last completed flow (kLastNone if none)
  int32_t saved;     // t_complete overwritten by the push that filled the ring (the last popped)
  int32_t assigned;  // arrivals assigned this launch
  uint32_t rcnt;     // Algorithm R count
  float scale;       // 1e6 / mu_s
  double den, rcp;   // SED: w + 1e-9 and its reciprocal
  bool act;
};

// The env's scalars (wave-uniform: SGPRs).
struct WaveEnv {
  uint32_t gid, episode, clock, dropped, arr_idx;
  int32_t next_arr;
  float next_work;
  uint32_t u2, u3;
};

// One batch of drawn arrivals (lane j: arrival base + j) and the log of the processed ones.
struct WaveBatch {
  int32_t ta;     // arrival time (relative us)
  float wk;       // Exp(1) work
  uint32_t u2, u3;
  int32_t lc;     // logged: chosen server (-1: dropped)
  int32_t ltc;    // logged: t_complete of the pushed flow
};

constexpr int kWaveKeyStride = 34;  // key table entries per server: n = 0 .. Q + 1 (Q <= 32)
constexpr int kWaveMaxS = 8;        // servers of the wave kernel (NG = 4 ring registers)
struct WaveLds {
  int32_t kt[kWaveMaxS * kWaveKeyStride];  // FAST single-choice keys of this step [server][n]
                                           // (first: no constant in its address, ds_read2
                                           // offsets are 8-bit)
  int2 img[32 * kWaveMaxS];       // ring image [pos][server] for the carried-in walk and `last`
  uint32_t own[kWaveMaxS * 128];  // insert owner of each (server, slot) in a flush: seq << 6 | lane
  uint32_t chg[4 * kWaveMaxS];    // written-slot masks [word][server]
  uint32_t big[kWaveMaxS];        // the servers' sticky kHcBig flags
};
// Server lanes a reduction / key table covers: 4 for NG <= 2 (S <= 4), 8 for NG = 4 (S <= 8).
template <int NG>
constexpr int kWaveLanesS = NG <= 2 ? 4 : 8;

__device__ __forceinline__ int32_t rdl(int32_t v, int l) { return __builtin_amdgcn_readlane(v, l); }
__device__ __forceinline__ uint32_t rdl(uint32_t v, int l) {
  return (uint32_t)__builtin_amdgcn_readlane((int)v, l);
}
__device__ __forceinline__ float rdl(float v, int l) {
  return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), l));
}
__device__ __forceinline__ uint32_t sat_add(uint32_t a, uint32_t b) {
  const uint32_t s = a + b;
  return s < a ? 0xFFFFFFFFu : s;  // count_inc applied b times
}

// Arrivals base .. base + 63 (lane j: arrival base + j), t0 = the time of arrival base: lane j's
// time is t0 + the gaps of arrivals base + 1 .. base + j (the oracle's draw_arrival chain
// next_arr = t_prev + gap; integer sums, so any order is exact).
template <bool TRACE>
__device__ __forceinline__ void wave_draw_batch(const DevState& st, const SimParams& p,
                                                const WaveEnv& E, uint32_t base, int32_t t0,
                                                int lane, WaveBatch& Bt) {
  const uint32_t k = base + (uint32_t)lane;
  const u32x4 d = philox4x32_10(u32x4{k, E.gid, E.episode, kStreamArrival << 24}, p.key0, p.key1);
  int32_t gap;
  float wk;
  if constexpr (TRACE) {
    const uint32_t r = trace_row(p, E.gid, E.episode, k);
    gap = (int32_t)st.trace_gap[r];
    wk = st.trace_work[r];
  } else {
    gap = (int32_t)(-lb_logf(u01_open0(d.x)) * p.mean_gap_us);
    wk = -lb_logf(u01_open0(d.y));
  }
  // inclusive prefix sum over the wave by DPP: row_shr 1 / 2 / 4 / 8 within each row of 16, then
  // row_bcast:15 and row_bcast:31 carry the row totals (no LDS round trips)
  int32_t t = lane == 0 ? 0 : gap;
  t += __builtin_amdgcn_update_dpp(0, t, 0x111, 0xF, 0xF, false);  // row_shr:1
  t += __builtin_amdgcn_update_dpp(0, t, 0x112, 0xF, 0xF, false);  // row_shr:2
  t += __builtin_amdgcn_update_dpp(0, t, 0x114, 0xF, 0xF, false);  // row_shr:4
  t += __builtin_amdgcn_update_dpp(0, t, 0x118, 0xF, 0xF, false);  // row_shr:8
  t += __builtin_amdgcn_update_dpp(0, t, 0x142, 0xA, 0xF, false);  // row_bcast:15 -> rows 1, 3
  t += __builtin_amdgcn_update_dpp(0, t, 0x143, 0xC, 0xF, false);  // row_bcast:31 -> rows 2, 3
  Bt.ta = t0 + t;
  Bt.wk = wk;
  Bt.u2 = d.z;
  Bt.u3 = d.w;
  Bt.lc = -1;
  Bt.ltc = 0;
}

// Flows of server lane s in the ring-lane masks `live` (its half of register s >> 1).
template <int NG>
__device__ __forceinline__ int32_t wave_count(const uint64_t (&live)[NG], int lane) {
  const bool odd = lane & 1;
  uint32_t w = odd ? (uint32_t)(live[0] >> 32) : (uint32_t)live[0];
#pragma unroll
  for (int g = 1; g < NG; ++g) {
    const uint32_t wg = odd ? (uint32_t)(live[g] >> 32) : (uint32_t)live[g];
    w = ((lane >> 1) & (NG - 1)) == g ? wg : w;
  }
  return __builtin_popcount(w);
}

// The reservoir inserts of batch lanes [0, nproc): flows that completed in this step, per server in
// arrival order (reservoir.py:64-85 with the arrival's draw word, reservoir_slot_r32).
__device__ __forceinline__ void wave_flush(const SimParams& p, WaveSrv& V, WaveEnv& E,
                                           const WaveBatch& Bt, int nproc, int lane,
                                           uint2* const res_b, uint32_t* const dur_b, WaveLds& Ld,
                                           uint32_t seq,
                                           uint32_t base_ms, uint32_t base_rem) {
  const int S = p.S;
  const int32_t dt = p.dt_us;
  const bool valid = lane < nproc && Bt.lc >= 0;
  E.dropped += (uint32_t)__builtin_popcountll(__ballot(lane < nproc && Bt.lc < 0));  // all full
  const bool ins = valid && Bt.ltc <= dt;
  uint32_t pre = 0u, rcb = 0u;
  float scale = p.svc_scale[0];
#pragma unroll
  for (int s = 0; s < kWaveMaxS; ++s) {
    if (s < S) {
      const bool mine = Bt.lc == s;
      const uint64_t m = __ballot(ins && mine);
      const uint32_t below = __mbcnt_hi((uint32_t)(m >> 32), __mbcnt_lo((uint32_t)m, 0u));
      const uint32_t rs = rdl(V.rcnt, s);
      pre = mine ? below : pre;
      rcb = mine ? rs : rcb;
      if (s > 0) scale = mine ? p.svc_scale[s] : scale;
      const uint32_t npush = (uint32_t)__builtin_popcountll(__ballot(valid && mine));
      const bool me = lane == s;
      V.rcnt = me ? sat_add(rs, (uint32_t)__builtin_popcountll(m)) : V.rcnt;
      V.pushed += me ? (int32_t)npush : 0;
      V.assigned += me ? (int32_t)npush : 0;
    }
  }
  const uint32_t cres = sat_add(rcb, pre);  // the count before this insert
  const int slot = ins ? reservoir_slot_r32(cres, Bt.u3) : -1;
  const uint32_t key = (uint32_t)Bt.lc * K + (uint32_t)slot;
  const uint32_t me_tag = (seq << 6) | (uint32_t)lane;
  if (slot >= 0) {
    atomicMax(&Ld.own[key], me_tag);  // the last insert into a slot is the one that stays
    atomicOr(&Ld.chg[((uint32_t)slot >> 5) * kWaveMaxS + (uint32_t)Bt.lc], 1u << (slot & 31));
  }
  wave_sync();
  if (slot >= 0 && Ld.own[key] == me_tag) {
    int32_t svc = (int32_t)(Bt.wk * scale);
    svc = svc < 1 ? 1 : svc;
    const uint32_t fct = lost_fct(p, (uint32_t)(Bt.ltc - Bt.ta),
                                  base_ms * 1000u + base_rem + (uint32_t)Bt.ta, E.gid, E.episode);
    res_b[key] = make_uint2(fct, base_ms + (base_rem + (uint32_t)Bt.ltc) / 1000u);
    // the duration plane (dur_sample): the age ltc - ta, or the service time svc = ltc - start
    if (dur_b != nullptr) dur_b[key] = p.dur_service ? (uint32_t)svc : (uint32_t)(Bt.ltc - Bt.ta);
  }
}

// The arrivals of one step.
//
// FAST single-choice policies (SED / LSQ with finite scores) read their keys from a per-step LDS
// table kt[s][n] = the order key of server s's score at n queued flows (0x7FFFFFFF: full): an
// iteration fetches the keys for both outcomes of its push (n and n + 1 at the next arrival) in
// one ds_read2 before it chooses, and the choice -> choice chain is a select, a DPP minimum and
// a ballot.  SED2 / LSQ2 and non-finite SED compute their scores in the loop.
template <int NG, int POLICY, bool TRACE, bool FAST, bool VC>
__device__ __forceinline__ void wave_event_loop(const DevState& st, const SimParams& p,
                                                WaveEnv& E, WaveSrv& V, WaveRing<NG>& R,
                                                int lane, uint2* const res_b,
                                                uint32_t* const dur_b, WaveLds& Ld,
                                                uint32_t& seq, uint32_t base_ms,
                                                uint32_t base_rem) {
  constexpr bool two_choice = (POLICY == 1 || POLICY == 3);
  constexpr bool lsq = (POLICY == 2 || POLICY == 3);
  constexpr bool TAB = FAST && !two_choice;
  constexpr int KT = kWaveKeyStride;
  const int S = p.S, Q = p.Q;
  const int32_t dt = p.dt_us;
  if (E.next_arr >= dt) return;

  auto score_of = [&](int32_t nn, double den, double rcp) -> float {  // node.c:393-404
    if constexpr (lsq) {
      return (float)nn;
    } else {
      const double c1 = (double)(nn + 1);
      const double q0 = c1 * rcp;
      double q = fma(fma(-q0, den, c1), rcp, q0);
      if (!FAST && q != q) {
        asm volatile("");
        q = c1 / den;
      }
      return (float)q;
    }
  };
  constexpr int LS = kWaveLanesS<NG>;  // server lanes of the reductions
  constexpr int LPS = 64 / LS;         // key-table lanes per server
  const int s4 = lane & (LS - 1);  // the server whose queue count this lane holds
  int32_t* const kt_s = Ld.kt + s4 * KT;
  if constexpr (TAB) {
    // the step's key table: lanes LPS s .. LPS s + LPS - 1 fill server s's entries n = 0 .. Q + 1
    const int ts = lane / LPS;
    const double den = __shfl(V.den, ts, 64), rcp = __shfl(V.rcp, ts, 64);
#pragma unroll
    for (int k = 0; k < (KT + LPS - 1) / LPS; ++k) {
      const int nn = (lane & (LPS - 1)) + LPS * k;
      if (nn < Q + 2)  // servers past S: never eligible
        Ld.kt[ts * KT + nn] = (nn < Q && ts < S) ? f32_key(score_of(nn, den, rcp)) : 0x7FFFFFFF;
    }
    wave_sync();
  }

  // batch 0: lane 0 is the pending arrival (its stored draw), lanes 1..63 the next ones
  uint32_t base = E.arr_idx;
  WaveBatch Bt;
  wave_draw_batch<TRACE>(st, p, E, base, E.next_arr, lane, Bt);
  Bt.wk = lane == 0 ? E.next_work : Bt.wk;
  Bt.u2 = lane == 0 ? E.u2 : Bt.u2;
  Bt.u3 = lane == 0 ? E.u3 : Bt.u3;
  int bi = 0;  // batch lane of the current arrival
  int32_t ta = E.next_arr;

  // server lane s's flows queued at time t, from one ballot per ring register.  VC (the one-launch
  // step, <= 2 envs per SIMD): its half selected per lane and counted by VALU -- the shorter chain,
  // a lone wave's step 2.5 us faster; else the four halves' popcounts by the scalar unit, packed as
  // bytes of one SGPR and unpacked by one v_bfe -- fewer VALU, 2.5 % faster at 4 envs per SIMD
  // (profiles/r03w/ab_wave_counts.txt)
  const uint32_t cnt_sh = (uint32_t)(lane & 3) * 8u;
  auto count_at = [&](int32_t t) -> int32_t {
    uint64_t m[NG];
#pragma unroll
    for (int g = 0; g < NG; ++g) m[g] = __ballot(R.tc[g] > t);
    if constexpr (VC) {
      return wave_count<NG>(m, lane);
    } else {
      uint32_t packed = (uint32_t)__builtin_popcount((uint32_t)m[0]) +
                        ((uint32_t)__builtin_popcount((uint32_t)(m[0] >> 32)) << 8);
      if constexpr (NG > 1)
        packed += ((uint32_t)__builtin_popcount((uint32_t)m[1]) << 16) +
                  ((uint32_t)__builtin_popcount((uint32_t)(m[1] >> 32)) << 24);
      if constexpr (NG > 2) {  // servers 4..7 in a second word
        const uint32_t packed2 = (uint32_t)__builtin_popcount((uint32_t)m[2]) +
                                 ((uint32_t)__builtin_popcount((uint32_t)(m[2] >> 32)) << 8) +
                                 ((uint32_t)__builtin_popcount((uint32_t)m[3]) << 16) +
                                 ((uint32_t)__builtin_popcount((uint32_t)(m[3] >> 32)) << 24);
        packed = (lane & 4) ? packed2 : packed;
      }
      return (int32_t)__builtin_amdgcn_ubfe(packed, cnt_sh, 8u);
    }
  };
  const uint32_t smask = (1u << S) - 1u;  // server lanes
  // push lane of server lane s: ring register (s >> 1) x 64 + lane 32 (s & 1) + write position
  int32_t pl = lane * 32 + V.wp;
  const int32_t pl_wrap = lane * 32 + Q;
  int32_t n = count_at(ta);
  int32_t key = 0;
  float score = 0.f;
  if constexpr (TAB) key = kt_s[n];
  else score = score_of(n, V.den, V.rcp);
  for (;;) {      // batches
    // arrivals bi .. lim - 1 of this batch come before dt (times increase with the lane); lane 63
    // opens the next batch
    // (lim > bi: the batch starts at an arrival before dt)
    const int lim = __builtin_ctzll(__ballot(Bt.ta >= dt) | (1ull << 63));
    do {
      const int32_t ta = rdl(Bt.ta, bi);
      const float work = rdl(Bt.wk, bi);
      const uint32_t u2 = rdl(Bt.u2, bi);
      // ---- look-ahead: the next arrival's queue counts without the flow pushed now, and the
      //      keys / scores for both outcomes (off the choice -> choice chain)
      const int32_t ta_n = rdl(Bt.ta, bi + 1);
      const int32_t n_n = count_at(ta_n);
      int32_t k0 = 0, k1 = 0;
      float sc0 = 0.f, sc1 = 0.f;
      if constexpr (TAB) {
        k0 = kt_s[n_n];
        k1 = kt_s[n_n + 1];
      } else {
        sc0 = score_of(n_n, V.den, V.rcp);
        sc1 = score_of(n_n + 1, V.den, V.rcp);
        // issue them before the choice (the in-order wave would otherwise run them after it)
        asm volatile("" ::"v"(sc0), "v"(sc1));
      }

      // ---- the arrival's server (node.c:388-441); full servers are not eligible
      int c = -1;
      if constexpr (TAB) {
        // finite scores: the eligible minimum, h among equal minima, else the lowest such server
        // (every server full: no eligible tie, and the find-first-set of 0 is -1: dropped)
        const int32_t mk = __builtin_amdgcn_readfirstlane(group_min_i32<LS>(key));
        const uint32_t hbit = 1u << (int)__umulhi(u2, (uint32_t)S);
        const uint32_t tie = (uint32_t)__ballot(key == mk) & (mk != 0x7FFFFFFF ? smask : 0u);
        const uint32_t sel = (tie & hbit) ? hbit : tie;
        c = sel ? __builtin_ctz(sel) : -1;
      } else if constexpr (two_choice) {
        const uint32_t em = (uint32_t)__ballot(n < Q) & smask;
        const int h1 = two_choice_h1(u2, S);
        const int h2 = two_choice_h2(u2, S);
        const float s1 = rdl(score, h1), s2 = rdl(score, h2);
        const bool ok1 = (em >> h1) & 1u, ok2 = (em >> h2) & 1u;
        c = (ok1 && ok2) ? ((s2 < s1) ? h2 : h1) : (ok1 ? h1 : (ok2 ? h2 : -1));
      } else {
        const bool elig = n < Q && lane < S;
        const uint32_t em = (uint32_t)__ballot(n < Q) & smask;
        const bool num = elig && score == score;
        const float m = key_f32(__builtin_amdgcn_readfirstlane(
            group_min_i32<LS>(num ? f32_key(score) : 0x7f800000)));
        const int h = (int)__umulhi(u2, (uint32_t)S);
        const int c0 = ((em >> h) & 1u) ? h : (em ? __builtin_ctz(em) : -1);
        const uint32_t tie = (uint32_t)__ballot(num && score == m) & ((1u << LS) - 1u);
        const uint32_t nan = (uint32_t)__ballot(score != score) & ((1u << LS) - 1u);
        c = c0 < 0 ? -1 : ((((tie | nan) >> c0) & 1u) ? c0 : (tie ? __builtin_ctz(tie) : -1));
      }
      const bool lg = lane == bi;  // this arrival's batch lane (the insert log)

      // ---- FIFO service on server c: every server lane prices the flow (an empty server's tail
      //      completed by ta, so max(tail, ta) is the start either way).  A dropped flow (c = -1:
      //      every server full, rare) runs the same straight line: lane -1 reads lane 63, whose
      //      push lane (>= 128) matches no ring lane, and no lane is `me`.
      int32_t svc_l = (int32_t)(work * V.scale);
      svc_l = svc_l < 1 ? 1 : svc_l;
      const int32_t tc = rdl((V.tail > ta ? V.tail : ta) + svc_l, c);
      const int T = rdl(pl, c);  // ring register x 64 + lane of the push
      if (rdl(n, c) == Q - 1) {  // rare: this push fills the ring -- keep the t_complete it
        int32_t old = rdl(R.tc[0], T & 63);  // overwrites (the last completion)
#pragma unroll
        for (int g = 1; g < NG; ++g) old = (T >> 6) == g ? rdl(R.tc[g], T & 63) : old;
        V.saved = lane == c ? old : V.saved;
      }
#pragma unroll
      for (int g = 0; g < NG; ++g) {
        const bool w = lane + 64 * g == T;
        R.tc[g] = w ? tc : R.tc[g];
        R.ta[g] = w ? ta : R.ta[g];
      }
      const bool me = lane == c;
      V.tail = me ? tc : V.tail;
      const int32_t pl1 = pl + 1 == pl_wrap ? lane * 32 : pl + 1;
      pl = me ? pl1 : pl;
      Bt.lc = lg ? c : Bt.lc;
      Bt.ltc = lg ? tc : Bt.ltc;
      // ---- the next arrival: the pushed flow is still queued at ta_n if tc > ta_n
      const bool adj = me && tc > ta_n;
      n = adj ? n_n + 1 : n_n;
      key = adj ? k1 : k0;
      score = adj ? sc1 : sc0;
    } while (++bi < lim);
    if (seq == (1u << 26)) {  // the 26-bit flush tag would wrap: older maxima in `own` would win
      wave_sync();
      for (int i = 0; i < kWaveMaxS * 128 / 64; ++i) Ld.own[i * 64 + lane] = 0u;
      wave_sync();
      seq = 1u;
    }
    wave_flush(p, V, E, Bt, bi, lane, res_b, dur_b, Ld, seq++, base_ms, base_rem);
    ta = rdl(Bt.ta, bi);
    if (ta >= dt) break;
    base += 63u;
    wave_draw_batch<TRACE>(st, p, E, base, ta, lane, Bt);
    bi = 0;
  }
  V.wp = pl - lane * 32;
  // the pending arrival (its time >= dt)
  E.arr_idx = base + (uint32_t)bi;
  E.next_arr = ta;
  E.next_work = rdl(Bt.wk, bi);
  E.u2 = rdl(Bt.u2, bi);
  E.u3 = rdl(Bt.u3, bi);
}

template <int NG, int POLICY, bool TRACE, bool VC>
__device__ __forceinline__ void sim_step_wave(const DevState& st, const SimParams& p, WaveEnv& E,
                                              WaveSrv& V, WaveRing<NG>& R, int lane,
                                              uint2* const res_b, uint32_t* const dur_b,
                                              WaveLds& Ld, uint32_t& seq,
                                              float w_own) {
  constexpr bool lsq = (POLICY == 2 || POLICY == 3);
  const int S = p.S, Q = p.Q;
  const int32_t dt = p.dt_us;
  const uint64_t base_us = (uint64_t)E.clock * (uint64_t)dt;
  const uint32_t base_ms = (uint32_t)(base_us / 1000u);
  const uint32_t base_rem = (uint32_t)(base_us - (uint64_t)base_ms * 1000u);
  const int rpos = lane & 31;
  if (V.act && !lsq) {
    V.den = (double)w_own + 1e-9;
    V.rcp = 1.0 / V.den;
  }
  V.pushed = 0;

  // ---- 1. carried-in flows that complete in this step, server lane by server lane, in FIFO
  //      order (their Algorithm R draws from the reservoir stream)
#pragma unroll
  for (int g = 0; g < NG; ++g) {
    const int srv = 2 * g + (lane >> 5);
    if (srv < S && rpos < Q) Ld.img[rpos * kWaveMaxS + srv] = make_int2(R.tc[g], R.ta[g]);
  }
  wave_sync();
  if (V.act && V.cnt0 > 0) {
    int pos = V.wp - V.cnt0;
    pos = pos < 0 ? pos + Q : pos;
    int32_t prev = V.last;
    uint32_t rc = V.rcnt;
    for (int i = 0; i < V.cnt0; ++i) {
      const int2 e = Ld.img[pos * kWaveMaxS + lane];
      if (e.x > dt) break;
      const u32x4 d = philox4x32_10(
          u32x4{rc >> 1, E.gid, E.episode, (kStreamReservoir << 24) | (uint32_t)lane}, p.key0,
          p.key1);
      const int slot = reservoir_slot(rc, d);
      if (slot >= 0) {
        const uint32_t fct =
            lost_fct(p, (uint32_t)(e.x - e.y), (uint32_t)base_us + (uint32_t)e.y, E.gid, E.episode);
        const uint32_t dur = dur_sample(p, e.x, e.y, e.y > prev ? e.y : prev);
        if (big_record(fct, dur)) Ld.big[lane] = 1u;  // this lane's own server
        res_b[(uint32_t)lane * K + (uint32_t)slot] =
            make_uint2(fct, base_ms + (base_rem + (uint32_t)e.x) / 1000u);
        if (dur_b != nullptr) dur_b[(uint32_t)lane * K + (uint32_t)slot] = dur;
        atomicOr(Ld.chg + ((uint32_t)slot >> 5) * kWaveMaxS + (uint32_t)lane, 1u << (slot & 31));
      }
      prev = e.x;
      rc = count_inc(rc);
      pos = pos + 1 == Q ? 0 : pos + 1;
    }
    V.rcnt = rc;
  }
  wave_sync();

  // ---- 2. the arrivals (SED / SED2 scores are finite unless some den is 0 / inf / NaN)
  const bool finite = lsq || !V.act || (fabs(V.den) >= 1e-30 && fabs(V.den) <= 1e300);
  if (__all(finite))
    wave_event_loop<NG, POLICY, TRACE, true, VC>(st, p, E, V, R, lane, res_b, dur_b, Ld, seq, base_ms,
                                             base_rem);
  else
    wave_event_loop<NG, POLICY, TRACE, false, VC>(st, p, E, V, R, lane, res_b, dur_b, Ld, seq, base_ms,
                                              base_rem);

  // ---- 3. completions up to dt; the server's count, head and last completion
  uint64_t live[NG];
#pragma unroll
  for (int g = 0; g < NG; ++g) live[g] = __ballot(R.tc[g] > dt);
  const int32_t n = wave_count<NG>(live, lane);
#pragma unroll
  for (int g = 0; g < NG; ++g) {
    const int srv = 2 * g + (lane >> 5);
    if (srv < S && rpos < Q) Ld.img[rpos * kWaveMaxS + srv].x = R.tc[g];
  }
  wave_sync();
  if (V.act && V.cnt0 + V.pushed > n) {  // a flow completed this step: the newest one
    if (n == Q) {
      V.last = V.saved;
    } else {
      int pl = V.wp - n - 1;
      pl = pl < 0 ? pl + Q : pl;
      V.last = Ld.img[pl * kWaveMaxS + lane].x;
    }
  }
  wave_sync();
  V.cnt0 = n;
  // ---- rebase to the next step's start
  E.next_arr -= dt;
#pragma unroll
  for (int g = 0; g < NG; ++g) {  // completed flows free their slots
    R.tc[g] = R.tc[g] > dt ? R.tc[g] - dt : kDead;
    R.ta[g] -= dt;
  }
  V.tail -= dt;
  V.last = (V.last < kLastNone + dt) ? kLastNone : V.last - dt;
  E.clock += 1u;
}

// One dynamics launch's work for env b by one wave: state in, the step (or reset + warm-up),
// state out.  Returns false (having done nothing) for an env outside the batch or the reset mask.
template <int NG, int MODE, int POLICY, bool TRACE, bool VC = false>
__device__ __forceinline__ bool dyn_wave_env(const DevState& st, const SimParams& p,
                                             const void* action, int action_dtype,
                                             int32_t* assign_out, const uint8_t* reset_mask,
                                             uint32_t b, int lane, WaveLds& Ld) {
  if (b >= (uint32_t)p.B) return false;
  if (MODE == kModeReset && reset_mask != nullptr && reset_mask[b] == 0) return false;
  const int S = p.S, Q = p.Q;
  const int rpos = lane & 31;
  uint2* const res_b = st.res + (size_t)b * (size_t)S * K;
  uint32_t* const dur_b = st.res_dur != nullptr ? st.res_dur + (size_t)b * (size_t)S * K : nullptr;

  WaveEnv E;
  E.gid = p.env_id_offset + b;
  WaveSrv V;
  V.act = lane < S;
  V.scale = p.svc_scale[0];
#pragma unroll
  for (int k = 1; k < kWaveMaxS; ++k) V.scale = (k == lane) ? p.svc_scale[k] : V.scale;
  V.den = 1.0;
  V.rcp = 1.0;
  V.assigned = 0;
  V.saved = 0;
  if (lane < 4 * kWaveMaxS) Ld.chg[lane] = 0u;
  if (lane < kWaveMaxS) Ld.big[lane] = 0u;
#pragma unroll
  for (int i = 0; i < kWaveMaxS * 128 / 64; ++i) Ld.own[i * 64 + lane] = 0u;
  uint32_t seq = 1u;
  WaveRing<NG> R;
#pragma unroll
  for (int g = 0; g < NG; ++g) {
    R.tc[g] = kDead;
    R.ta[g] = 0;
  }
  const uint32_t sb = b * (uint32_t)S + (uint32_t)lane;  // server lane's server (lane < S)

  float w_own = 1.0f;
  auto reset_in = [&]() {  // a new episode (env.py:186-213): its first arrival, empty servers
    E.episode = st.episode[b] + 1u;
    E.clock = 0u;
    E.dropped = 0u;
    E.arr_idx = 0u;
    {  // arrival 0 (draw_arrival with t_prev = 0)
      const u32x4 d =
          philox4x32_10(u32x4{0u, E.gid, E.episode, kStreamArrival << 24}, p.key0, p.key1);
      int32_t gap;
      float wk;
      if constexpr (TRACE) {
        const uint32_t r = trace_row(p, E.gid, E.episode, 0u);
        gap = (int32_t)st.trace_gap[r];
        wk = st.trace_work[r];
      } else {
        gap = (int32_t)(-lb_logf(u01_open0(d.x)) * p.mean_gap_us);
        wk = -lb_logf(u01_open0(d.y));
      }
      E.next_arr = __builtin_amdgcn_readfirstlane(gap);
      E.next_work = __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(wk)));
      E.u2 = (uint32_t)__builtin_amdgcn_readfirstlane((int)d.z);
      E.u3 = (uint32_t)__builtin_amdgcn_readfirstlane((int)d.w);
    }
    V.cnt0 = 0;
    V.wp = 0;
    V.tail = 0;
    V.last = kLastNone;
    V.rcnt = 0u;
    // emptied reservoirs: slot 0 marked written, so the next observe recomputes every server of
    // the env (its cached features are the last episode's)
    if (lane < S) Ld.chg[lane] = 1u;
  };
  auto load_in = [&]() {  // the env, its ring lanes and server fields from HBM, the step's weight
    E.episode = st.episode[b];
    E.clock = st.clock[b];
    E.dropped = st.dropped[b];
    E.arr_idx = st.arr_idx[b];
    E.next_arr = st.next_arr[b];
    E.next_work = st.next_work[b];
    E.u2 = st.next_u2[b];
    E.u3 = st.next_u3[b];
    // every load first, from clamped in-range addresses (the ring lanes' slots and their servers'
    // head / count words, the server lane's own words and action), then the selects: one HBM
    // round trip (branches around the loads waited inside them, and the discrete weight came from
    // a table behind the action's load, profiles/r06o/)
    int2 e[NG];
    uint32_t hcg[NG];
#pragma unroll
    for (int g = 0; g < NG; ++g) {
      const int srv = 2 * g + (lane >> 5);
      const bool ok = srv < S && rpos < Q;
      const uint32_t sv = b * (uint32_t)S + (uint32_t)(ok ? srv : 0);
      e[g] = st.ring[(size_t)sv * (size_t)Q + (ok ? rpos : 0)];
      hcg[g] = st.hc[sv];
    }
    const uint32_t sbl = V.act ? sb : b * (uint32_t)S;
    const uint32_t hc = st.hc[sbl];
    const int32_t last = st.last_tc[sbl];
    const uint32_t rcnt = st.res_count[sbl];
    const float aw = action_weight_sel(p, action, action_dtype, (size_t)sbl);
#pragma unroll
    for (int g = 0; g < NG; ++g) {  // ring lanes: live if within [head, head + count)
      const int srv = 2 * g + (lane >> 5);
      if (srv < S && rpos < Q) {
        const int head = (int)(hcg[g] & kHcHead), cnt = (int)(hcg[g] >> 16);
        int rel = rpos - head;
        rel = rel < 0 ? rel + Q : rel;
        R.tc[g] = rel < cnt ? e[g].x : kDead;
        R.ta[g] = e[g].y;
      }
    }
    V.cnt0 = 0;
    V.wp = 0;
    V.tail = 0;
    V.last = kLastNone;
    V.rcnt = 0u;
    if (V.act) {
      const int head = (int)(hc & kHcHead);
      V.cnt0 = (int32_t)(hc >> 16);
      Ld.big[lane] = (hc & kHcBig) ? 1u : 0u;
      const int wp = head + V.cnt0;
      V.wp = wp >= Q ? wp - Q : wp;
      V.last = last;
      V.rcnt = rcnt;
      w_own = aw;
    }
    {  // tail = t_complete of the last queued flow, from the ring lanes (no dependent load)
      const int tp = V.wp == 0 ? Q - 1 : V.wp - 1;
      const int src = (lane & 1) * 32 + (tp & 31);
      int32_t tl = __shfl(R.tc[0], src, 64);
#pragma unroll
      for (int g = 1; g < NG; ++g) {
        const int32_t tg = __shfl(R.tc[g], src, 64);
        tl = ((lane >> 1) & (NG - 1)) == g ? tg : tl;
      }
      V.tail = (V.act && V.cnt0 > 0) ? tl : 0;
    }
  };
  auto reset_out = [&](int32_t ep_step) {
    V.assigned = 0;  // the warm-up's assignments are not the step's
    if (lane == 0) {
      st.ep_step[b] = ep_step;
      st.ep_return[b] = 0.0;
    }
  };
  if constexpr (MODE == kModeStep) {
    load_in();
    wave_sync();
    sim_step_wave<NG, POLICY, TRACE, VC>(st, p, E, V, R, lane, res_b, dur_b, Ld, seq, w_own);
  } else if constexpr (MODE == kModeReset) {
    reset_in();
    wave_sync();
    for (int k = 0; k < p.warmup_steps; ++k)
      sim_step_wave<NG, POLICY, TRACE, VC>(st, p, E, V, R, lane, res_b, dur_b, Ld, seq, 1.0f);
    reset_out(0);
  } else {  // kModeStepNR: an env done last step resets in place of stepping (ep_step = -1)
    const bool rs = st.ep_step[b] >= p.max_steps;
    int nsim = 1;
    if (rs) {
      reset_in();
      nsim = p.warmup_steps;
    } else {
      load_in();
    }
    wave_sync();
    for (int k = 0; k < nsim; ++k)
      sim_step_wave<NG, POLICY, TRACE, VC>(st, p, E, V, R, lane, res_b, dur_b, Ld, seq, w_own);
    if (rs) reset_out(-1);
  }

  // ---- state out: the queued flows, the server fields, the env words
#pragma unroll
  for (int g = 0; g < NG; ++g) {
    const int srv = 2 * g + (lane >> 5);
    if (srv < S && rpos < Q && R.tc[g] > 0)  // queued (rebased: t_complete > 0)
      st.ring[(size_t)(b * (uint32_t)S + (uint32_t)srv) * (size_t)Q + rpos] =
          make_int2(R.tc[g], R.ta[g]);
  }
  wave_sync();
  if (V.act) {
    int head = V.wp - V.cnt0;
    head = head < 0 ? head + Q : head;
    bool big = Ld.big[lane] != 0u;
    if (p.big_in_step) {  // the in-step records this launch wrote (big_written), by any lane
      const uint32_t cw[4] = {Ld.chg[lane], Ld.chg[kWaveMaxS + lane], Ld.chg[2 * kWaveMaxS + lane],
                              Ld.chg[3 * kWaveMaxS + lane]};
      __builtin_amdgcn_s_waitcnt(0);  // the wave's stores acknowledged by L2 (vmcnt 0)
      __asm__ volatile("" ::: "memory");
      big |= big_written(st, sb, cw, V.rcnt);
    }
    st.hc[sb] = (uint32_t)head | (big ? kHcBig : 0u) | ((uint32_t)V.cnt0 << 16);
    st.last_tc[sb] = V.last;
    st.res_count[sb] = V.rcnt;
    *reinterpret_cast<uint4*>(st.chg + (size_t)sb * 4) =
        make_uint4(Ld.chg[lane], Ld.chg[kWaveMaxS + lane], Ld.chg[2 * kWaveMaxS + lane],
                   Ld.chg[3 * kWaveMaxS + lane]);
    if (MODE != kModeReset && assign_out != nullptr) assign_out[sb] = V.assigned;
  }
  if (lane == 0) {
    st.episode[b] = E.episode;
    st.clock[b] = E.clock;
    st.dropped[b] = E.dropped;
    st.arr_idx[b] = E.arr_idx;
    st.next_arr[b] = E.next_arr;
    st.next_work[b] = E.next_work;
    st.next_u2[b] = E.u2;
    st.next_u3[b] = E.u3;
  }
  return true;
}

template <int NG, int MODE, int POLICY, bool TRACE>
__global__ void __launch_bounds__(64)
    dynamics_wave_kernel(DevState st, SimParams p, const void* action, int action_dtype,
                         int32_t* assign_out, const uint8_t* reset_mask) {
  __shared__ WaveLds Ld;
  dyn_wave_env<NG, MODE, POLICY, TRACE>(st, p, action, action_dtype, assign_out, reset_mask,
                                        blockIdx.x, (int)threadIdx.x, Ld);
}

}  // namespace lbk
