// lbsim_dyn_group.h — dynamics with one LANE per SERVER, for batches too small to fill the chip
// with one lane per env.
//
// dynamics_kernel (lbsim_kernels.h) gives each env one lane, so a batch of B envs is B/64 waves:
// 4096 envs (BASELINE configs[1]) are 64 waves on 1024 SIMDs, 8192 × 16-server envs (configs[4]
// per GPU) 128.  Here an env is a group of G = pow2 >= S lanes, lane s owning server s; the wave
// holds 64/G envs and the grid is B·G/64 waves.  Same event sequence, same arithmetic, same state
// layout as dynamics_kernel, so the two mappings are interchangeable between
// launches and bit-identical to the oracle.
//
// Arrival-driven like dynamics_kernel's sim_step: each iteration, every lane pops its own server's
// head if it completed by the next arrival (a group with a second due pop spends one more
// iteration), then the group assigns the arrival:
//   SED / LSQ choice: the reference's scan "start at the hashed server h, replace on a strictly
//     lower score" equals: h (or the first eligible server when h is full) if its score is the
//     minimum or NaN, else the lowest eligible server holding the minimum — with finite scores a
//     (score, rank) minimum over two DPP min reductions inside the group's row; with NaN scores
//     one DPP min reduction and ballots;
//   SED2 / LSQ2: the two candidates' scores broadcast by OR-reducing a one-hot word.
// Arrivals are drawn ahead, G at a time: every G iterations lane j of a group draws the group's
// arrival cbase + j (Philox block, gap, work) into LDS, so the Philox block and its two logs cost
// one pass per G iterations (the loop is latency-bound at small batches: these were the longest
// chain of an iteration).  The pushed flow's sample is inserted at once if it completes in this
// step, with its arrival's draw word as the Algorithm R draw (reservoir_slot_r32).
// Per-server fields are plain registers (one server per lane); the queue window lives in LDS
// [slot][lane].
#pragma once

#include "lbsim_kernels.h"

namespace lbk {

constexpr int kGroupWL = 8;  // LDS queue window per server: 64 lanes x 8 x 8 B = 4 KiB per wave
// kModeStepNR: 1 = the Philox round keys formed inside the draw-ahead block (group_event_loop
// KEYS: 120 VGPRs, no spills); 0 = hoisted as in the plain step (126 VGPRs at the 4-wave cap, 4
// spilled): 152.1-152.8 -> 150.6 us at 65536 x 4 (profiles/r06i/) -- the plain kernel shed the
// full handles' code, so the hoisted keys fit the budget again
#ifndef LBSIM_DYN_NR_KEYS
#define LBSIM_DYN_NR_KEYS 0
#endif

// Reductions over the aligned G-lane group (G <= 16: one DPP row).  Lanes read only within their
// group, so groups that left the event loop (inactive lanes) are never read.  mov_dpp with
// bound_ctrl and full masks lets the DPP combiner fold each step into one v_min/v_or with a DPP
// source; the event selection runs its two reductions interleaved (no wait states between a
// step's write and the next step's DPP read).
template <int CTRL>
__device__ __forceinline__ uint32_t gdpp(uint32_t v) {
  return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, CTRL, 0xF, 0xF, true);
}
// NaN-free f32 <-> int32 with the same order (-0 just below +0; the callers compare the result
// back as a float, so +-0 stay equal there)
__device__ __forceinline__ int32_t f32_key(float x) {
  const int32_t b = (int32_t)__float_as_uint(x);
  return b ^ ((b >> 31) & 0x7FFFFFFF);
}
__device__ __forceinline__ float key_f32(int32_t k) {
  return __uint_as_float((uint32_t)(k ^ ((k >> 31) & 0x7FFFFFFF)));
}
template <int CTRL>
__device__ __forceinline__ void gmin_step(int32_t& a, int32_t& b) {
  const int32_t oa = (int32_t)gdpp<CTRL>((uint32_t)a);
  const int32_t ob = (int32_t)gdpp<CTRL>((uint32_t)b);
  a = oa < a ? oa : a;
  b = ob < b ? ob : b;
}
// min over the group of two ints, interleaved
template <int G>
__device__ __forceinline__ void group_min2(int32_t& a, int32_t& b) {
  gmin_step<0xB1>(a, b);                          // quad_perm [1,0,3,2]
  if constexpr (G >= 4) gmin_step<0x4E>(a, b);    // quad_perm [2,3,0,1]
  if constexpr (G >= 8) gmin_step<0x141>(a, b);   // row_half_mirror
  if constexpr (G >= 16) gmin_step<0x140>(a, b);  // row_mirror
  if constexpr (G >= 32) {  // across DPP rows (S > 16): crossbar shuffles
    int32_t oa = __shfl_xor(a, 16, 64), ob = __shfl_xor(b, 16, 64);
    a = oa < a ? oa : a;
    b = ob < b ? ob : b;
    if constexpr (G >= 64) {
      oa = __shfl_xor(a, 32, 64);
      ob = __shfl_xor(b, 32, 64);
      a = oa < a ? oa : a;
      b = ob < b ? ob : b;
    }
  }
}
template <int G>
__device__ __forceinline__ int32_t group_min_i32(int32_t v) {
  int32_t o = (int32_t)gdpp<0xB1>((uint32_t)v);
  v = o < v ? o : v;
  if constexpr (G >= 4) { o = (int32_t)gdpp<0x4E>((uint32_t)v); v = o < v ? o : v; }
  if constexpr (G >= 8) { o = (int32_t)gdpp<0x141>((uint32_t)v); v = o < v ? o : v; }
  if constexpr (G >= 16) { o = (int32_t)gdpp<0x140>((uint32_t)v); v = o < v ? o : v; }
  if constexpr (G >= 32) { o = __shfl_xor(v, 16, 64); v = o < v ? o : v; }
  if constexpr (G >= 64) { o = __shfl_xor(v, 32, 64); v = o < v ? o : v; }
  return v;
}
template <int G>
__device__ __forceinline__ uint32_t group_add(uint32_t v) {  // every lane holds the group's sum
  v += gdpp<0xB1>(v);
  if constexpr (G >= 4) v += gdpp<0x4E>(v);
  if constexpr (G >= 8) v += gdpp<0x141>(v);
  if constexpr (G >= 16) v += gdpp<0x140>(v);
  if constexpr (G >= 32) v += (uint32_t)__shfl_xor((int)v, 16, 64);
  if constexpr (G >= 64) v += (uint32_t)__shfl_xor((int)v, 32, 64);
  return v;
}
template <int G>
__device__ __forceinline__ uint32_t group_or(uint32_t v) {
  v |= gdpp<0xB1>(v);
  if constexpr (G >= 4) v |= gdpp<0x4E>(v);
  if constexpr (G >= 8) v |= gdpp<0x141>(v);
  if constexpr (G >= 16) v |= gdpp<0x140>(v);
  if constexpr (G >= 32) v |= (uint32_t)__shfl_xor((int)v, 16, 64);
  if constexpr (G >= 64) v |= (uint32_t)__shfl_xor((int)v, 32, 64);
  return v;
}
// This lane's group's bits of a wave ballot.
template <int G>
__device__ __forceinline__ uint64_t group_bits(uint64_t m, int gbase) {
  return G == 64 ? m : (m >> gbase) & ((1ull << (G & 63)) - 1ull);
}

// The server this lane owns (fields of DESIGN.md §4, in registers).
struct SrvLane {
  int32_t cnt, head_tc, head, lh, tail, last, assigned;
  int32_t qcap;     // Q, or 0 while the server is down (fail_prob > 0): not eligible, as full
  bool big;         // the server's sticky kHcBig flag
  uint32_t rcnt;
  int32_t lost;     // n_flow_on_mode VPP (p.leak): the server's lost-FIN flows completed so far
                    // (DevState::lost_on, never decremented: lbhash.h:193,214); its SED / LSQ
                    // scores count them with the queue (node.c:395-437 read as_stat n_flow_on)
  uint32_t* chgw;   // LDS [4][64]: word w of this lane's 128-bit mask of the reservoir slots
                    // written this launch (DevState::chg), set by one ds_or per insert
  float score, scale;
  double den, rcp;
  bool act;  // s < S
  // split handles (lost-FIN, SimParams::split): the duration reservoir's count, the pending
  // guesses' ring head / count, the head entry's due word (absolute us mod 2^32), and the guesses
  // this lane dropped at a full ring in this launch
  uint32_t rcnt_d;
  int32_t phead, pcnt;
  uint32_t pdue, over;
};

// ALIAS table of the group in LDS: word f of active position k at [f][gbase + k].  Every lane of
// the group builds the same table (same values to the same words).
struct GroupAliasTab {
  int32_t* t;
  int gbase;
  __device__ int32_t& operator()(int f, int k) const { return t[f * 64 + gbase + k]; }
};

// ---- split handles (lost-FIN; oracle split_add / pend_push / pend_flush): the
//      fct and duration reservoirs of a server make their own decisions, and a timed-out flow's
//      guess waits in the server's pending ring (HBM, sorted by due time) until its wrap-up.
//      Rare paths of the general event loop: a lane loops on its own.
// One sample into the fct (is_dur false) or duration reservoir of server row sb: own count, own
// slot (res_slot; the duration reservoir draws as a run without losses would, the fct
// reservoir's stream word carries 1 << 16), {us, ts} record; a
// carried-in or deferred sample (!has_r) sets the big flag at its store.
__device__ __forceinline__ void split_add(const DevState& st, const SimParams& p, SrvLane& V,
                                          uint32_t sb, uint32_t gid, uint32_t episode, int s,
                                          bool is_dur, uint32_t v, uint32_t ts_ms, bool has_r,
                                          uint32_t r) {
  const uint32_t c = is_dur ? V.rcnt_d : V.rcnt;
  const int slot = res_slot(p, c, has_r, r, gid, episode,
                            (kStreamReservoir << 24) | (is_dur ? 0u : 1u << 16) | (uint32_t)s);
  if (slot >= 0) {
    if (!has_r && v >= kPackLimit) V.big = true;
    uint2* rec = is_dur ? reinterpret_cast<uint2*>(st.res_dur) : st.res;
    rec[(size_t)sb * K + (uint32_t)slot] = make_uint2(v, ts_ms);
    atomicOr(V.chgw + ((uint32_t)slot >> 5) * 64u, 1u << (slot & 31));
  }
  if (is_dur) V.rcnt_d = count_inc(c);
  else V.rcnt = count_inc(c);
}
// The guesses due by step time t (relative us) into the fct reservoir, in due order, each stamped
// with its due time (lbhash.h:182-217: the bucket's next flow records now - t_init - 40 s).
__device__ __forceinline__ void split_flush(const DevState& st, const SimParams& p, SrvLane& V,
                                            uint32_t sb, uint32_t gid, uint32_t episode, int s,
                                            int32_t t, uint64_t base_us) {
  const int P = p.pend_P;
  const uint2* ring = st.pend + (size_t)sb * (uint32_t)P;
  while (V.pcnt > 0) {
    const int32_t rel = (int32_t)(V.pdue - (uint32_t)base_us);
    if (rel > t) break;
    const uint32_t val = ring[V.phead].y;
    const uint32_t ts = (uint32_t)((uint64_t)((int64_t)base_us + (int64_t)rel) / 1000u);
    split_add(st, p, V, sb, gid, episode, s, false, val, ts, false, 0u);
    V.phead = V.phead + 1 == P ? 0 : V.phead + 1;
    V.pcnt -= 1;
    if (V.pcnt > 0) V.pdue = ring[V.phead].x;
  }
}
// A guess due at `due` into the sorted ring (insertion from the tail; an equal due goes after
// the entries already there); a full ring drops it (V.over, summed into lf_over).
__device__ __forceinline__ void split_push(const DevState& st, const SimParams& p, SrvLane& V,
                                           uint32_t sb, uint32_t due, uint32_t val) {
  const int P = p.pend_P;
  if (V.pcnt == P) {
    V.over += 1u;
    return;
  }
  uint2* ring = st.pend + (size_t)sb * (uint32_t)P;
  int i = V.pcnt;
  while (i > 0) {
    int pos = V.phead + i - 1;
    pos = pos >= P ? pos - P : pos;
    const uint2 e = ring[pos];
    if ((int32_t)(e.x - due) <= 0) break;
    ring[pos + 1 == P ? 0 : pos + 1] = e;
    --i;
  }
  int pos = V.phead + i;
  pos = pos >= P ? pos - P : pos;
  ring[pos] = make_uint2(due, val);
  V.pcnt += 1;
  if (i == 0) V.pdue = due;
}
// A flow completing at tc (arrived at ta; relative us) on a split handle (oracle pop_until): the
// guesses due by tc, its duration sample now (lbhash.h:129-136), then its fct -- now (RSTACK,
// :116-124) or, lost, as a guess due at tc + flow_timeout + the bucket wait (:182-192, :204-213).
__device__ __forceinline__ void split_complete(const DevState& st, const SimParams& p, SrvLane& V,
                                               uint32_t sb, uint32_t gid, uint32_t episode, int s,
                                               int32_t tc, int32_t ta, uint32_t dur, uint32_t ts_ms,
                                               bool has_r, uint32_t r, uint64_t base_us) {
  split_flush(st, p, V, sb, gid, episode, s, tc, base_us);
  split_add(st, p, V, sb, gid, episode, s, true, dur, ts_ms, has_r, r);
  int32_t wait = 0;
  if (lf_wait(p, (uint32_t)base_us + (uint32_t)ta, gid, episode, wait))
    split_push(st, p, V, sb,
               (uint32_t)base_us + (uint32_t)tc + (uint32_t)(p.lf_off_us + 40000000) +
                   (uint32_t)wait,
               lf_guess((uint32_t)(tc - ta), p.lf_off_us, wait));
  else
    split_add(st, p, V, sb, gid, episode, s, false, (uint32_t)(tc - ta), ts_ms, has_r, r);
}
// reservoir_mode VPP: the server's bins zeroed (reset, failure; VPP's zeroed shm).
__device__ __forceinline__ void vpp_zero_bins(const DevState& st, const SimParams& p, uint32_t sb) {
  uint4* r4 = reinterpret_cast<uint4*>(st.res + (size_t)sb * K);
  for (int i = 0; i < K / 2; ++i) r4[i] = make_uint4(0u, 0u, 0u, 0u);
  if (st.res_dur != nullptr) {
    const int n4 = p.split ? K / 2 : K / 4;
    uint4* d4 = reinterpret_cast<uint4*>(st.res_dur + (size_t)sb * K * (p.split ? 2u : 1u));
    for (int i = 0; i < n4; ++i) d4[i] = make_uint4(0u, 0u, 0u, 0u);
  }
}

// Loop constants of one step: the Philox keys and the scalars the loop reads, pinned in VGPRs so
// the loop never reloads them from the kernarg segment.  Only the two base keys are kept: round
// r's keys (k + r * the Weyl constants) are formed inside the draw-ahead block, 20 adds per G
// iterations instead of 18 more live VGPRs (116 -> 100; dynamics 1-2 % faster at 4096 x 4,
// 65536 x 8 and 262144 x 4, unchanged at 65536 x 4: profiles/r03/ab_dyn_round_keys.txt).
struct GroupConst {
  uint32_t k0, k1;
  float mean_gap;
  int32_t dt;
  uint32_t base_ms, base_rem;
};
__device__ __forceinline__ GroupConst group_const(const SimParams& p, uint32_t base_ms,
                                                  uint32_t base_rem) {
  GroupConst c;
  c.k0 = vpin(p.key0);
  c.k1 = vpin(p.key1);
  c.mean_gap = vpin(p.mean_gap_us);
  c.dt = vpin(p.dt_us);
  c.base_ms = vpin(base_ms);
  c.base_rem = vpin(base_rem);
  return c;
}

// The event loop of sim_step_group (section 2).  FAST (wave-uniform): every SED score finite, so no
// NaN fallback division and no NaN ballot.  KEYS: the Philox round keys are formed inside the
// draw-ahead block instead of being hoisted into 20 loop-long VGPRs (LBSIM_DYN_NR_KEYS for
// kModeStepNR; the plain step hoists them: 4 us faster at 65536 x 4, profiles/r06c/).
// FULL: the handle's features beyond the plain simulator -- n_flow_on_mode VPP's lost-flow counts,
// a duration plane (duration_mode SERVICE), lost-FIN deferral (split reservoirs), reservoir_mode
// VPP -- compiled only into dynamics_group_full_kernel, so none of their registers weigh on the
// plain kernel (126 VGPRs, 4 waves per SIMD; with them inlined it took 164).
template <int G, int POLICY, bool TRACE, bool FAST, bool KEYS = false, bool FULL = false>
__device__ __forceinline__ void group_event_loop(const DevState& st, const SimParams& p,
                                                 LaneState<1>& E, SrvLane& V, int s, int gbase,
                                                 int n_alias, const GroupConst& gc, int2* win,
                                                 int32_t* atab, int4* acache, uint2* const my_res,
                                                 int2* const my_ring) {
  constexpr int WL = kGroupWL;
  constexpr bool two_choice = (POLICY == 1 || POLICY == 3);
  constexpr bool alias = POLICY == kPolicyAlias;
  constexpr bool lsq = (POLICY == 2 || POLICY == 3);
  const int S = p.S, Q = p.Q;
  const int32_t dt = gc.dt;
  const GroupAliasTab tab{atab, gbase};
  const int lane = gbase + s;
  auto wslot = [&](int i) -> int2* { return win + i * 64 + lane; };
  auto mark = [&](int slot) {  // the slot's bit in the lane's 128-bit written-slot mask
    atomicOr(V.chgw + ((uint32_t)slot >> 5) * 64u, 1u << (slot & 31));
  };
  // Draw-ahead: every G iterations (a wave-uniform schedule: all active groups loop in step) lane
  // j of a group draws arrival cbase + j (cbase = the group's next undrawn arrival) -- its Philox
  // block, gap and work -- into the group's slots acache[gbase + j].  One arrival at most is
  // consumed per iteration, so the G slots last until the next refill, and the Philox block and
  // the two logs cost one pass per G iterations instead of one per iteration.
  uint32_t cbase = 0u;
  uint32_t it = 0u;
  // TRACE: the trace row of arrival kbase, advanced by the arrivals consumed between refills (one
  // 64-bit modulo per step instead of one per drawn arrival)
  uint32_t kbase = E.arr_idx + 1u, rbase = 0u;
  if constexpr (TRACE) rbase = trace_row(p, E.gid, E.episode, kbase);
  for (;;) {
    if ((it & (uint32_t)(G - 1)) == 0u) {
      cbase = E.arr_idx + 1u;
      const uint32_t k = cbase + (uint32_t)s;
      uint32_t rk0[10], rk1[10];
      uint32_t k0 = gc.k0, k1 = gc.k1;
      if constexpr (KEYS) asm volatile("" : "+v"(k0), "+v"(k1));  // opaque: not hoisted
#pragma unroll
      for (int r = 0; r < 10; ++r) {
        rk0[r] = k0 + (uint32_t)r * 0x9E3779B9u;
        rk1[r] = k1 + (uint32_t)r * 0xBB67AE85u;
      }
      const u32x4 d = philox_rk(u32x4{k, E.gid, E.episode, kStreamArrival << 24}, rk0, rk1);
      int32_t gap;
      float wk;
      if constexpr (TRACE) {
        const uint32_t rows = p.trace_rows;
        rbase += cbase - kbase;  // <= G arrivals since the last refill
        kbase = cbase;
        while (rbase >= rows) rbase -= rows;
        uint32_t r = rbase + (uint32_t)s;
        while (r >= rows) r -= rows;
        gap = (int32_t)st.trace_gap[r];
        wk = st.trace_work[r];
      } else {  // (the two logs as one packed-f32 polynomial measured 2 % slower: r05t)
        gap = (int32_t)(-lb_logf(u01_open0(d.x)) * gc.mean_gap);
        wk = -lb_logf(u01_open0(d.y));
      }
      acache[lane] = make_int4(gap, __float_as_int(wk), (int)d.z, (int)d.w);
      __builtin_amdgcn_wave_barrier();
    }
    // the next arrival (arr_idx + 1, within the draw-ahead window: at most one arrival per
    // iteration since the refill) is read now, so its LDS round trip overlaps the queue head's
    // instead of following the choice
    const int4 nx = acache[gbase + (int)(E.arr_idx + 1u - cbase)];
    ++it;
    const bool arrival_due = E.next_arr < dt;  // the same in every lane of the group
    const int32_t th = arrival_due ? E.next_arr : dt;
    const bool due = V.act && V.cnt > 0 && V.head_tc <= th;
    if constexpr (FULL) {  // n_flow_on_mode VPP: a popped lost-FIN flow stays in n_flow_on
      if (p.leak && due &&
          lf_lost(p, gc.base_ms * 1000u + gc.base_rem + (uint32_t)wslot(V.lh)->y, E.gid, E.episode))
        V.lost += 1;
    }
    if (due && V.cnt > WL) {  // rare: the slot the pop frees takes queue entry WL from the ring
      int pw = V.head + WL;
      pw = pw >= Q ? pw - Q : pw;
      *wslot(V.lh) = my_ring[(uint32_t)pw];
      __builtin_amdgcn_s_waitcnt(kWaitVmcnt0);
    }
    // (reading the entry after the new head one iteration ahead, into a register, measured 4 us
    // slower at 65536 x 4: profiles/r06c/)
    const int nl = (V.lh + 1) & (WL - 1);
    const int32_t nt = wslot(nl)->x;  // next head (valid if cnt > 1)
    V.last = due ? V.head_tc : V.last;
    V.cnt -= due ? 1 : 0;
    V.head = due ? ((V.head + 1 == Q) ? 0 : V.head + 1) : V.head;
    V.lh = due ? nl : V.lh;
    // (computing the choice key here, before the next head's LDS read is waited for, measured
    // 3 us slower at 65536 x 4, profiles/r06e/)
    V.head_tc = due ? nt : V.head_tc;
    const bool more = group_bits<G>(__ballot(due && V.cnt > 0 && nt <= th), gbase) != 0ull;
    if (!arrival_due && !more) break;  // group-uniform
    const bool arr = arrival_due && !more;

    // ---- the arrival: choose a server (node.c:388-441); full servers are not eligible
    const int32_t ta = E.next_arr;
    if constexpr (!alias) {
      // the data plane's n_flow_on: the queue, plus the lost-FIN flows it never decremented
      // (n_flow_on_mode VPP only: the general loop; V.lost = 0 otherwise)
      const int32_t nfo = FULL ? V.cnt + V.lost : V.cnt;
      if constexpr (lsq) {
        V.score = (float)nfo;
      } else {  // (cnt + 1) / den correctly rounded (Markstein), division for den 0 / inf / NaN
        const double c = (double)(nfo + 1);
        const double q0 = c * V.rcp;
        double q = fma(fma(-q0, V.den, c), V.rcp, q0);
        if (!FAST && q != q) {
          asm volatile("");
          q = c / V.den;
        }
        V.score = (float)q;
      }
    }
    const bool elig = V.act && V.cnt < V.qcap;
    const uint64_t em = group_bits<G>(__ballot(elig), gbase);
    int chosen = -1;
    if constexpr (alias) {
      if (n_alias > 0) {
        const int a = alias_pick(tab, n_alias, E.u2);
        chosen = ((em >> a) & 1u) ? a : -1;
      }
    } else if constexpr (two_choice) {
      const int h1 = two_choice_h1(E.u2, S);
      const int h2 = two_choice_h2(E.u2, S);
      const uint32_t bits = __float_as_uint(V.score);
      const float s1 = __uint_as_float(group_or<G>(s == h1 ? bits : 0u));
      const float s2 = __uint_as_float(group_or<G>(s == h2 ? bits : 0u));
      const bool ok1 = (em >> h1) & 1u, ok2 = (em >> h2) & 1u;
      chosen = (ok1 && ok2) ? ((s2 < s1) ? h2 : h1) : (ok1 ? h1 : (ok2 ? h2 : -1));
    } else if constexpr (FAST) {
      // finite scores: the scan's result is the eligible minimum, h among equal minima, else the
      // lowest such server -- a lexicographic (score, rank) minimum with rank 0 for h and s + 1
      // otherwise, as two DPP min reductions (no ballots, no 64-bit group masks)
      const int32_t key = elig ? f32_key(V.score) : 0x7FFFFFFF;  // finite keys < 0x7f800001
      const int32_t mk = group_min_i32<G>(key);
      const int h = (int)__umulhi(E.u2, (uint32_t)S);
      const int32_t rk = (elig && key == mk) ? (s == h ? 0 : s + 1) : 0xFF;
      const int32_t mr = group_min_i32<G>(rk);
      chosen = mr == 0xFF ? -1 : (mr == 0 ? h : mr - 1);
    } else {
      const bool num = elig && V.score == V.score;
      const float m = key_f32(group_min_i32<G>(num ? f32_key(V.score) : 0x7f800000));
      const int h = (int)__umulhi(E.u2, (uint32_t)S);
      const int c0 = ((em >> h) & 1u) ? h : (em ? __builtin_ctzll(em) : -1);
      const uint64_t tie = group_bits<G>(__ballot(num && V.score == m), gbase);
      const uint64_t nan = FAST ? 0ull : group_bits<G>(__ballot(V.score != V.score), gbase);
      chosen = c0 < 0 ? -1 : ((((tie | nan) >> c0) & 1u) ? c0 : (tie ? __builtin_ctzll(tie) : -1));
    }
    const bool push = arr && chosen >= 0;
    E.dropped += (arr && chosen < 0) ? 1u : 0u;
    const bool mine = push && s == chosen;

    // ---- FIFO service on the chosen server (its lane)
    const int32_t start_a = V.cnt > 0 ? (V.tail > ta ? V.tail : ta) : ta;
    int32_t svc = (int32_t)(E.next_work * V.scale);
    svc = svc < 1 ? 1 : svc;
    const int32_t tc_a = start_a + svc;
    const bool ins = mine && tc_a <= dt;  // completes in this step: its sample now

    // ---- the pushed flow's Algorithm R draw is this arrival's word r (E.u3)
    const int slot = (FULL && p.res_vpp) ? (int)(E.u3 >> 25) : reservoir_slot_r32(V.rcnt, E.u3);
    bool split = false;  // split handles (lost-FIN): their own inserts (split_complete)
    if constexpr (FULL) {
      split = p.split != 0;
      if (split && ins) {
        const uint64_t base_us = (uint64_t)gc.base_ms * 1000u + gc.base_rem;
        split_complete(st, p, V, (uint32_t)((size_t)(my_res - st.res) / K), E.gid, E.episode, s,
                       tc_a, ta, p.dur_service ? (uint32_t)svc : (uint32_t)(tc_a - ta),
                       gc.base_ms + (gc.base_rem + (uint32_t)tc_a) / 1000u, true, E.u3, base_us);
      }
    }
    if (!split && ins && slot >= 0) {
      // lost-FIN flows only on split handles: fct = tc - ta here
      const uint32_t fct = (uint32_t)(tc_a - ta);
      my_res[(uint32_t)slot] = make_uint2(fct, gc.base_ms + (gc.base_rem + (uint32_t)tc_a) / 1000u);
      if constexpr (FULL) {  // the duration plane:
        if (st.res_dur != nullptr)  // the age tc - ta, or the service time svc = tc - start
          st.res_dur[(size_t)(my_res - st.res) + (uint32_t)slot] =
              p.dur_service ? (uint32_t)svc : (uint32_t)(tc_a - ta);
      }
      mark(slot);
    }
    // (a branch-free push, non-pushing lanes storing to scratch slots, measured 3 us slower at
    // 65536 x 4, profiles/r06e/)
    if (mine) {
      const int2 e = make_int2(tc_a, ta);
      if (V.cnt < WL) {
        *wslot((V.lh + V.cnt) & (WL - 1)) = e;
      } else {
        int pos = V.head + V.cnt;
        pos = pos >= Q ? pos - Q : pos;
        my_ring[(uint32_t)pos] = e;
        asm volatile("");  // no flat store (see dynamics_kernel)
      }
      V.tail = tc_a;
      V.assigned += 1;
      V.head_tc = V.cnt == 0 ? tc_a : V.head_tc;
      V.cnt += 1;
      V.rcnt = (ins && !split) ? count_inc(V.rcnt) : V.rcnt;
    }

    // ---- next arrival (identical in every lane of the group): arrival arr_idx + 1 from the
    //      group's draw-ahead slots
    const int32_t na = ta + nx.x;
    const float nw = __int_as_float(nx.y);
    const uint32_t nu2 = (uint32_t)nx.z, nu3 = (uint32_t)nx.w;
    E.next_arr = arr ? na : E.next_arr;
    E.next_work = arr ? nw : E.next_work;
    E.u2 = arr ? nu2 : E.u2;
    E.u3 = arr ? nu3 : E.u3;
    E.arr_idx += arr ? 1u : 0u;
  }
}

template <int G, int POLICY, bool TRACE, bool KEYS = false, bool FULL = false>
__device__ __forceinline__ void sim_step_group(const DevState& st, const SimParams& p,
                                               LaneState<1>& E, SrvLane& V, uint32_t b, int s,
                                               int gbase, float w_own, const float (&wall)[G],
                                               int2* win, int32_t* atab, int4* acache) {
  constexpr int WL = kGroupWL;
  const int S = p.S, Q = p.Q;
  const int32_t dt = p.dt_us;
  const uint64_t base_us = (uint64_t)E.clock * (uint64_t)dt;
  const uint32_t base_ms = (uint32_t)(base_us / 1000u);
  const uint32_t base_rem = (uint32_t)(base_us - (uint64_t)base_ms * 1000u);
  constexpr bool alias = POLICY == kPolicyAlias;
  constexpr bool lsq = (POLICY == 2 || POLICY == 3);
  const uint32_t sb = b * (uint32_t)S + (uint32_t)s;  // valid when V.act
  uint2* const my_res = st.res + (size_t)sb * K;
  int2* const my_ring = st.ring + (size_t)sb * (size_t)Q;
  const GroupAliasTab tab{atab, gbase};
  const int lane = gbase + s;
  int n_alias = 0;
  if constexpr (alias) {
    n_alias = build_alias<G>(wall, S, tab);
  } else if (V.act && !lsq) {
    V.den = (double)w_own + 1e-9;
    V.rcp = 1.0 / V.den;
  }
  auto wslot = [&](int i) -> int2* { return win + i * 64 + lane; };
  auto mark = [&](int slot) {  // the slot's bit in the lane's 128-bit written-slot mask
    atomicOr(V.chgw + ((uint32_t)slot >> 5) * 64u, 1u << (slot & 31));
  };

  // ---- 0. server failure / recovery (fail_prob > 0, a uniform branch): one Philox draw per
  //      server, stream 5, counter (clock, gid, episode); a failing server loses its queue (the
  //      flows count as dropped) and its reservoirs; a down server takes no flows
  if (p.fail_thr != 0u) {
    const u32x4 d = philox4x32_10(
        u32x4{E.clock, E.gid, E.episode, (kStreamFailure << 24) | (uint32_t)s}, p.key0, p.key1);
    const uint32_t u = d.x >> 8;
    const bool was_down = V.qcap == 0;
    const bool fails = V.act && !was_down && u < p.fail_thr;
    const bool recovers = V.act && was_down && u < p.rec_thr;
    E.dropped += group_add<G>(fails ? (uint32_t)V.cnt : 0u);
    if (fails) {
      V.cnt = 0;
      V.last = kLastNone;
      V.rcnt = 0u;
      V.big = false;
      mark(0);  // emptied: the next observe recomputes the (zero) features
      V.lost = 0;
      if constexpr (FULL) {
        V.rcnt_d = 0u;  // split: the duration reservoir and the pending guesses go too
        V.pcnt = 0;
        V.phead = 0;
        if (p.res_vpp) vpp_zero_bins(st, p, sb);
      }
    }
    V.qcap = fails ? 0 : (recovers ? Q : V.qcap);
  }

  // ---- 1. this lane's carried-in flows that complete in this step: samples in FIFO order.  The
  //      window's entries (LDS) in one loop and the rare ones past it (HBM ring) in another: one
  //      loop over both read each entry through a flat load, and its vmcnt wait -- the counter
  //      gfx950 shares between loads and stores -- waited for the previous insert's record store
  //      every flow (profiles/r06o/)
  if (V.act && V.cnt > 0 && V.head_tc <= dt) {
    int32_t prev = V.last;
    uint32_t rc = V.rcnt;
    auto insert = [&](int32_t etc, int32_t eta) {
      if (FULL && p.split) {  // lost-FIN: split reservoirs and deferred guesses (split_complete)
        split_complete(st, p, V, sb, E.gid, E.episode, s, etc, eta,
                       dur_sample(p, etc, eta, eta > prev ? eta : prev),
                       base_ms + (base_rem + (uint32_t)etc) / 1000u, false, 0u, base_us);
        rc = V.rcnt;
      } else {
        const u32x4 d = philox4x32_10(
            u32x4{rc >> 1, E.gid, E.episode, (kStreamReservoir << 24) | (uint32_t)s}, p.key0,
            p.key1);
        // reservoir_mode VPP: slot rand() % 128 for every sample (res_slot)
        const int slot =
            (FULL && p.res_vpp) ? (int)(((rc & 1u) ? d.w : d.y) >> 25) : reservoir_slot(rc, d);
        if (slot >= 0) {
          // (lost-FIN flows only on split handles; the duration sample differs from the fct only
          // under duration_mode SERVICE: a full handle)
          const uint32_t fct = (uint32_t)(etc - eta);
          const uint32_t dur = FULL ? dur_sample(p, etc, eta, eta > prev ? eta : prev) : fct;
          V.big |= big_record(fct, dur);
          store_record(st, (size_t)sb * K + (uint32_t)slot, fct, dur,
                       base_ms + (base_rem + (uint32_t)etc) / 1000u);
          mark(slot);
        }
        rc = count_inc(rc);
      }
      prev = etc;
    };
    const int nwin = V.cnt < WL ? V.cnt : WL;
    int i = 0;
    bool past = false;  // an entry completing after dt was reached
    for (; i < nwin; ++i) {
      const int2 e = *wslot((V.lh + i) & (WL - 1));
      if (e.x > dt) {
        past = true;
        break;
      }
      insert(e.x, e.y);
    }
    if (!past) {  // rare: queued beyond the window
      int pos = V.head + i;
      pos = pos >= Q ? pos - Q : pos;
      for (; i < V.cnt; ++i) {
        const int2 e = my_ring[(uint32_t)pos];
        if (e.x > dt) break;
        insert(e.x, e.y);
        pos = pos + 1 == Q ? 0 : pos + 1;
      }
    }
    V.rcnt = rc;
  }

  // ---- 2. one arrival per iteration (as dynamics_kernel's sim_step), the group in step.  SED /
  //      SED2 scores can only be NaN when some den is 0 / inf / NaN: a wave whose servers all have
  //      finite scores runs the loop without the NaN fallbacks (a wave-uniform choice).
  const GroupConst gc = group_const(p, base_ms, base_rem);
  const bool finite = lsq || alias || !V.act ||
                      (fabs(V.den) >= 1e-30 && fabs(V.den) <= 1e300);  // false for NaN
  if constexpr (FULL) {  // (a full handle always runs the general loop)
    group_event_loop<G, POLICY, TRACE, false, KEYS, true>(st, p, E, V, s, gbase, n_alias, gc, win,
                                                          atab, acache, my_res, my_ring);
    // split handles: the guesses due by the step's end (oracle sim_step)
    if (p.split && V.act) split_flush(st, p, V, sb, E.gid, E.episode, s, dt, base_us);
  } else if (__all(finite)) {
    group_event_loop<G, POLICY, TRACE, true, KEYS>(st, p, E, V, s, gbase, n_alias, gc, win, atab,
                                                   acache, my_res, my_ring);
  } else {
    group_event_loop<G, POLICY, TRACE, false, KEYS>(st, p, E, V, s, gbase, n_alias, gc, win, atab,
                                                    acache, my_res, my_ring);
  }

  // ---- rebase to the next step's start (this lane's server)
  E.next_arr -= dt;
  if (V.act) {
    for (int i = 0; i < WL && i < V.cnt; ++i) {
      int2* e = wslot((V.lh + i) & (WL - 1));
      e->x -= dt;
      e->y -= dt;
    }
    int pos = V.head + WL;
    if (pos >= Q) pos -= Q;
    for (int i = WL; i < V.cnt; ++i) {
      int2 e = my_ring[(uint32_t)pos];
      e.x -= dt;
      e.y -= dt;
      my_ring[(uint32_t)pos] = e;
      pos = (pos + 1 == Q) ? 0 : pos + 1;
    }
    V.head_tc -= dt;
    V.tail -= dt;
    V.last = (V.last < kLastNone + dt) ? kLastNone : V.last - dt;
  }
  E.clock += 1u;
}

// LDS of one dynamics wave (dynamics_group_kernel, fused_step_kernel).
template <int POLICY>
struct DynGroupLds {
  int2 win[kGroupWL * 64];                          // queue windows, [slot][lane]
  int4 acache[64];                                  // draw-ahead arrival slots, [group][G]
  uint32_t chgw[4 * 64];                            // written-slot masks, [word][lane]
  int32_t atab[POLICY == kPolicyAlias ? 2 * 64 : 1];  // ALIAS tables, [word][lane] (last: the
                                                      // others keep their 16-B aligned offsets)
};

// One step (or reset) of the 64 / G envs of wave `wave` (env b = wave * 64 / G + lane / G), lane s
// of a group owning server s: state in, the event loop, state back to HBM.  Lanes of envs past B
// (or outside the reset mask) return at once, whole groups together.
template <int G, int MODE, int POLICY, bool TRACE, bool FULL = false>
__device__ __forceinline__ void dyn_group_wave(const DevState& st, const SimParams& p,
                                               const void* action, int action_dtype,
                                               int32_t* assign_out, const uint8_t* reset_mask,
                                               uint32_t wave, int lane, DynGroupLds<POLICY>& L) {
  static_assert(G == 2 || G == 4 || G == 8 || G == 16 || G == 32 || G == 64,
                "group = a power of two lanes of the wave");
  constexpr int WL = kGroupWL;
  constexpr bool alias = POLICY == kPolicyAlias;
  int2* const win = L.win;
  int32_t* const atab = L.atab;
  int4* const acache = L.acache;
  uint32_t* const chgw = L.chgw;
  const int s = lane & (G - 1);
  const int gbase = lane & ~(G - 1);
  // envs per wave: 64 / G, or fewer (p.dyn_epw) to put more waves in flight -- lanes of groups
  // past it leave at once, like envs past B
  const int epw = p.dyn_epw > 0 ? p.dyn_epw : 64 / G;
  if (lane / G >= epw) return;
  const uint32_t b = wave * (uint32_t)epw + (uint32_t)(lane / G);
  if (b >= (uint32_t)p.B) return;  // whole groups leave together
  const int S = p.S, Q = p.Q;
  if (MODE == kModeReset && reset_mask != nullptr && reset_mask[b] == 0) return;

  LaneState<1> E;
  E.gid = p.env_id_offset + b;
  SrvLane V;
  V.act = s < S;
  V.over = 0u;
  uint32_t lfo_base = 0u;  // split: the env's lf_over at launch start (0 after a reset)
  V.scale = p.svc_scale[0];
#pragma unroll
  for (int k = 1; k < G; ++k) V.scale = (k == s) ? p.svc_scale[k] : V.scale;
  V.den = 1.0;
  V.rcp = 1.0;
  V.score = 0.f;
  V.assigned = 0;
  V.lh = 0;
#pragma unroll
  for (int w = 0; w < 4; ++w) chgw[w * 64 + lane] = 0u;
  V.chgw = chgw + lane;
  const uint32_t sb = b * (uint32_t)S + (uint32_t)s;
  float wall[G];
  float w_own = 1.0f;

  auto reset_in = [&]() {  // a new episode (env.py:186-213): its first arrival, empty servers
    E.episode = st.episode[b] + 1u;
    E.clock = 0u;
    E.dropped = 0u;
    E.arr_idx = 0u;
    draw_arrival<1>(st, p, E, 0);
    V.cnt = 0;
    V.head_tc = 0;
    V.head = 0;
    V.tail = 0;
    V.last = kLastNone;
    V.rcnt = 0u;
    V.qcap = Q;  // every server is up at the episode start
    V.big = false;
    V.lost = 0;  // n_flow_on_mode VPP: no lost flows yet
    V.rcnt_d = 0u;  // split: empty duration reservoir, no pending guesses
    V.phead = 0;
    V.pcnt = 0;
    V.pdue = 0u;
    lfo_base = 0u;
    if constexpr (FULL) {
      if (p.res_vpp && V.act) vpp_zero_bins(st, p, sb);  // VPP's zeroed bins
    }
    // emptied reservoirs: slot 0 marked written, so the next observe recomputes every server of
    // the env (its cached features are the last episode's)
    if (V.act) chgw[lane] = 1u;
#pragma unroll
    for (int k = 0; k < G; ++k) wall[k] = 1.0f;
  };
  auto load_in = [&]() {  // the env and this lane's server from HBM, the step's weights
    // Two HBM round trips: every word of the env and of the lane's server is requested before any
    // is waited for (lanes past S read server 0's words and ignore them: no branch whose compares
    // would wait inside it), then the queued entries of the 8-entry window at the head those words
    // give, all at once (the tail and the head time are among them unless the queue is longer).
    // The load-then-wait chain this replaces (hc, then one window entry after the other, then
    // the discrete weight table) was ~6 round trips at the start of every wave of a one-round
    // grid (profiles/r06o/).
    const uint32_t sbl = V.act ? sb : b * (uint32_t)S;
    E.episode = st.episode[b];
    E.clock = st.clock[b];
    E.dropped = st.dropped[b];
    E.arr_idx = st.arr_idx[b];
    E.next_arr = st.next_arr[b];
    E.next_work = st.next_work[b];
    E.u2 = st.next_u2[b];
    E.u3 = st.next_u3[b];
    const uint32_t hc = st.hc[sbl];
    const int32_t last = st.last_tc[sbl];
    const uint32_t rcnt = st.res_count[sbl];
    const float aw = action_weight_sel(p, action, action_dtype, (size_t)sbl);
    V.qcap = Q;
    V.lost = 0;
    V.rcnt_d = 0u;
    V.phead = 0;
    V.pcnt = 0;
    V.pdue = 0u;
    if (FULL && p.split) lfo_base = st.lf_over[b];
    if (FULL && V.act) {
      if (p.leak) V.lost = (int32_t)st.lost_on[sb];
      if (p.split) {
        V.rcnt_d = st.res_count_dur[sb];
        const uint32_t ph = st.pend_hc[sb];
        V.phead = (int32_t)(ph & 0xFFFFu);
        V.pcnt = (int32_t)(ph >> 16);
        if (V.pcnt > 0) V.pdue = st.pend[(size_t)sb * (uint32_t)p.pend_P + (uint32_t)V.phead].x;
      }
    }
    if (st.down != nullptr && V.act && st.down[sb] != 0u) V.qcap = 0;  // (fail_prob handles)
    const int head = V.act ? (int)(hc & kHcHead) : 0;
    const int cnt = V.act ? (int32_t)(hc >> 16) : 0;
    // (only the cnt queued entries: all 8 in every lane read 17 MB more at 65536 x 4, at the
    // moment every wave of the one-round grid loads its state -- 5 us slower, profiles/r06o/)
    int2 wv[WL];
    const int2* const row = st.ring + sbl * (uint32_t)Q;
#pragma unroll
    for (int i = 0; i < WL; ++i) wv[i] = make_int2(0, 0);
#pragma unroll
    for (int i = 0; i < WL; ++i) {
      if (i < cnt) {
        int pos = head + i;
        pos = pos >= Q ? pos - Q : pos;
        wv[i] = row[pos];
      }
    }
    V.head = head;
    V.big = V.act && (hc & kHcBig) != 0u;
    V.cnt = cnt;
    V.last = V.act ? last : kLastNone;
    V.rcnt = V.act ? rcnt : 0u;
#pragma unroll
    for (int i = 0; i < WL; ++i)
      if (i < cnt) win[i * 64 + lane] = wv[i];
    int32_t tail = wv[0].x;
#pragma unroll
    for (int i = 1; i < WL; ++i) tail = cnt == i + 1 ? wv[i].x : tail;
    if (cnt > WL) {  // a longer queue: its tail entry past the window
      int tp = head + cnt - 1;
      if (tp >= Q) tp -= Q;
      tail = row[tp].x;
    }
    V.tail = cnt > 0 ? tail : 0;
    V.head_tc = cnt > 0 ? wv[0].x : 0;
    if (V.act) w_own = aw;
    if constexpr (alias) {
#pragma unroll
      for (int k = 0; k < G; ++k)
        wall[k] = k < S ? action_weight(p, action, action_dtype, (size_t)b * S + (size_t)k) : 1.0f;
    }
  };
  auto reset_out = [&](int32_t ep_step) {  // episode counters; the warm-up's assignments are not
    V.assigned = 0;                        // the step's
    if (s == 0) {
      st.ep_step[b] = ep_step;
      st.ep_return[b] = 0.0;
    }
  };
  if constexpr (MODE == kModeStep) {
    load_in();
    sim_step_group<G, POLICY, TRACE, false, FULL>(st, p, E, V, b, s, gbase, w_own, wall, win, atab,
                                                  acache);
  } else if constexpr (MODE == kModeReset) {
    reset_in();
    for (int k = 0; k < p.warmup_steps; ++k)
      sim_step_group<G, POLICY, TRACE, false, FULL>(st, p, E, V, b, s, gbase, 1.0f, wall, win,
                                                    atab, acache);
    reset_out(0);
  } else {
    // kModeStepNR (next-step auto-reset): an env whose last step returned done resets in place of
    // stepping (its action ignored; ep_step = -1 tells the observe to report the reset).  One call
    // site, run warmup_steps times for a resetting group and once for the others (a wave with no
    // resetting group runs the plain step; one with some runs the longest trip, the others masked
    // off).  Two call sites, one per branch, took 133-137 VGPRs with scratch (3 waves per SIMD,
    // 190 us against the plain step's 149 at 65536 x 4, profiles/r06b/modes).
    const bool rs = st.ep_step[b] >= p.max_steps;
    if (rs) reset_in();
    else load_in();
    const int nsteps = rs ? p.warmup_steps : 1;
    const float w = rs ? 1.0f : w_own;
    for (int k = 0; k < nsteps; ++k)
      sim_step_group<G, POLICY, TRACE, LBSIM_DYN_NR_KEYS != 0, FULL>(st, p, E, V, b, s, gbase, w,
                                                                     wall, win, atab, acache);
    if (rs) reset_out(-1);
  }

  // ---- this lane's server back to HBM (window into the ring), then the env words (lane 0)
  if (V.act) {
    for (int i = 0; i < WL && i < V.cnt; ++i) {
      int pos = V.head + i;
      if (pos >= Q) pos -= Q;
      int li = V.lh + i;
      li = li >= WL ? li - WL : li;
      st.ring[sb * (uint32_t)Q + (uint32_t)pos] = win[li * 64 + lane];
    }
    if (p.big_in_step) {  // the in-step records this launch wrote (big_written)
      const uint32_t cw[4] = {chgw[lane], chgw[64 + lane], chgw[128 + lane], chgw[192 + lane]};
      __builtin_amdgcn_s_waitcnt(0);  // the wave's stores acknowledged by L2 (vmcnt 0)
      __asm__ volatile("" ::: "memory");
      V.big |= big_written(st, sb, cw, V.rcnt, V.rcnt_d);
    }
    if (FULL && p.split) {
      st.res_count_dur[sb] = V.rcnt_d;
      st.pend_hc[sb] = (uint32_t)V.phead | ((uint32_t)V.pcnt << 16);
    }
    st.hc[sb] = (uint32_t)V.head | (V.big ? kHcBig : 0u) | ((uint32_t)V.cnt << 16);
    st.last_tc[sb] = V.last;
    st.res_count[sb] = V.rcnt;
    if (st.down != nullptr) st.down[sb] = V.qcap == 0 ? 1u : 0u;
    if (FULL && p.leak) st.lost_on[sb] = (uint32_t)V.lost;
    *reinterpret_cast<uint4*>(st.chg + (size_t)sb * 4) =
        make_uint4(chgw[lane], chgw[64 + lane], chgw[128 + lane], chgw[192 + lane]);
    if (MODE != kModeReset && assign_out != nullptr) assign_out[sb] = V.assigned;  // 0 if reset
  }
  // split: the guesses this env's servers dropped at full rings (every lane of the group adds)
  const uint32_t over = (FULL && p.split) ? group_add<G>(V.over) : 0u;
  if (s == 0) {
    if (FULL && p.split) st.lf_over[b] = lfo_base + over;
    st.episode[b] = E.episode;
    st.clock[b] = E.clock;
    st.dropped[b] = E.dropped;
    st.arr_idx[b] = E.arr_idx;
    st.next_arr[b] = E.next_arr;
    st.next_work[b] = E.next_work;
    st.next_u2[b] = E.u2;
    st.next_u3[b] = E.u3;
  }
}

// WAVES: the occupancy the register allocation targets (1 = unconstrained: 100 VGPRs, 4 waves per
// SIMD).  WAVES = 5 (96 VGPRs, 2 spilled) pays only when the grid holds more than 4 waves per
// SIMD (262144 x 4: -6 %, 65536 x 8: -1.6 %) and costs 9 % at 65536 x 4, whose 4,096 waves are
// exactly 4 per SIMD (profiles/r03/ab_dyn_round_keys.txt): the launcher picks it by grid size.
template <int G, int MODE, int POLICY, bool TRACE, int WAVES = 1>
__global__ void __launch_bounds__(64, WAVES)
    dynamics_group_kernel(DevState st, SimParams p, const void* action, int action_dtype,
                          int32_t* assign_out, const uint8_t* reset_mask) {
  __shared__ DynGroupLds<POLICY> L;
  dyn_group_wave<G, MODE, POLICY, TRACE>(st, p, action, action_dtype, assign_out, reset_mask,
                                         blockIdx.x, (int)threadIdx.x, L);
}

// The same for a full handle (group_event_loop's FULL: n_flow_on_mode VPP, a duration plane,
// lost-FIN deferral, reservoir_mode VPP): the general event loop with every feature, on its own
// register budget.
template <int G, int MODE, int POLICY, bool TRACE>
__global__ void __launch_bounds__(64)
    dynamics_group_full_kernel(DevState st, SimParams p, const void* action, int action_dtype,
                               int32_t* assign_out, const uint8_t* reset_mask) {
  __shared__ DynGroupLds<POLICY> L;
  dyn_group_wave<G, MODE, POLICY, TRACE, true>(st, p, action, action_dtype, assign_out,
                                               reset_mask, blockIdx.x, (int)threadIdx.x, L);
}

}  // namespace lbk
