// lbsim_dyn_wave.h — dynamics with one WAVE per env, for batches too small to fill the chip
// (BASELINE configs[0] 1 x 4, configs[1] at 4096 x 4): the event loop is one env's dependent chain,
// so its length per arrival, not issue throughput, sets the step time.
//
// The server-per-lane kernel (lbsim_dyn_group.h) spends ~150 dependent instructions per event-loop
// iteration: a pop per iteration (extra iterations when two completions fall between arrivals), an
// LDS round trip for the next queue head and one for the next drawn arrival, two DPP reductions
// and the draw-ahead refill every G iterations.  Here the whole env is one wave and its state is
// laid out so that an arrival costs a few wave-wide instructions:
//   * ring lanes: the FIFO of server s is lanes 16 s .. 16 s + 15 of NR VGPR pairs {t_complete,
//     t_arrival}; ring position pos of server s is register pos >> 4, lane 16 s + (pos & 15), so
//     the HBM ring loads and stores lane for lane.  A 64-bit `live` mask per
//     register marks the flows still queued.  The pops before an arrival at ta are one v_cmp per
//     register (live &= ballot(t_complete > ta)): the completions due by ta leave in one step,
//     whatever their number (the oracle's pop_until, lbsim_oracle.c sim_step);
//   * server lanes: lane s < S holds server s's fields (write position, tail, Algorithm R count,
//     SED denominator); its flow count is the popcount of its 16 bits of `live`.  The choice is
//     the group kernel's lexicographic minimum (one DPP min over the quad, then a ballot of the
//     ties), the push one select in ring lane 16 c + (pos & 15) and one in server lane c;
//   * arrivals: 64 at a time, lane j drawing arrival base + j (its Philox block, gap and work, or
//     its trace row) with the arrival times as one wave prefix sum; the loop reads arrival k with
//     v_readlane (uniform, in SGPRs), so no LDS access and no draw sits on the chain.
// Same event sequence, same arithmetic, same state layout as the other two
// mappings: interchangeable between launches, bit-identical to the oracle.  S <= 4, Q <= 32 and the
// SED / SED2 / LSQ / LSQ2 policies (ALIAS and larger shapes use the group kernel: dyn_wave_ok in
// lbsim_internal.h).
#pragma once

#include "lbsim_dyn_group.h"

namespace lbk {

constexpr int kWaveRingLanes = 16;  // ring positions per server per VGPR (4 servers per wave)

template <int NR>
struct WaveRing {
  int32_t tc[NR], ta[NR];  // lane 16 s + k: ring position 16 r + k of server s
  uint64_t live[NR];       // lanes holding a queued flow (uniform)
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

struct WaveLds {
  int2 img[32 * 4];      // ring image [pos][server] for the carried-in walk and `last`
  uint32_t chg[4 * 4];   // written-slot masks [word][server]
};

__device__ __forceinline__ int32_t rdl(int32_t v, int l) { return __builtin_amdgcn_readlane(v, l); }
__device__ __forceinline__ uint32_t rdl(uint32_t v, int l) {
  return (uint32_t)__builtin_amdgcn_readlane((int)v, l);
}
__device__ __forceinline__ float rdl(float v, int l) {
  return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), l));
}

// Arrivals base .. base + 63 (lane j: arrival base + j), their times as offsets from t_prev, the
// time of arrival base - 1 (the oracle's draw_arrival chain next_arr = t_prev + gap).
template <bool TRACE>
__device__ __forceinline__ void wave_draw_batch(const DevState& st, const SimParams& p,
                                                const WaveEnv& E, uint32_t base, int32_t t_prev,
                                                int lane, int32_t& bta, float& bwk,
                                                uint32_t& bu2, uint32_t& bu3) {
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
  int32_t t = gap;  // inclusive prefix sum over the wave (integer: any order is exact)
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const int32_t v = __shfl_up(t, (unsigned)o, 64);
    t += lane >= o ? v : 0;
  }
  bta = t_prev + t;
  bwk = wk;
  bu2 = d.z;
  bu3 = d.w;
}

// Flows of server lane s queued now (its 16 bits of each live mask).
template <int NR>
__device__ __forceinline__ int32_t wave_count(const WaveRing<NR>& R, int s4) {
  int32_t n = 0;
#pragma unroll
  for (int r = 0; r < NR; ++r)
    n += __builtin_popcount((uint32_t)(R.live[r] >> (16 * s4)) & 0xFFFFu);
  return n;
}

// One step of the env, w_own = this server lane's weight.
template <int NR, int POLICY, bool TRACE, bool FAST>
__device__ __forceinline__ void wave_event_loop(const DevState& st, const SimParams& p,
                                                WaveEnv& E, WaveSrv& V, WaveRing<NR>& R,
                                                int lane, uint3* const res_b, uint32_t* chg,
                                                uint32_t base_ms, uint32_t base_rem) {
  constexpr bool two_choice = (POLICY == 1 || POLICY == 3);
  constexpr bool lsq = (POLICY == 2 || POLICY == 3);
  const int S = p.S, Q = p.Q;
  const int32_t dt = p.dt_us;
  const int s4 = lane & 3;
  int bi = 64;  // batch lane of the next arrival (64: draw a batch first)
  int32_t bta = 0;
  float bwk = 0.f;
  uint32_t bu2 = 0u, bu3 = 0u;
  while (E.next_arr < dt) {
    const int32_t ta = E.next_arr;
    // ---- completions due by ta leave the queues
#pragma unroll
    for (int r = 0; r < NR; ++r) R.live[r] &= __ballot(R.tc[r] > ta);
    const int32_t n = wave_count<NR>(R, s4);

    // ---- the arrival's server (node.c:388-441); full servers are not eligible
    float score = 0.f;
    if constexpr (lsq) {
      score = (float)n;
    } else {
      const double c = (double)(n + 1);
      const double q0 = c * V.rcp;
      double q = fma(fma(-q0, V.den, c), V.rcp, q0);
      if (!FAST && q != q) {
        asm volatile("");
        q = c / V.den;
      }
      score = (float)q;
    }
    const bool elig = V.act && n < Q;
    int c = -1;
    if constexpr (two_choice) {
      const int h1 = two_choice_h1(E.u2, S);
      const int h2 = two_choice_h2(E.u2, S);
      const uint32_t em = (uint32_t)__ballot(elig) & 0xFu;
      const float s1 = rdl(score, h1), s2 = rdl(score, h2);
      const bool ok1 = (em >> h1) & 1u, ok2 = (em >> h2) & 1u;
      c = (ok1 && ok2) ? ((s2 < s1) ? h2 : h1) : (ok1 ? h1 : (ok2 ? h2 : -1));
    } else if constexpr (FAST) {
      // finite scores: the eligible minimum, h among equal minima, else the lowest such server
      const int32_t key = elig ? f32_key(score) : 0x7FFFFFFF;
      const int32_t mk = __builtin_amdgcn_readfirstlane(group_min_i32<4>(key));
      if (mk != 0x7FFFFFFF) {
        const int h = (int)__umulhi(E.u2, (uint32_t)S);
        const uint32_t tie = (uint32_t)__ballot(elig && key == mk) & 0xFu;
        c = ((tie >> h) & 1u) ? h : __builtin_ctz(tie);
      }
    } else {
      const bool num = elig && score == score;
      const float m = key_f32(
          __builtin_amdgcn_readfirstlane(group_min_i32<4>(num ? f32_key(score) : 0x7f800000)));
      const int h = (int)__umulhi(E.u2, (uint32_t)S);
      const uint32_t em = (uint32_t)__ballot(elig) & 0xFu;
      const int c0 = ((em >> h) & 1u) ? h : (em ? __builtin_ctz(em) : -1);
      const uint32_t tie = (uint32_t)__ballot(num && score == m) & 0xFu;
      const uint32_t nan = (uint32_t)__ballot(score != score) & 0xFu;
      c = c0 < 0 ? -1 : ((((tie | nan) >> c0) & 1u) ? c0 : (tie ? __builtin_ctz(tie) : -1));
    }

    if (c >= 0) {
      // ---- FIFO service on server c: every server lane prices the flow, lane c's is pushed
      const int32_t start_l = n > 0 ? (V.tail > ta ? V.tail : ta) : ta;
      int32_t svc_l = (int32_t)(E.next_work * V.scale);
      svc_l = svc_l < 1 ? 1 : svc_l;
      const int32_t tc = rdl(start_l + svc_l, c);
      const int pos = rdl(V.wp, c);
      const int L = c * kWaveRingLanes + (pos & (kWaveRingLanes - 1));
      const bool me = lane == c;
      if (NR == 1 || pos < kWaveRingLanes) {
        if (rdl(n, c) == Q - 1) {  // this push fills the ring: keep the last popped t_complete
          const int32_t old = rdl(R.tc[0], L);
          V.saved = me ? old : V.saved;
        }
        R.tc[0] = lane == L ? tc : R.tc[0];
        R.ta[0] = lane == L ? ta : R.ta[0];
        R.live[0] |= 1ull << L;
      } else {
        if (rdl(n, c) == Q - 1) {
          const int32_t old = rdl(R.tc[NR - 1], L);
          V.saved = me ? old : V.saved;
        }
        R.tc[NR - 1] = lane == L ? tc : R.tc[NR - 1];
        R.ta[NR - 1] = lane == L ? ta : R.ta[NR - 1];
        R.live[NR - 1] |= 1ull << L;
      }
      V.tail = me ? tc : V.tail;
      V.wp = me ? (V.wp + 1 == Q ? 0 : V.wp + 1) : V.wp;
      V.assigned += me ? 1 : 0;
      V.pushed += me ? 1 : 0;
      if (tc <= dt) {  // completes in this step: its sample now, with its arrival's draw word
        const uint32_t rc = rdl(V.rcnt, c);
        const int slot = reservoir_slot_r32(rc, E.u3);
        if (slot >= 0 && me) {
          res_b[(uint32_t)c * K + (uint32_t)slot] =
              make_uint3((uint32_t)(tc - ta), (uint32_t)(tc - rdl(start_l, c)),
                         base_ms + (base_rem + (uint32_t)tc) / 1000u);
          atomicOr(chg + ((uint32_t)slot >> 5) * 4u + (uint32_t)c, 1u << (slot & 31));
        }
        V.rcnt = me ? count_inc(rc) : V.rcnt;
      }
    } else {
      E.dropped += 1u;
    }

    // ---- the next arrival: arrival arr_idx + 1 from the batch
    if (bi == 64) {
      wave_draw_batch<TRACE>(st, p, E, E.arr_idx + 1u, ta, lane, bta, bwk, bu2, bu3);
      bi = 0;
    }
    E.next_arr = rdl(bta, bi);
    E.next_work = rdl(bwk, bi);
    E.u2 = rdl(bu2, bi);
    E.u3 = rdl(bu3, bi);
    E.arr_idx += 1u;
    ++bi;
  }
}

template <int NR, int POLICY, bool TRACE>
__device__ __forceinline__ void sim_step_wave(const DevState& st, const SimParams& p, WaveEnv& E,
                                              WaveSrv& V, WaveRing<NR>& R, int lane,
                                              uint3* const res_b, WaveLds& Ld, float w_own) {
  constexpr bool lsq = (POLICY == 2 || POLICY == 3);
  const int S = p.S, Q = p.Q;
  const int32_t dt = p.dt_us;
  const uint64_t base_us = (uint64_t)E.clock * (uint64_t)dt;
  const uint32_t base_ms = (uint32_t)(base_us / 1000u);
  const uint32_t base_rem = (uint32_t)(base_us - (uint64_t)base_ms * 1000u);
  const int rs = lane >> 4, rk = lane & (kWaveRingLanes - 1);  // ring lane: server, position
  if (V.act && !lsq) {
    V.den = (double)w_own + 1e-9;
    V.rcp = 1.0 / V.den;
  }
  V.pushed = 0;

  // ---- 1. carried-in flows that complete in this step, server lane by server lane, in FIFO
  //      order (their Algorithm R draws from the reservoir stream)
#pragma unroll
  for (int r = 0; r < NR; ++r) {
    const int pos = r * kWaveRingLanes + rk;
    if (rs < S && pos < Q) Ld.img[pos * 4 + rs] = make_int2(R.tc[r], R.ta[r]);
  }
  wave_sync();
  if (V.act && V.cnt0 > 0) {
    int pos = V.wp - V.cnt0;
    pos = pos < 0 ? pos + Q : pos;
    int32_t prev = V.last;
    uint32_t rc = V.rcnt;
    for (int i = 0; i < V.cnt0; ++i) {
      const int2 e = Ld.img[pos * 4 + lane];
      if (e.x > dt) break;
      const u32x4 d = philox4x32_10(
          u32x4{rc >> 1, E.gid, E.episode, (kStreamReservoir << 24) | (uint32_t)lane}, p.key0,
          p.key1);
      const int slot = reservoir_slot(rc, d);
      if (slot >= 0) {
        res_b[(uint32_t)lane * K + (uint32_t)slot] =
            make_uint3((uint32_t)(e.x - e.y), (uint32_t)(e.x - (e.y > prev ? e.y : prev)),
                       base_ms + (base_rem + (uint32_t)e.x) / 1000u);
        atomicOr(Ld.chg + ((uint32_t)slot >> 5) * 4u + (uint32_t)lane, 1u << (slot & 31));
      }
      prev = e.x;
      rc = count_inc(rc);
      pos = pos + 1 == Q ? 0 : pos + 1;
    }
    V.rcnt = rc;
  }

  // ---- 2. the arrivals (SED / SED2 scores are finite unless some den is 0 / inf / NaN)
  const bool finite = lsq || !V.act || (fabs(V.den) >= 1e-30 && fabs(V.den) <= 1e300);
  if (__all(finite))
    wave_event_loop<NR, POLICY, TRACE, true>(st, p, E, V, R, lane, res_b, Ld.chg, base_ms,
                                             base_rem);
  else
    wave_event_loop<NR, POLICY, TRACE, false>(st, p, E, V, R, lane, res_b, Ld.chg, base_ms,
                                              base_rem);

  // ---- 3. completions up to dt; the server's count, head and last completion
#pragma unroll
  for (int r = 0; r < NR; ++r) R.live[r] &= __ballot(R.tc[r] > dt);
  const int32_t n = wave_count<NR>(R, lane & 3);
#pragma unroll
  for (int r = 0; r < NR; ++r) {
    const int pos = r * kWaveRingLanes + rk;
    if (rs < S && pos < Q) Ld.img[pos * 4 + rs].x = R.tc[r];
  }
  wave_sync();
  if (V.act && V.cnt0 + V.pushed > n) {  // a flow completed this step: the newest one
    if (n == Q) {
      V.last = V.saved;
    } else {
      int pl = V.wp - n - 1;
      pl = pl < 0 ? pl + Q : pl;
      pl = pl < 0 ? pl + Q : pl;
      V.last = Ld.img[pl * 4 + lane].x;
    }
  }
  wave_sync();
  V.cnt0 = n;
  // ---- rebase to the next step's start
  E.next_arr -= dt;
#pragma unroll
  for (int r = 0; r < NR; ++r) {
    R.tc[r] -= dt;
    R.ta[r] -= dt;
  }
  V.tail -= dt;
  V.last = (V.last < kLastNone + dt) ? kLastNone : V.last - dt;
  E.clock += 1u;
}

// One dynamics launch for env b (one wave): state in, the step (or reset + warm-up), state out.
template <int NR, int MODE, int POLICY, bool TRACE>
__global__ void __launch_bounds__(64)
    dynamics_wave_kernel(DevState st, SimParams p, const void* action, int action_dtype,
                         int32_t* assign_out, const uint8_t* reset_mask) {
  __shared__ WaveLds Ld;
  const uint32_t b = blockIdx.x;
  if (b >= (uint32_t)p.B) return;
  if (MODE == kModeReset && reset_mask != nullptr && reset_mask[b] == 0) return;
  const int lane = (int)threadIdx.x;
  const int S = p.S, Q = p.Q;
  const int rs = lane >> 4, rk = lane & (kWaveRingLanes - 1);
  uint3* const res_b = st.res + (size_t)b * (size_t)S * K;

  WaveEnv E;
  E.gid = p.env_id_offset + b;
  WaveSrv V;
  V.act = lane < S;
  V.scale = p.svc_scale[0];
#pragma unroll
  for (int k = 1; k < 4; ++k) V.scale = (k == lane) ? p.svc_scale[k] : V.scale;
  V.den = 1.0;
  V.rcp = 1.0;
  V.assigned = 0;
  V.saved = 0;
  if (lane < 16) Ld.chg[lane] = 0u;
  WaveRing<NR> R;
#pragma unroll
  for (int r = 0; r < NR; ++r) {
    R.tc[r] = 0;
    R.ta[r] = 0;
    R.live[r] = 0ull;
  }
  const uint32_t sb = b * (uint32_t)S + (uint32_t)lane;  // server lane's server (lane < S)

  if (MODE == kModeReset) {
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
    wave_sync();
    for (int k = 0; k < p.warmup_steps; ++k)
      sim_step_wave<NR, POLICY, TRACE>(st, p, E, V, R, lane, res_b, Ld, 1.0f);
    if (lane == 0) {
      st.ep_step[b] = 0;
      st.ep_return[b] = 0.0;
    }
  } else {
    E.episode = st.episode[b];
    E.clock = st.clock[b];
    E.dropped = st.dropped[b];
    E.arr_idx = st.arr_idx[b];
    E.next_arr = st.next_arr[b];
    E.next_work = st.next_work[b];
    E.u2 = st.next_u2[b];
    E.u3 = st.next_u3[b];
    // ring lanes: this lane's ring positions, live if within [head, head + count)
    bool lv[NR];
#pragma unroll
    for (int r = 0; r < NR; ++r) lv[r] = false;
    if (rs < S) {
      const uint32_t hc = st.hc[b * (uint32_t)S + (uint32_t)rs];
      const int head = (int)(hc & 0xFFFFu), cnt = (int)(hc >> 16);
      const int2* ring = st.ring + (size_t)(b * (uint32_t)S + (uint32_t)rs) * (size_t)Q;
#pragma unroll
      for (int r = 0; r < NR; ++r) {
        const int pos = r * kWaveRingLanes + rk;
        if (pos < Q) {
          int rel = pos - head;
          rel = rel < 0 ? rel + Q : rel;
          lv[r] = rel < cnt;
          if (lv[r]) {
            const int2 e = ring[pos];
            R.tc[r] = e.x;
            R.ta[r] = e.y;
          }
        }
      }
    }
#pragma unroll
    for (int r = 0; r < NR; ++r) R.live[r] = __ballot(lv[r]);
    V.cnt0 = 0;
    V.wp = 0;
    V.tail = 0;
    V.last = kLastNone;
    V.rcnt = 0u;
    float w_own = 1.0f;
    if (V.act) {
      const uint32_t hc = st.hc[sb];
      const int head = (int)(hc & 0xFFFFu);
      V.cnt0 = (int32_t)(hc >> 16);
      int wp = head + V.cnt0;
      V.wp = wp >= Q ? wp - Q : wp;
      V.last = st.last_tc[sb];
      V.rcnt = st.res_count[sb];
      if (V.cnt0 > 0) {
        const int tp = V.wp == 0 ? Q - 1 : V.wp - 1;
        V.tail = st.ring[(size_t)sb * (size_t)Q + (size_t)tp].x;
      }
      w_own = action_weight(p, action, action_dtype, (size_t)sb);
    }
    wave_sync();
    sim_step_wave<NR, POLICY, TRACE>(st, p, E, V, R, lane, res_b, Ld, w_own);
  }

  // ---- state out: the queued flows, the server fields, the env words
  if (rs < S) {
    int2* ring = st.ring + (size_t)(b * (uint32_t)S + (uint32_t)rs) * (size_t)Q;
#pragma unroll
    for (int r = 0; r < NR; ++r) {
      const int pos = r * kWaveRingLanes + rk;
      if (pos < Q && ((R.live[r] >> lane) & 1ull)) ring[pos] = make_int2(R.tc[r], R.ta[r]);
    }
  }
  wave_sync();
  if (V.act) {
    int head = V.wp - V.cnt0;
    head = head < 0 ? head + Q : head;
    st.hc[sb] = (uint32_t)head | ((uint32_t)V.cnt0 << 16);
    st.last_tc[sb] = V.last;
    st.res_count[sb] = V.rcnt;
    *reinterpret_cast<uint4*>(st.chg + (size_t)sb * 4) =
        make_uint4(Ld.chg[lane], Ld.chg[4 + lane], Ld.chg[8 + lane], Ld.chg[12 + lane]);
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
}

}  // namespace lbk
