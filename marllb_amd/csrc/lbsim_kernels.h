// lbsim_kernels.h — gfx950 kernels of the vectorised LB environment.
//
//   dynamics_kernel<MAXS>  one LANE per env: Poisson arrivals -> SED/LSQ assignment (node.c:388-441)
//                          -> per-server FIFO service -> completion samples (lbhash.h:116-135) ->
//                          Algorithm R reservoir inserts (reservoir.py:50-85).  Integer/fp32
//                          sequential work whose trip count differs per env, so lanes (not waves)
//                          carry envs; state stays in VGPRs for the whole step.
//   observe_kernel         one WAVE per env: per server, the 128-slot reservoirs are read
//                          coalesced (2 slots/lane), bitonic-sorted across the wave, and reduced
//                          into the 11-column observation (features.py:256-286), then reward
//                          (rewards.py:290-381), done/return bookkeeping (env.py:261-281) and
//                          optional running normalisation (env.py:450-470).
//   features_kernel        the observe-kernel feature routine on caller-given reservoirs.
//   reward_kernel          the observe-kernel reward routine on caller-given observations.
//
// Bit-reproducibility rules: compiled with -ffp-contract=off; only IEEE basic
// ops on the state path; every floating sum that feeds an output follows numpy's pairwise order.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "lbsim_math.h"

namespace lbk {

constexpr int K = 128;   // reservoir slots (reservoir.py:31)
constexpr int NF = 11;   // observation columns (env.py:46-48)
constexpr int MAX_S = 64;  // LBSIM_MAX_SERVERS (S > 16: the server-per-lane dynamics only)
constexpr int32_t kLastNone = -(1 << 30);
constexpr int kModeStep = 0;
// s_waitcnt immediate with vmcnt = 0 and expcnt/lgkmcnt left at their maxima (gfx9 encoding).
constexpr int kWaitVmcnt0 = 0x0F70;
constexpr int kModeReset = 1;
// A step launch of a handle with next-step auto-reset (lbsim_config_t::next_step_reset): the
// dynamics reset, in place of stepping, the envs whose last step returned done.  A separate
// instantiation, so the default step kernels carry none of the reset code.
constexpr int kModeStepNR = 2;

struct DevState {
  // per env [B]
  int32_t* next_arr;    // relative us of the next arrival (>= 0 after rebase)
  float* next_work;     // Exp(1) work of the next arrival
  uint32_t* next_u2;    // hash word of the next arrival (SED start; 2-choice: both candidates)
  uint32_t* next_u3;    // Algorithm R draw word of the next arrival's flow (reservoir_slot_r32)
  uint32_t* arr_idx;    // Philox counter of the next arrival
  uint32_t* episode;    // episode index (RNG counter word z)
  uint32_t* clock;      // simulated steps since reset (warm-up included)
  int32_t* ep_step;     // user-visible step in episode (env.py:230)
  uint32_t* dropped;    // arrivals dropped because every server queue was full (this episode)
  int32_t* norm_count;  // running-normalisation count (env.py:461)
  double* ep_return;    // episode return (env.py:264)
  // per server [B*S]
  uint32_t* hc;         // ring head | count << 16
  int32_t* last_tc;     // completion time of the last popped flow (relative us)
  uint32_t* res_count;  // samples offered to the reservoirs (Algorithm R count)
  // ring [B*S*Q] of {t_complete, t_arrival}, relative us
  int2* ring;
  // reservoirs [B*S*K]; flow completion time / duration samples in integer microseconds (the
  // feature value of a sample is (float)us * 1e-6f seconds, us_to_seconds)
  uint2* res;           // [B*S*K] slot records {fct us, timestamp ms}: an insert is one 8-B store
                        // (global_store_dwordx2), a server's 128 records are 1 KiB
  // [B*S*K] duration us of each slot, only when a record's duration can differ from its fct
  // (duration_mode SERVICE, or lost-FIN guesses); nullptr otherwise: the duration reservoir IS
  // the fct reservoir (paired records), and observe reads 8 B per slot
  uint32_t* res_dur;
  // unchanged-reservoir skip of observe: chg[(b*S + s)*4 + w] bit i set if slot
  // 32 w + i of server s was written by the last dynamics launch (its two reservoirs share every
  // replacement decision); fcache[(b*S + s)*10 + f] = the server's 10 reservoir features at the
  // last observe.  A server whose reservoirs were not written keeps the same features (values,
  // timestamps and n = min(count, K) are unchanged: count only grows without a write once full).
  uint32_t* chg;
  float* fcache;
  // server failures (only if fail_prob > 0, else nullptr): down[b*S + s] = 1 while server s is down
  uint32_t* down;
  // n_flow_on_mode VPP with lost-FIN (SimParams::leak, else nullptr): lost_on[b*S + s] = lost-FIN
  // flows of server s completed since the episode start / its last failure, never decremented
  // (lbhash.h:193,214); observation column 0 adds it (n_flow_on)
  uint32_t* lost_on;
  // lost-FIN deferral (SimParams::split, else nullptr): the duration reservoir's
  // own count [B*S] (res_dur is then [B*S*K] {duration us, timestamp ms} records, read as uint2),
  // each server's pending timed-out fct guesses [B*S*P] {due us mod 2^32 (absolute: clock * dt +
  // t), guess us} sorted by due time with pend_hc = head | count << 16 [B*S], and lf_over [B]:
  // guesses dropped at a full ring this episode
  uint32_t* res_count_dur;
  uint32_t* pend_hc;
  uint2* pend;
  uint32_t* lf_over;
  // stateless features API only: caller's separate value / timestamp arrays [n*K]
  const uint32_t* feat_vals;
  const uint32_t* feat_ts;
  // running normalisation [B*S*11] (nullptr when disabled)
  double* norm_mean;
  double* norm_std;
  // arrival trace (TRACE source; nullptr otherwise), shared by all envs: us gap before each row,
  // mean-1 work of each row
  const uint32_t* trace_gap;
  const float* trace_work;
};

struct SimParams {
  int32_t B, S, Q;
  int32_t dt_us;
  float mean_gap_us;
  float svc_scale[MAX_S];
  uint32_t key0, key1;
  uint32_t env_id_offset;
  int32_t policy;
  int32_t action_type;
  int32_t num_discrete;
  float dw[8];
  float min_w, max_w;
  int32_t warmup_steps;
  int32_t max_steps;
  int32_t reward_metric;
  int32_t reward_field;
  float decay_c;  // log2(decay_factor) / 1000, per integer millisecond of age
  int32_t normalize;
  int32_t trace;          // 1: arrivals replay the trace (LBSIM_ARRIVAL_TRACE)
  uint32_t trace_rows;
  // lost-FIN flows (lost_fct): 24-bit probability threshold (0 = off), flow_timeout - 40 s in us,
  // mean bucket wait in us
  uint32_t lf_thr;
  int32_t lf_off_us;
  float lf_wait_us;
  // server failure / recovery (fail_transitions): 24-bit thresholds per server-step (fail 0 = off)
  uint32_t fail_thr, rec_thr;
  // a flow that arrives and completes in one step can store a sample >= kPackLimit (the kHcBig
  // flag then needs tracking inside the event loop): only with dt >= kPackLimit us or lost-FIN
  // guesses (an in-step fct is <= dt and its duration <= its fct otherwise)
  int32_t big_in_step;
  // next-step auto-reset (lbsim_config_t::next_step_reset): a step launch resets the envs whose
  // last step returned done (ep_step >= max_steps) instead of stepping them
  int32_t next_reset;
  // envs per wave of dynamics_group_kernel (0: 64 / G, every lane used); set by its launcher
  int32_t dyn_epw;
  // lbsim_config_t::duration_mode == SERVICE (dur_sample): the duration sample is the service
  // time, not the flow's age
  int32_t dur_service;
  // n_flow_on_mode VPP and lost-FIN on: count the lost flows per server (DevState::lost_on)
  int32_t leak;
  // lost-FIN on: split fct / duration reservoirs and deferred guesses (DevState::pend), P entries
  // per server; the wrap-up delay of a guess is lf_off_us + 40 s + its wait
  int32_t split, pend_P;
  // reservoir_mode VPP: every sample overwrites slot rand() % 128 (lbhash.h:108,179), bins zeroed
  // at reset / failure
  int32_t res_vpp;
};

constexpr uint32_t kStreamFailure = 5u;  // Philox stream of the failure / recovery draws

// us << 7 | slot must stay below the 0xFFFFFFFF filler of empty slots (observe's one-pass sort).
constexpr uint32_t kPackLimit = (1u << 25) - 1u;
// DevState::hc = ring head | kHcBig | count << 16 (head < Q <= 64).  kHcBig is sticky: a record
// with a sample >= kPackLimit us (as an unsigned word: negative lost-FIN guesses included) was
// stored in the server's reservoirs since they were last emptied (reset, failure).  Observe's
// register-resident path (one-pass sort of us << 7 | slot) needs every sample below kPackLimit;
// the flag lets it decide from the hc word it loads anyway, without a pass over the records.
constexpr uint32_t kHcBig = 1u << 15;
constexpr uint32_t kHcHead = kHcBig - 1u;
__device__ __forceinline__ bool big_record(uint32_t fct, uint32_t dur) {
  return (fct > dur ? fct : dur) >= kPackLimit;
}
// When it is set: a carried-in flow's record (its fct spans earlier steps) at its store; a record
// of a flow that arrived and completed in the launch's steps only if such a record can be big
// (SimParams::big_in_step: dt >= kPackLimit us, or lost-FIN guesses), by one scan of the slots
// the launch wrote (below the count) at its end -- nothing in the event loop.  oracle: the same.
// The record words are read device-coherent: in the wave kernel other lanes stored them.
// sb: the (env, server) row; its duration words from the duration plane when the handle has one.
__device__ __forceinline__ bool big_written(const DevState& st, size_t sb,
                                            const uint32_t (&chg)[4], uint32_t count,
                                            uint32_t count_dur = 0u) {
  const uint32_t n = count < (uint32_t)K ? count : (uint32_t)K;
  const uint32_t* fs = reinterpret_cast<const uint32_t*>(st.res + sb * K);
  // a split handle's duration reservoir: {us, ts} records with their own count
  const bool split = st.res_count_dur != nullptr;  // count_dur: the lane's register copy
  const uint32_t cd = split ? count_dur : count;
  const uint32_t nd = cd < (uint32_t)K ? cd : (uint32_t)K;
  const uint32_t* ds = st.res_dur != nullptr ? st.res_dur + sb * K * (split ? 2u : 1u) : nullptr;
  const uint32_t dstep = split ? 2u : 1u;
  bool big = false;
  for (int w = 0; w < 4; ++w) {
    uint32_t m = chg[w];
    while (m) {
      const uint32_t slot = 32u * (uint32_t)w + (uint32_t)__builtin_ctz(m);
      m &= m - 1u;
      if (slot >= n && slot >= nd) continue;
      const uint32_t f = slot < n ? __hip_atomic_load(fs + 2 * slot, __ATOMIC_RELAXED,
                                                      __HIP_MEMORY_SCOPE_AGENT) : 0u;
      const uint32_t d = slot >= nd ? 0u
                         : (ds != nullptr ? __hip_atomic_load(ds + dstep * slot, __ATOMIC_RELAXED,
                                                              __HIP_MEMORY_SCOPE_AGENT)
                                          : f);
      big |= big_record(f, d);
    }
  }
  return big;
}

// A reservoir insert: the {fct, ts} record (one dwordx2 store) and, when the handle has a duration
// plane, the duration word.  idx = (env, server) row * K + slot.
__device__ __forceinline__ void store_record(const DevState& st, size_t idx, uint32_t fct,
                                             uint32_t dur, uint32_t ts_ms) {
  st.res[idx] = make_uint2(fct, ts_ms);
  if (st.res_dur != nullptr) st.res_dur[idx] = dur;
}

// murmur3's 32-bit finaliser (fmix32): the lost-FIN hash.
__device__ __forceinline__ uint32_t lf_mix(uint32_t h) {
  h ^= h >> 16;
  h *= 0x85EBCA6Bu;
  h ^= h >> 13;
  h *= 0xC2B2AE35u;
  h ^= h >> 16;
  return h;
}

// fct + off + wait as a signed int32 us sample, saturated (the config bound keeps it in range for
// Poisson work; trace work is unbounded).  oracle: the same.
// With fct in [0, 2^31), |off| <= 1000 s (lbsim_config_validate) and wait >= 0, fct + off cannot
// overflow and the sum can only pass INT32_MAX: two saturating 32-bit adds (v_add_i32 clamp)
// give the 64-bit sum clamped, without 64-bit registers in the event loop.
__device__ __forceinline__ uint32_t lf_guess(uint32_t fct, int32_t off, int32_t wait) {
  const int32_t a = __builtin_elementwise_add_sat((int32_t)fct, off);
  return (uint32_t)__builtin_elementwise_add_sat(a, wait);
}

// The fct sample of a completed flow, fct = tc - ta (lbhash.h:116-124, RSTACK: now - t_init), or,
// for a flow whose FIN/RST the data plane missed (probability lost_fin_prob), VPP's timed-out guess
// (lbhash.h:175-217): the entry expires flow_timeout after the flow's last packet (its completion),
// the next flow hashed into the bucket takes it after an exponential wait of mean flow_buckets /
// arrival_rate, and the plugin records now - t_init - LB_DEFAULT_FLOW_TIMEOUT (40 s, stats.h:27)
// = fct + flow_timeout - 40 s + wait, signed us.  Lost or not and the wait are a hash of (seed,
// global env id, episode, the flow's absolute arrival us mod 2^32): a pure function of the flow,
// the same whichever step, kernel or shard records it (oracle_lost_fin_fct).  abs_ta =
// (uint32)(clock * dt) + ta.  Off (lf_thr == 0, a uniform branch): fct unchanged.
__device__ __forceinline__ uint32_t lost_fct(const SimParams& p, uint32_t fct, uint32_t abs_ta,
                                             uint32_t gid, uint32_t episode) {
  if (p.lf_thr == 0u) return fct;
  const uint32_t salt =
      lf_mix(lf_mix(p.key0 ^ (episode * 0x9E3779B9u)) ^ gid ^ (p.key1 * 0x85EBCA6Bu));
  const uint32_t h = lf_mix(abs_ta ^ salt);
  if ((h >> 8) >= p.lf_thr) return fct;
  const uint32_t h2 = lf_mix(h ^ 0x6A09E667u);
  const int32_t wait = (int32_t)(-lb_logf(u01_open0(h2)) * p.lf_wait_us);
  return lf_guess(fct, p.lf_off_us, wait);
}

// The flow-duration sample of a flow completing at tc that arrived at ta.  AGE
// (default): the flow's age at its last data packet, tc - ta -- VPP records time_now - t_init on
// every plain ACK after the first (lbhash.h:129-136), the last one at the completion -- so the
// backlog wait is in it.  SERVICE (p.dur_service, a uniform branch): tc - start, start = max(ta,
// the predecessor's tc), the service time alone.
__device__ __forceinline__ uint32_t dur_sample(const SimParams& p, int32_t tc, int32_t ta,
                                               int32_t start) {
  return (uint32_t)(tc - (p.dur_service ? start : ta));
}

// Lost or not, and the bucket wait in us (oracle lf_test), of the flow that arrived at abs_ta.
__device__ __forceinline__ bool lf_wait(const SimParams& p, uint32_t abs_ta, uint32_t gid,
                                        uint32_t episode, int32_t& wait) {
  const uint32_t salt =
      lf_mix(lf_mix(p.key0 ^ (episode * 0x9E3779B9u)) ^ gid ^ (p.key1 * 0x85EBCA6Bu));
  const uint32_t h = lf_mix(abs_ta ^ salt);
  if ((h >> 8) >= p.lf_thr) return false;
  const uint32_t h2 = lf_mix(h ^ 0x6A09E667u);
  wait = (int32_t)(-lb_logf(u01_open0(h2)) * p.lf_wait_us);
  return true;
}

// Whether the flow that arrived at abs_ta is a lost-FIN flow (the test of lost_fct).
__device__ __forceinline__ bool lf_lost(const SimParams& p, uint32_t abs_ta, uint32_t gid,
                                        uint32_t episode) {
  const uint32_t salt =
      lf_mix(lf_mix(p.key0 ^ (episode * 0x9E3779B9u)) ^ gid ^ (p.key1 * 0x85EBCA6Bu));
  return (lf_mix(abs_ta ^ salt) >> 8) < p.lf_thr;
}

// n_flow_on_mode VPP (p.leak): a lost-FIN flow adds one to its server's lost_on count when it is
// popped (its completion), whether or not Algorithm R keeps its sample, so that from then on the
// server's n_flow_on -- the observation's column 0 and the SED / LSQ scores of the arrivals after
// it -- keeps it (lbhash.h:193,214 never decrement it; node.c:395-437 score on it).  The kernels
// keep the count in registers during the event loop (the general loop: leak handles never run the
// FAST one) and store it at the end; oracle: pop_until, score_of.

// Observation column 0: the server's flows in flight, plus its lost-FIN flows under n_flow_on_mode
// VPP (read device-coherent: the one-launch forms observe right after their own dynamics).
__device__ __forceinline__ float n_flow_on(const DevState& st, size_t sb) {
  uint32_t n = st.hc[sb] >> 16;
  if (st.lost_on != nullptr)
    n += __hip_atomic_load(st.lost_on + sb, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  return (float)n;
}

constexpr uint32_t kTraceEnvStride = 7919u;        // SURVEY §8d C3 per-env offset
constexpr uint32_t kTraceEpisodeStride = 1000003u;  // next episode, another window

// Trace row of arrival k of env gid in episode `episode` (>= 1).
__device__ __forceinline__ uint32_t trace_row(const SimParams& p, uint32_t gid, uint32_t episode,
                                              uint32_t k) {
  const uint64_t v = (uint64_t)gid * kTraceEnvStride +
                     (uint64_t)(episode - 1u) * kTraceEpisodeStride + (uint64_t)k;
  return (uint32_t)(v % (uint64_t)p.trace_rows);
}

// ================================================================ dynamics (one lane = one env)

// Queue window in LDS: the first WL entries of each server's FIFO live in LDS, laid out
// [server][slot][lane] so a wave's 64 per-lane ds_read_b64 of one (server, slot) pair are
// conflict-free whatever slot each lane is at.  The event loop then reads no global memory (a
// global load there forces s_waitcnt vmcnt(0) behind every outstanding store, which at one wave
// per SIMD serialises the loop on memory latency) and writes the HBM ring only for queue entries
// at index >= WL (an entry's index only decreases, so such entries stay in HBM until a refill
// brings them into the window).  At kernel exit the window is written back, so between kernels
// the HBM ring holds every in-flight flow (the snapshot layout of DESIGN.md §4).  Most flows are
// born and complete inside one step and never touch HBM.
template <int MAXS>
struct Win {
  static constexpr int WL = MAXS <= 4 ? 8 : (MAXS <= 8 ? 4 : 2);  // LDS <= 16 / 16 / 16 KiB
  static_assert((WL & (WL - 1)) == 0, "window slots wrap by mask");
};

// Per-server fields read or written only for the server an arrival picks live in LDS, lane-major
// ([field][server][lane], conflict-free): one ds_read/ds_write per field instead of an S-way
// register select chain.  Fields every server needs at every arrival (cnt, head_tc, the window /
// ring head positions, the SED denominators) stay in registers.
enum SrvField {
  F_TAIL = 0,  // t_complete of the last queued flow (valid if cnt > 0)
  F_RCNT,      // Algorithm R count of the server's reservoirs
  F_ASSIGNED,  // arrivals assigned this launch (assign_count_out)
  F_SCALE,     // (unused by the env-per-lane loop: service scales are VGPR constants)
  F_TAB0,      // ALIAS table of this step, active position s: odd (f32 bits)
  F_TAB1,      //   alias | server << 8
  F_NUM
};

template <int MAXS>
struct LaneState {
  static constexpr int WL = Win<MAXS>::WL;
  int32_t cnt[MAXS];      // flows in flight (n_flow_on)
  int32_t head_tc[MAXS];  // t_complete of the head flow (valid if cnt > 0)
  int32_t lh[MAXS];       // window slot of the head flow
  int32_t head[MAXS];     // ring position of the head flow
  int32_t last[MAXS];     // t_complete of the last completed flow (kLastNone if none)
  int32_t next_arr;
  float next_work;
  uint32_t u2, u3, arr_idx, episode, clock, dropped;
  uint32_t gid;
  uint32_t downm;         // bit s: server s is down (fail_prob > 0), not eligible as a full one
  uint32_t bigm;          // bit s: server s's kHcBig flag
  // TRACE: row of arrival arr_idx + 1 and its prefetched gap / work (loaded an arrival ahead so
  // the event loop never waits on the trace)
  uint32_t row;
  int32_t pf_gap;
  float pf_work;
};

struct Lds {
  int2* q;       // queue window [server][slot][lane]
  int32_t* f;    // per-server fields [field][server][lane]
  int lane;
  uint32_t* m;   // slots written this launch [server][word][lane] (DevState::chg), or nullptr
};

// Record that reservoir slot `slot` of server s was written (ds_or_b32, no return value).
template <int MAXS>
__device__ __forceinline__ void mark_slot(const Lds& l, int s, int slot) {
  atomicOr(&l.m[(s * 4 + (slot >> 5)) * 64 + l.lane], 1u << (slot & 31));
}

template <int MAXS>
__device__ __forceinline__ int32_t& fld(const Lds& l, int field, int s) {
  return l.f[(field * MAXS + s) * 64 + l.lane];
}

// LDS window slot (server s, slot i) of this lane.
template <int MAXS>
__device__ __forceinline__ int2* qslot(const Lds& l, int s, int i) {
  return l.q + ((s * Win<MAXS>::WL + i) * 64 + l.lane);
}

// The lane's scratch slot after the window rows: the target of a push that does not happen, so
// the push store needs no branch.
template <int MAXS>
__device__ __forceinline__ int2* qdummy(const Lds& l) {
  return l.q + (MAXS * Win<MAXS>::WL * 64 + l.lane);
}

constexpr int kPolicyAlias = 4;

// SED score (n_flow_on + 1) / (1e-9 + w) in double, stored as f32 (node.c:393-399); LSQ: n.
// (ALIAS keeps its table in the den fields and uses no score.)
__device__ __forceinline__ float policy_score(int policy, int32_t cnt, double den) {
  if (policy == 2 /*LSQ*/ || policy == 3 /*LSQ2*/) return (float)cnt;
  if (policy == kPolicyAlias) return 0.0f;
  return (float)((double)(cnt + 1) / den);
}

// The same score inside the event loop, with rcp = 1 / den computed once per step: (cnt + 1) / den
// correctly rounded as q0 = c·rcp, q = q0 + fma(−q0, den, c)·rcp (Markstein's corrected quotient:
// bit-identical to the division for every finite non-zero den — checked over every 7th float
// weight in [2^-10, 2^10) × c = 1..65 and 2e8 random weights, tools/markstein_check.c).  den = 0,
// ±inf or NaN make q NaN and take the division.  3 f64 ops instead of the ~12 of a division.
__device__ __forceinline__ float policy_score_r(int policy, int32_t cnt, double den, double rcp) {
  if (policy == 2 /*LSQ*/ || policy == 3 /*LSQ2*/) return (float)cnt;
  if (policy == kPolicyAlias) return 0.0f;
  const double c = (double)(cnt + 1);
  const double q0 = c * rcp;
  double q = fma(fma(-q0, den, c), rcp, q0);
  if (q != q) {  // rare: a real branch (the asm keeps the division from being speculated)
    asm volatile("");
    q = c / den;
  }
  return (float)q;
}

template <int MAXS, typename T>
__device__ __forceinline__ T sel(const T (&a)[MAXS], int i) {
  T v = a[0];
#pragma unroll
  for (int k = 1; k < MAXS; ++k) v = (k == i) ? a[k] : v;
  return v;
}

// ALIAS table of this step (node.c:442-460 over gen_alias, src/lb/shm_proxy.py:127-146): the
// servers with weight > 0 in index order (register_as_weights, shm_proxy.py:642-648) are the
// active list; gen_alias runs in float64 exactly as the reference's Python (sequential sum,
// avg = sum / (n + 1e-6), p = w / (avg + 1e-6), small / big generators in index order, a big
// reduced below 1 becomes the next small).  Stored per active position k in the lane's table
// fields: F_TAB0 = odd (f32 bits, the alias_t float), F_TAB1 = alias | server << 8.
// `tab(f, k)` is the table word f (0: odd, 1: alias | server << 8) of active position k.
// Returns the active count.
template <int MAXS, typename Tab>
__device__ int build_alias(const float (&w)[MAXS], int S, Tab tab) {
  int n = 0;
  double sum = 0.0;
#pragma unroll
  for (int s = 0; s < MAXS; ++s) {
    if (s < S && w[s] > 0.0f) {
      tab(0, n) = (int32_t)0x3f800000;  // (1, 0)
      tab(1, n) = s << 8;
      sum += (double)w[s];
      ++n;
    }
  }
  const double avg = sum / ((double)n + 1e-6);
  auto wk = [&](int k) { return (double)sel<MAXS>(w, tab(1, k) >> 8); };
  int si = 0, bi = 0, sk = -1, bk = -1;
  double sp = 0.0, bp = 0.0;
  auto next_small = [&]() {
    while (si < n && !(wk(si) < avg)) ++si;
    if (si < n) { sk = si; sp = wk(si) / (avg + 1e-6); ++si; } else { sk = -1; }
  };
  auto next_big = [&]() {
    while (bi < n && !(wk(bi) >= avg)) ++bi;
    if (bi < n) { bk = bi; bp = wk(bi) / (avg + 1e-6); ++bi; } else { bk = -1; }
  };
  next_small();
  next_big();
  while (bk >= 0 && sk >= 0) {
    tab(0, sk) = (int32_t)__float_as_uint((float)sp);
    tab(1, sk) = (tab(1, sk) & ~0xFF) | bk;
    bp = bp - (1.0 - sp);
    if (bp < 1.0) { sk = bk; sp = bp; next_big(); } else { next_small(); }
  }
  return n;
}

// ALIAS pick for an arrival with hash word u: rand_num = U * n (U = 24 bits of u, in [0, 1)),
// bucket = (int)rand_num, the alias if rand_num - bucket > odd[bucket] (node.c:449-460).
template <typename Tab>
__device__ __forceinline__ int alias_pick(Tab tab, int n, uint32_t u) {
  const float rn = (float)(u >> 8) * 5.9604644775390625e-8f * (float)n;
  int bucket = (int)rn;
  bucket = bucket > n - 1 ? n - 1 : bucket;
  const float odd = __uint_as_float((uint32_t)tab(0, bucket));
  const int k = (rn - (float)bucket) > odd ? (tab(1, bucket) & 0xFF) : bucket;
  return tab(1, k) >> 8;
}

// The per-lane kernel keeps the table in the lane's den fields.
template <int MAXS>
struct FieldAliasTab {
  const Lds& l;
  __device__ int32_t& operator()(int f, int k) const { return fld<MAXS>(l, F_TAB0 + f, k); }
};

// Arrival draw for one arrival index: gap to it, its work, its two hash words.
__device__ __forceinline__ void arrival_from_draw(const SimParams& p, const u32x4& d,
                                                  int32_t t_prev, int32_t& next_arr,
                                                  float& work, uint32_t& u2, uint32_t& u3) {
  const int32_t gap = (int32_t)(-lb_logf(u01_open0(d.x)) * p.mean_gap_us);
  next_arr = t_prev + gap;
  work = -lb_logf(u01_open0(d.y));
  u2 = d.z;
  u3 = d.w;
}

template <int MAXS>
__device__ __forceinline__ void draw_arrival(const DevState& st, const SimParams& p,
                                             LaneState<MAXS>& L, int32_t t_prev) {
  const u32x4 d = philox4x32_10(u32x4{L.arr_idx, L.gid, L.episode, kStreamArrival << 24},
                                p.key0, p.key1);
  if (p.trace) {
    const uint32_t r = trace_row(p, L.gid, L.episode, L.arr_idx);
    L.next_arr = t_prev + (int32_t)st.trace_gap[r];
    L.next_work = st.trace_work[r];
    L.u2 = d.z;
    L.u3 = d.w;
  } else {
    arrival_from_draw(p, d, t_prev, L.next_arr, L.next_work, L.u2, L.u3);
  }
}

// TRACE: position the prefetch at arrival arr_idx + 1 (kernel entry).
template <int MAXS>
__device__ __forceinline__ void trace_prefetch(const DevState& st, const SimParams& p,
                                               LaneState<MAXS>& L) {
  if (p.trace) {
    L.row = trace_row(p, L.gid, L.episode, L.arr_idx + 1u);
    L.pf_gap = (int32_t)st.trace_gap[L.row];
    L.pf_work = st.trace_work[L.row];
  }
}

// Kernel entry: per-server state from HBM; the first WL entries of every queue into LDS.
template <int MAXS>
__device__ __forceinline__ void load_servers(const DevState& st, const SimParams& p,
                                             LaneState<MAXS>& L, uint32_t b, const Lds& l) {
  constexpr int WL = LaneState<MAXS>::WL;
  L.downm = 0u;
  L.bigm = 0u;
#pragma unroll
  for (int s = 0; s < MAXS; ++s) {
    L.cnt[s] = 0;
    L.head_tc[s] = 0;
    L.lh[s] = 0;
    L.head[s] = 0;
    L.last[s] = kLastNone;
    if (s < p.S) {
      const uint32_t sb = b * (uint32_t)p.S + (uint32_t)s;
      const uint32_t hc = st.hc[sb];
      const int head = (int)(hc & kHcHead);
      L.cnt[s] = (int32_t)(hc >> 16);
      L.head[s] = head;
      L.bigm |= (hc & kHcBig) ? 1u << s : 0u;
      if (st.down != nullptr && st.down[sb] != 0u) L.downm |= 1u << s;
      L.last[s] = st.last_tc[sb];
      fld<MAXS>(l, F_RCNT, s) = (int32_t)st.res_count[sb];
      fld<MAXS>(l, F_ASSIGNED, s) = 0;
#pragma unroll
      for (int w = 0; w < 4; ++w) l.m[(s * 4 + w) * 64 + l.lane] = 0u;
      int32_t tail = 0;
      for (int i = 0; i < WL && i < L.cnt[s]; ++i) {
        int pos = head + i;
        if (pos >= p.Q) pos -= p.Q;
        *qslot<MAXS>(l, s, i) = st.ring[sb * (uint32_t)p.Q + (uint32_t)pos];
      }
      if (L.cnt[s] > 0) {
        int tp = head + L.cnt[s] - 1;
        if (tp >= p.Q) tp -= p.Q;
        tail = st.ring[sb * (uint32_t)p.Q + (uint32_t)tp].x;
        L.head_tc[s] = st.ring[sb * (uint32_t)p.Q + (uint32_t)head].x;
      }
      fld<MAXS>(l, F_TAIL, s) = tail;
    }
  }
}

// Reset: empty queues and reservoirs.
template <int MAXS>
__device__ __forceinline__ void clear_servers(const SimParams& p, LaneState<MAXS>& L,
                                              const Lds& l) {
  L.downm = 0u;  // every server is up at the episode start
  L.bigm = 0u;
#pragma unroll
  for (int s = 0; s < MAXS; ++s) {
    L.cnt[s] = 0;
    L.head_tc[s] = 0;
    L.lh[s] = 0;
    L.head[s] = 0;
    fld<MAXS>(l, F_TAIL, s) = 0;
    L.last[s] = kLastNone;
    fld<MAXS>(l, F_RCNT, s) = 0;
    fld<MAXS>(l, F_ASSIGNED, s) = 0;
    // emptied reservoirs: slot 0 marked written, so the next observe recomputes every server
    // (its cached features are the last episode's)
#pragma unroll
    for (int w = 0; w < 4; ++w) l.m[(s * 4 + w) * 64 + l.lane] = (w == 0 && s < p.S) ? 1u : 0u;
  }
}

// Algorithm R slot (reservoir.py:64-85) of the sample that makes count cres + 1, for a flow
// carried in from an earlier step: slot cres while the reservoir fills, else j = randint(0,
// cres + 1) from the 64-bit half (cres & 1) of the reservoir-stream Philox block d of index
// cres >> 1, kept if j < K (-1: not stored).
__device__ __forceinline__ int reservoir_slot(uint32_t cres, const u32x4& d) {
  const uint32_t hi = (cres & 1u) ? d.w : d.y;
  const uint32_t lo = (cres & 1u) ? d.z : d.x;
  const uint64_t j = mulhi64_by_u33(hi, lo, (uint64_t)cres + 1u);
  return cres < (uint32_t)K ? (int)cres : (j < (uint64_t)K ? (int)j : -1);
}

// The slot one sample takes in a reservoir holding c samples (-1: not kept; oracle res_slot): ALGR
// (reservoir.py:64-85) or VPP (every sample to slot rand() % 128, lbhash.h:108,179: the top 7
// bits of the draw).  A flow that arrived in this step (has_r) draws with its arrival's word r;
// otherwise the reservoir stream's block (c >> 1), half (c & 1), counter word w3.
__device__ __forceinline__ int reservoir_slot_r32(uint32_t cres, uint32_t r);
__device__ __forceinline__ int res_slot(const SimParams& p, uint32_t c, bool has_r, uint32_t r,
                                        uint32_t gid, uint32_t episode, uint32_t w3) {
  if (!p.res_vpp && c < (uint32_t)K) return (int)c;
  if (has_r) return p.res_vpp ? (int)(r >> 25) : reservoir_slot_r32(c, r);
  const u32x4 d = philox4x32_10(u32x4{c >> 1, gid, episode, w3}, p.key0, p.key1);
  if (p.res_vpp) return (int)(((c & 1u) ? d.w : d.y) >> 25);
  return reservoir_slot(c, d);
}

// Algorithm R slot of a flow that arrives and completes in the same step: the draw is its arrival's
// word r (word w of the arrival's Philox block, drawn when the arrival was), j = floor(r (cres + 1)
// / 2^32) (Lemire multiply-shift; r·cres + r is one v_mad_u64_u32 and never overflows 64 bits;
// bias <= (cres + 1) / 2^32).  No Philox block per insert.
__device__ __forceinline__ int reservoir_slot_r32(uint32_t cres, uint32_t r) {
  const uint32_t j = (uint32_t)(((uint64_t)r * cres + r) >> 32);
  return cres < (uint32_t)K ? (int)cres : (j < (uint32_t)K ? (int)j : -1);
}

// SED2 / LSQ2 candidates from the arrival's hash word u: the high and the low 16 bits, each
// mapped to [0, S) by multiply-shift (node.c:409-441's two hashes).
__device__ __forceinline__ int two_choice_h1(uint32_t u, int S) { return (int)(((u >> 16) * (uint32_t)S) >> 16); }
__device__ __forceinline__ int two_choice_h2(uint32_t u, int S) { return (int)(((u & 0xFFFFu) * (uint32_t)S) >> 16); }

__device__ __forceinline__ uint32_t count_inc(uint32_t c) { return c != 0xFFFFFFFFu ? c + 1u : c; }

// Loop constants of one step, pinned in VGPRs.  At one wave per SIMD most of the 512 VGPRs are
// free, while SGPRs are scarce (the Philox round keys alone take 20): constants left in SGPRs were
// re-loaded from the kernarg segment inside the loop (s_load + s_waitcnt lgkmcnt(0), which also
// waits for every LDS access in flight).  vpin() makes a uniform value a VGPR the compiler cannot
// rematerialise from memory.
__device__ __forceinline__ uint32_t vpin(uint32_t x) {
  uint32_t r;
  asm volatile("v_mov_b32 %0, %1" : "=v"(r) : "v"(x));
  return r;
}
__device__ __forceinline__ float vpin(float x) { return __uint_as_float(vpin(__float_as_uint(x))); }
__device__ __forceinline__ int32_t vpin(int32_t x) { return (int32_t)vpin((uint32_t)x); }

template <int MAXS>
struct EvConst {
  uint32_t rk0[10], rk1[10];  // Philox round keys
  float mean_gap, scale[MAXS];
  int32_t dt, S, Q;
  uint32_t base_ms, base_rem;
};

template <int MAXS>
__device__ __forceinline__ EvConst<MAXS> ev_const(const SimParams& p, uint32_t base_ms,
                                                   uint32_t base_rem) {
  EvConst<MAXS> c;
  uint32_t k0 = p.key0, k1 = p.key1;
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    c.rk0[r] = vpin(k0);
    c.rk1[r] = vpin(k1);
    k0 += 0x9E3779B9u;
    k1 += 0xBB67AE85u;
  }
  c.mean_gap = vpin(p.mean_gap_us);
#pragma unroll
  for (int s = 0; s < MAXS; ++s) c.scale[s] = vpin(s < p.S ? p.svc_scale[s] : 1.0f);
  c.dt = vpin(p.dt_us);
  c.S = p.S;
  c.Q = p.Q;
  c.base_ms = vpin(base_ms);
  c.base_rem = vpin(base_rem);
  return c;
}

// Philox4x32-10 with precomputed round keys (same bits as philox4x32_10).
__device__ __forceinline__ u32x4 philox_rk(u32x4 c, const uint32_t (&rk0)[10],
                                           const uint32_t (&rk1)[10]) {
  constexpr uint32_t M0 = 0xD2511F53u, M1 = 0xCD9E8D57u;
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    const uint64_t p0 = (uint64_t)M0 * c.x;
    const uint64_t p1 = (uint64_t)M1 * c.z;
    // hi ^ y ^ k as one v_bitop3_b32 (truth table 0x96 = a ^ b ^ c)
    c = u32x4{(uint32_t)__builtin_amdgcn_bitop3_b32((uint32_t)(p1 >> 32), c.y, rk0[r], 0x96),
              (uint32_t)p1,
              (uint32_t)__builtin_amdgcn_bitop3_b32((uint32_t)(p0 >> 32), c.w, rk1[r], 0x96),
              (uint32_t)p0};
  }
  return c;
}

// The event loop of sim_step (section 2, specification in the comment block below).
//  * every server's next-head LDS read is issued at the top of the iteration, before anything
//    branches, so the S reads are in flight together; the rare refill of a queue longer than the
//    window is one branch for all servers;
//  * the chosen server's tail, Algorithm R count and assignment count are register arrays
//    selected like cnt (REGF, MAXS <= 8), not dependent LDS round trips; service scales are
//    VGPR constants;
//  * FAST (wave-uniform): every SED score finite, so no NaN fallback and no "first eligible"
//    variant of the argmin.
template <int MAXS, int POLICY, bool TRACE, bool FAST>
__device__ __forceinline__ void event_loop(const DevState& st, const SimParams& p,
                                           LaneState<MAXS>& L, const Lds& l,
                                           const EvConst<MAXS>& ec, const double (&den)[MAXS],
                                           const double (&rcp)[MAXS], int n_alias,
                                           uint2* const my_res, int2* const my_ring) {
  constexpr int WL = LaneState<MAXS>::WL;
  constexpr bool REGF = MAXS <= 8;
  constexpr bool two_choice = (POLICY == 1 || POLICY == 3);
  constexpr bool alias = POLICY == kPolicyAlias;
  constexpr bool lsq = (POLICY == 2 || POLICY == 3);
  const int S = ec.S, Q = ec.Q;
  const int32_t dt = ec.dt;
  int32_t tail[MAXS], asg[MAXS];
  uint32_t rcnt[MAXS];
  // hs[s]: the head's window slot without the wrap (lh + pops so far); the slot is hs & (WL - 1)
  // and the ring position head + (hs - lh) mod Q is needed only on the rare ring paths and at the
  // end, so a pop is one add instead of the lh / head wrap-and-select pairs
  // (rbase[s] + hs[s] + k) mod Q is the ring position of queue entry k
  int32_t hs[MAXS], rbase[MAXS];
#pragma unroll
  for (int s = 0; s < MAXS; ++s) {
    hs[s] = L.lh[s];
    rbase[s] = L.head[s] - L.lh[s] + Q;  // >= 1: lh < WL <= Q
  }
  if constexpr (REGF) {
#pragma unroll
    for (int s = 0; s < MAXS; ++s) {
      tail[s] = s < S ? fld<MAXS>(l, F_TAIL, s) : 0;
      rcnt[s] = s < S ? (uint32_t)fld<MAXS>(l, F_RCNT, s) : 0u;
      asg[s] = 0;
    }
  }
  // n_flow_on_mode VPP (p.leak, the general loop only): each server's lost-FIN flows completed so
  // far (DevState::lost_on), counted at their pop and added to the queue count in the SED / LSQ
  // scores (node.c:395-437 read as_stat n_flow_on, never decremented for them: lbhash.h:193,214)
  const size_t row0 = (size_t)(my_res - st.res) / K;  // the env's first (env, server) row
  int32_t lost[MAXS];
#pragma unroll
  for (int s = 0; s < MAXS; ++s) lost[s] = 0;
  if constexpr (!FAST) {
    if (p.leak) {
#pragma unroll
      for (int s = 0; s < MAXS; ++s) lost[s] = s < S ? (int32_t)st.lost_on[row0 + (size_t)s] : 0;
    }
  }
  for (;;) {
    const bool arrival_due = L.next_arr < dt;
    const int32_t th = arrival_due ? L.next_arr : dt;  // a completion at the arrival time goes first
    int32_t nt[MAXS];
    bool due[MAXS];
    bool refill = false;
#pragma unroll
    for (int s = 0; s < MAXS; ++s) {
      nt[s] = qslot<MAXS>(l, s, (hs[s] + 1) & (WL - 1))->x;  // next head (valid if cnt > 1)
      due[s] = (s < S) & (L.cnt[s] > 0) & (L.head_tc[s] <= th);
      refill |= due[s] & (L.cnt[s] - 1 >= WL);
    }
    if constexpr (!FAST) {  // a popped lost-FIN flow stays in n_flow_on (before the refill below
      if (p.leak) {         // overwrites the head's window slot)
#pragma unroll
        for (int s = 0; s < MAXS; ++s)
          if (due[s] && lf_lost(p, ec.base_ms * 1000u + ec.base_rem +
                                       (uint32_t)qslot<MAXS>(l, s, hs[s] & (WL - 1))->y,
                                L.gid, L.episode))
            lost[s] += 1;
      }
    }
    if (refill) {  // rare: bring queue entry WL (ring) into the slot the pop frees
#pragma unroll
      for (int s = 0; s < MAXS; ++s) {
        if (due[s] && L.cnt[s] - 1 >= WL)
          *qslot<MAXS>(l, s, hs[s] & (WL - 1)) =
              my_ring[(uint32_t)s * (uint32_t)Q + (uint32_t)(rbase[s] + hs[s] + WL) % (uint32_t)Q];
      }
      __builtin_amdgcn_s_waitcnt(kWaitVmcnt0);  // drain in the rare branch, not at the back-edge
    }
    bool more = false;
#pragma unroll
    for (int s = 0; s < MAXS; ++s) {  // pop each server's head if it completed by th
      L.last[s] = due[s] ? L.head_tc[s] : L.last[s];
      L.cnt[s] -= due[s] ? 1 : 0;
      hs[s] += due[s] ? 1 : 0;
      L.head_tc[s] = due[s] ? nt[s] : L.head_tc[s];
      more |= due[s] & (L.cnt[s] > 0) & (nt[s] <= th);
    }
    if (!arrival_due && !more) break;
    const bool arr = arrival_due & !more;

    // ---- the arrival: choose a server (node.c:388-441); full servers are not eligible
    const int32_t ta = L.next_arr;
    float score[MAXS];
    if constexpr (!alias) {
      bool bad = false;
#pragma unroll
      for (int s = 0; s < MAXS; ++s) {
        if constexpr (lsq) {
          score[s] = (float)(L.cnt[s] + lost[s]);
        } else {  // (cnt + 1) / den correctly rounded by Markstein's corrected quotient
          const double c = (double)(L.cnt[s] + lost[s] + 1);
          const double q0 = c * rcp[s];
          const double q = fma(fma(-q0, den[s], c), rcp[s], q0);
          if constexpr (!FAST) bad |= q != q;
          score[s] = (float)q;
        }
      }
      if (!FAST && !lsq && bad) {  // den 0 / inf / NaN: the division
#pragma unroll
        for (int s = 0; s < MAXS; ++s) {
          const float q = score[s];
          if (q != q) score[s] = (float)((double)(L.cnt[s] + lost[s] + 1) / den[s]);
        }
      }
    }
    int chosen = -1;
    if constexpr (alias) {  // full server: the flow is dropped (ALIAS has no eligibility test)
      if (n_alias > 0) {
        const int a = alias_pick(FieldAliasTab<MAXS>{l}, n_alias, L.u2);
        chosen = (sel<MAXS>(L.cnt, a) < Q && !((L.downm >> a) & 1u)) ? a : -1;
      }
    } else if constexpr (two_choice) {  // SED2 / LSQ2: keep the second candidate if strictly better
      const int h1 = two_choice_h1(L.u2, S);
      const int h2 = two_choice_h2(L.u2, S);
      float s1 = 0.f, s2 = 0.f;
      bool ok1 = false, ok2 = false;
#pragma unroll
      for (int s = 0; s < MAXS; ++s) {
        s1 = (s == h1) ? score[s] : s1;
        ok1 = (s == h1) ? (L.cnt[s] < Q && !((L.downm >> s) & 1u)) : ok1;
        s2 = (s == h2) ? score[s] : s2;
        ok2 = (s == h2) ? (L.cnt[s] < Q && !((L.downm >> s) & 1u)) : ok2;
      }
      chosen = (ok1 && ok2) ? ((s2 < s1) ? h2 : h1) : (ok1 ? h1 : (ok2 ? h2 : -1));
    } else {  // SED / LSQ: start at the hashed server, replace on strictly lower score
      const int h = (int)__umulhi(L.u2, (uint32_t)S);  // (u * S) >> 32
      float best = __uint_as_float(0x7f800000u);  // +inf: any finite score replaces it
#pragma unroll
      for (int s = 0; s < MAXS; ++s) {
        const bool m = (s == h) & (L.cnt[s] < Q) & !((L.downm >> s) & 1u);
        chosen = m ? s : chosen;
        best = m ? score[s] : best;
      }
      if (FAST || lsq) {  // every score finite: "replace on strictly lower" from +inf is exact
#pragma unroll
        for (int s = 0; s < MAXS; ++s) {
          const bool m = (s < S) & (L.cnt[s] < Q) & !((L.downm >> s) & 1u) & (score[s] < best);
          chosen = m ? s : chosen;
          best = m ? score[s] : best;
        }
      } else {  // NaN / inf scores: the first eligible server is taken whatever its score
#pragma unroll
        for (int s = 0; s < MAXS; ++s) {
          const bool m = (s < S) & (L.cnt[s] < Q) & !((L.downm >> s) & 1u) &
                         ((chosen < 0) | (score[s] < best));
          chosen = m ? s : chosen;
          best = m ? score[s] : best;
        }
      }
    }
    const bool push = arr && chosen >= 0;
    L.dropped += (arr && chosen < 0) ? 1u : 0u;

    // ---- the chosen server: FIFO service starts when its last queued flow ends
    const int cs = push ? chosen : 0;
    int32_t c_cnt = 0, c_hs = 0, c_rb = 0, c_tail = 0;
    uint32_t cres = 0u;
    float c_scale = 1.0f;
#pragma unroll
    for (int s = 0; s < MAXS; ++s) {
      const bool m = s == cs;
      c_cnt = m ? L.cnt[s] : c_cnt;
      c_hs = m ? hs[s] : c_hs;
      c_rb = m ? rbase[s] : c_rb;
      c_scale = m ? ec.scale[s] : c_scale;
      if constexpr (REGF) {
        c_tail = m ? tail[s] : c_tail;
        cres = m ? rcnt[s] : cres;
      }
    }
    if constexpr (!REGF) {
      c_tail = fld<MAXS>(l, F_TAIL, cs);
      cres = (uint32_t)fld<MAXS>(l, F_RCNT, cs);
    }
    const int32_t start_a = c_cnt > 0 ? (c_tail > ta ? c_tail : ta) : ta;
    int32_t svc = (int32_t)(L.next_work * c_scale);
    svc = svc < 1 ? 1 : svc;
    const int32_t tc_a = start_a + svc;
    // completes in this step: its sample now (duration: age tc - ta, or svc = tc - start)
    const bool ins = push && tc_a <= dt;

    // ---- one Philox block, the next arrival's; the pushed flow's Algorithm R draw is this
    //      arrival's word r (L.u3)
    const u32x4 d = philox_rk(u32x4{L.arr_idx + 1u, L.gid, L.episode, kStreamArrival << 24},
                              ec.rk0, ec.rk1);
    const int slot = reservoir_slot_r32(cres, L.u3);
    if (ins && slot >= 0) {
      const uint32_t fct = lost_fct(p, (uint32_t)(tc_a - ta),
                                    ec.base_ms * 1000u + ec.base_rem + (uint32_t)ta, L.gid, L.episode);
      const uint32_t ri = (uint32_t)cs * (uint32_t)K + (uint32_t)slot;
      my_res[ri] = make_uint2(fct, ec.base_ms + (ec.base_rem + (uint32_t)tc_a) / 1000u);
      if constexpr (!FAST) {  // the duration plane (sim_step sends its handles to this loop)
        if (st.res_dur != nullptr)
          st.res_dur[(size_t)(my_res - st.res) + ri] = dur_sample(p, tc_a, ta, start_a);
      }
      mark_slot<MAXS>(l, cs, slot);
    }
    // queue index < WL: the LDS window (a push that does not happen writes the lane's scratch
    // slot); beyond it: the HBM ring (overflow, rare)
    *((push & (c_cnt < WL)) ? qslot<MAXS>(l, cs, (c_hs + c_cnt) & (WL - 1)) : qdummy<MAXS>(l)) =
        make_int2(tc_a, ta);
    if (push && c_cnt >= WL) {
      const uint32_t pos = (uint32_t)(c_rb + c_hs + c_cnt) % (uint32_t)Q;
      my_ring[(uint32_t)cs * (uint32_t)Q + pos] = make_int2(tc_a, ta);
      // keeps the compiler from sinking the store into a flat (generic pointer) store shared with
      // the window store, which counts in lgkmcnt too: every LDS wait would then wait on it
      asm volatile("");
    }
    if constexpr (REGF) {
#pragma unroll
      for (int s = 0; s < MAXS; ++s) {
        const bool m = push & (s == cs);
        tail[s] = m ? tc_a : tail[s];
        asg[s] += m ? 1 : 0;
        rcnt[s] = (ins & (s == cs)) ? count_inc(cres) : rcnt[s];
      }
    } else {
      fld<MAXS>(l, F_TAIL, cs) = push ? tc_a : c_tail;
      atomicAdd(&fld<MAXS>(l, F_ASSIGNED, cs), push ? 1 : 0);  // ds_add_u32: no read-back
      fld<MAXS>(l, F_RCNT, cs) = (int32_t)(ins ? count_inc(cres) : cres);
    }
#pragma unroll
    for (int s = 0; s < MAXS; ++s) {
      const bool m = push & (s == cs);
      L.head_tc[s] = (m && c_cnt == 0) ? tc_a : L.head_tc[s];
      L.cnt[s] += m ? 1 : 0;
    }

    // ---- next arrival (draw d belongs to arrival index arr_idx + 1)
    int32_t na;
    float nw;
    uint32_t nu2, nu3;
    if constexpr (TRACE) {  // the prefetched row; the next prefetch is issued one arrival ahead
      na = ta + L.pf_gap;
      nw = L.pf_work;
      nu2 = d.z;
      nu3 = d.w;
      if (arr) {
        L.row = (L.row + 1u == p.trace_rows) ? 0u : L.row + 1u;
        L.pf_gap = (int32_t)st.trace_gap[L.row];
        L.pf_work = st.trace_work[L.row];
      }
    } else {
      na = ta + (int32_t)(-lb_logf(u01_open0(d.x)) * ec.mean_gap);
      nw = -lb_logf(u01_open0(d.y));
      nu2 = d.z;
      nu3 = d.w;
    }
    L.next_arr = arr ? na : L.next_arr;
    L.next_work = arr ? nw : L.next_work;
    L.u2 = arr ? nu2 : L.u2;
    L.u3 = arr ? nu3 : L.u3;
    L.arr_idx += arr ? 1u : 0u;
  }
#pragma unroll
  for (int s = 0; s < MAXS; ++s) {
    L.head[s] = (int32_t)((uint32_t)(rbase[s] + hs[s]) % (uint32_t)Q);
    L.lh[s] = hs[s] & (WL - 1);
  }
  if constexpr (!FAST) {
    if (p.leak) {
#pragma unroll
      for (int s = 0; s < MAXS; ++s)
        if (s < S) st.lost_on[row0 + (size_t)s] = (uint32_t)lost[s];
    }
  }
  if constexpr (REGF) {
#pragma unroll
    for (int s = 0; s < MAXS; ++s) {
      if (s < S) {
        fld<MAXS>(l, F_TAIL, s) = tail[s];
        fld<MAXS>(l, F_RCNT, s) = (int32_t)rcnt[s];
        fld<MAXS>(l, F_ASSIGNED, s) += asg[s];
      }
    }
  }
}

// One simulated step of dt_us with server weights w[] (env.py:230-259 with real dynamics).
//
// Arrival-driven, as the oracle: a FIFO server fixes a flow's completion time when the flow is
// queued (tc = max(ta, tail) + svc), so its completion sample {fct = tc - ta, duration (dur_sample),
// ts(tc)} is known at the push, and a server's reservoir sees its samples in FIFO order whatever
// the interleaving with other servers.  So:
//   1. flows carried in from earlier steps that complete in this one are inserted first, server
//      by server in FIFO order (their predecessor's completion is last[s]);
//   2. the loop runs one iteration per arrival: first every server pops its flows completed at or
//      before the arrival (one pop per server per iteration, in parallel over the unrolled
//      servers; a lane with a second due pop spends one more iteration before its arrival), then
//      the arrival is assigned on the counts (node.c:388-441) and pushed, and its sample inserted
//      now if it completes in this step (Algorithm R draw of the server's count);
//   3. after the last arrival, the pops up to dt; then the rebase.
// The body is straight-line and predicated, so the 64 lanes (64 envs) stay converged; an iteration
// costs one arrival's work (one Philox block, the next arrival's draw, whose word w is also that
// flow's Algorithm R draw), and a lane iterates ~arrivals times instead of arrivals + completions.  Every
// reservoir gets the same insert sequence as the oracle's event order, so the state is bit-identical.
template <int MAXS, int POLICY, bool TRACE>
__device__ __forceinline__ void sim_step(const DevState& st, const SimParams& p,
                                         LaneState<MAXS>& L, uint32_t b, const float (&w)[MAXS],
                                         const Lds& l) {
  constexpr int WL = LaneState<MAXS>::WL;
  const int S = p.S, Q = p.Q;
  const int32_t dt = p.dt_us;
  // sample timestamps: ts_ms = (clock * dt + tc) / 1000 = base_ms + (base_rem + tc) / 1000
  const uint64_t base_us = (uint64_t)L.clock * (uint64_t)dt;
  const uint32_t base_ms = (uint32_t)(base_us / 1000u);
  const uint32_t base_rem = (uint32_t)(base_us - (uint64_t)base_ms * 1000u);
  constexpr bool alias = POLICY == kPolicyAlias;
  constexpr bool lsq = (POLICY == 2 || POLICY == 3);
  const uint32_t b0 = b * (uint32_t)S;
  // this env's reservoirs and rings as per-lane (VGPR) pointers: no kernarg reload in the loop
  uint2* const my_res = st.res + (size_t)b0 * K;
  int2* const my_ring = st.ring + (size_t)b0 * (size_t)Q;
  int n_alias = 0;
  double den[MAXS], rcp[MAXS];
  // SED scores (cnt + 1) / den stay finite (cnt + 1 <= 65) for every finite |den| >= 1e-30
  bool finite_scores = true;
#pragma unroll
  for (int s = 0; s < MAXS; ++s) {
    den[s] = 1.0;
    rcp[s] = 1.0;
  }
  if constexpr (alias) {
    n_alias = build_alias<MAXS>(w, S, FieldAliasTab<MAXS>{l});
  } else if constexpr (!lsq) {
#pragma unroll
    for (int s = 0; s < MAXS; ++s) {
      if (s < S) {
        den[s] = (double)w[s] + 1e-9;
        rcp[s] = 1.0 / den[s];
        finite_scores &= fabs(den[s]) >= 1e-30 && fabs(den[s]) <= 1e300;  // false for NaN
      }
    }
  }

  // ---- 0. server failure / recovery (fail_prob > 0, a uniform branch): one Philox draw per
  //      server, stream 5, counter (clock, gid, episode); a failing server loses its queue (the
  //      flows count as dropped) and its reservoirs; a down server takes no flows
  if (p.fail_thr != 0u) {
    for (int s = 0; s < S; ++s) {
      const u32x4 d = philox4x32_10(
          u32x4{L.clock, L.gid, L.episode, (kStreamFailure << 24) | (uint32_t)s}, p.key0, p.key1);
      const uint32_t u = d.x >> 8;
      const bool was_down = (L.downm >> s) & 1u;
      if (was_down) {
        if (u < p.rec_thr) L.downm &= ~(1u << s);
      } else if (u < p.fail_thr) {
        L.downm |= 1u << s;
        L.bigm &= ~(1u << s);
#pragma unroll
        for (int k = 0; k < MAXS; ++k) {  // register arrays: constant indices only
          if (k == s) {
            L.dropped += (uint32_t)L.cnt[k];
            L.cnt[k] = 0;
            L.last[k] = kLastNone;
          }
        }
        fld<MAXS>(l, F_RCNT, s) = 0;
        mark_slot<MAXS>(l, s, 0);  // emptied: the next observe recomputes the (zero) features
        if (p.leak) st.lost_on[b0 + (uint32_t)s] = 0u;
      }
    }
  }

  // ---- 1. carried-in flows completing in this step: samples in FIFO order per server
#pragma unroll
  for (int s = 0; s < MAXS; ++s) {
    if (s < S && L.cnt[s] > 0 && L.head_tc[s] <= dt) {
      int32_t prev = L.last[s];
      uint32_t rc = (uint32_t)fld<MAXS>(l, F_RCNT, s);
      const int c = L.cnt[s];
      int32_t etc = L.head_tc[s];
      int32_t eta = qslot<MAXS>(l, s, L.lh[s])->y;
      int i = 0;
      for (;;) {
        const u32x4 d = philox4x32_10(
            u32x4{rc >> 1, L.gid, L.episode, (kStreamReservoir << 24) | (uint32_t)s}, p.key0, p.key1);
        const int slot = reservoir_slot(rc, d);
        if (slot >= 0) {
          const uint32_t fct =
              lost_fct(p, (uint32_t)(etc - eta), (uint32_t)base_us + (uint32_t)eta, L.gid, L.episode);
          const uint32_t dur = dur_sample(p, etc, eta, eta > prev ? eta : prev);
          L.bigm |= big_record(fct, dur) ? 1u << s : 0u;
          store_record(st, (size_t)(b0 + (uint32_t)s) * K + (size_t)slot, fct, dur,
                       base_ms + (base_rem + (uint32_t)etc) / 1000u);
          mark_slot<MAXS>(l, s, slot);
        }
        prev = etc;
        rc = count_inc(rc);
        if (++i >= c) break;
        int2 e;
        if (i < WL) {
          int li = L.lh[s] + i;
          li = li >= WL ? li - WL : li;
          e = *qslot<MAXS>(l, s, li);
        } else {  // rare: beyond the window
          int pos = L.head[s] + i;
          pos = pos >= Q ? pos - Q : pos;
          e = my_ring[(uint32_t)s * (uint32_t)Q + (uint32_t)pos];
        }
        etc = e.x;
        eta = e.y;
        if (etc > dt) break;
      }
      fld<MAXS>(l, F_RCNT, s) = (int32_t)rc;
    }
  }

  // ---- 2. one arrival per iteration (3. the final pops up to dt in the last iterations).  The
  //      SED/SED2 scores can only be NaN when some den is 0 / inf / NaN: a wave whose envs all
  //      have finite scores runs the loop without the NaN fallbacks (a wave-uniform choice).
  const EvConst<MAXS> ec = ev_const<MAXS>(p, base_ms, base_rem);
  if ((lsq || alias || __all(finite_scores)) && !p.leak && st.res_dur == nullptr)
    event_loop<MAXS, POLICY, TRACE, true>(st, p, L, l, ec, den, rcp, n_alias, my_res, my_ring);
  else
    event_loop<MAXS, POLICY, TRACE, false>(st, p, L, l, ec, den, rcp, n_alias, my_res, my_ring);

  // ---- rebase relative times to the next step's start: the LDS window in place, the HBM ring
  //      entries beyond it read-modify-written (queues longer than WL only)
  L.next_arr -= dt;
#pragma unroll
  for (int s = 0; s < MAXS; ++s) {
    if (s < S) {
      const int lh = L.lh[s];
      for (int i = 0; i < WL && i < L.cnt[s]; ++i) {
        int li = lh + i;
        li = li >= WL ? li - WL : li;
        int2* e = qslot<MAXS>(l, s, li);
        e->x -= dt;
        e->y -= dt;
      }
      const uint32_t sbase = b0 + (uint32_t)s;
      int pos = L.head[s] + WL;
      if (pos >= Q) pos -= Q;
      for (int i = WL; i < L.cnt[s]; ++i) {
        int2 e = st.ring[sbase * (uint32_t)Q + (uint32_t)pos];
        e.x -= dt;
        e.y -= dt;
        st.ring[sbase * (uint32_t)Q + (uint32_t)pos] = e;
        pos = (pos + 1 == Q) ? 0 : pos + 1;
      }
      L.head_tc[s] -= dt;
      fld<MAXS>(l, F_TAIL, s) -= dt;
      L.last[s] = (L.last[s] < kLastNone + dt) ? kLastNone : L.last[s] - dt;
    }
  }
  L.clock += 1u;
}

// Kernel exit: the LDS window back to the ring so HBM holds every in-flight flow, and the
// per-server state words.
template <int MAXS>
__device__ __forceinline__ void store_servers(const DevState& st, const SimParams& p,
                                              const LaneState<MAXS>& L, uint32_t b,
                                              const Lds& l, int32_t* assign_out) {
  constexpr int WL = LaneState<MAXS>::WL;
#pragma unroll
  for (int s = 0; s < MAXS; ++s) {
    if (s < p.S) {
      const uint32_t sb = b * (uint32_t)p.S + (uint32_t)s;
      const int head = L.head[s], lh = L.lh[s];
      for (int i = 0; i < WL && i < L.cnt[s]; ++i) {
        int pos = head + i;
        if (pos >= p.Q) pos -= p.Q;
        int li = lh + i;
        li = li >= WL ? li - WL : li;
        st.ring[sb * (uint32_t)p.Q + (uint32_t)pos] = *qslot<MAXS>(l, s, li);
      }
      bool big = (L.bigm >> s) & 1u;
      if (p.big_in_step) {  // the in-step records this launch wrote (big_written)
        const uint32_t cw[4] = {l.m[(s * 4 + 0) * 64 + l.lane], l.m[(s * 4 + 1) * 64 + l.lane],
                                l.m[(s * 4 + 2) * 64 + l.lane], l.m[(s * 4 + 3) * 64 + l.lane]};
        __builtin_amdgcn_s_waitcnt(0);  // the wave's stores acknowledged by L2 (vmcnt 0)
        __asm__ volatile("" ::: "memory");
        big |= big_written(st, sb, cw, (uint32_t)fld<MAXS>(l, F_RCNT, s));
      }
      st.hc[sb] = (uint32_t)head | (big ? kHcBig : 0u) | ((uint32_t)L.cnt[s] << 16);
      st.last_tc[sb] = L.last[s];
      st.res_count[sb] = (uint32_t)fld<MAXS>(l, F_RCNT, s);
      if (st.down != nullptr) st.down[sb] = (L.downm >> s) & 1u;
      if (assign_out != nullptr) assign_out[sb] = fld<MAXS>(l, F_ASSIGNED, s);
      *reinterpret_cast<uint4*>(st.chg + (size_t)sb * 4) =
          make_uint4(l.m[(s * 4 + 0) * 64 + l.lane], l.m[(s * 4 + 1) * 64 + l.lane],
                     l.m[(s * 4 + 2) * 64 + l.lane], l.m[(s * 4 + 3) * 64 + l.lane]);
    }
  }
}

__device__ __forceinline__ float action_weight(const SimParams& p, const void* action, int dtype,
                                               size_t idx) {
  if (p.action_type == 0) {  // discrete: discrete_weights[int(a)] (env.py:344-346)
    int64_t a = (dtype == 1) ? ((const int64_t*)action)[idx]
                             : (int64_t)((const int32_t*)action)[idx];
    if (a < 0) a += p.num_discrete;  // python negative indexing
    if (a < 0) a = 0;
    if (a >= p.num_discrete) a = p.num_discrete - 1;
    return p.dw[a];
  }
  // continuous: np.clip(f32(a), min_w, max_w) (env.py:349-351); NaN passes through
  const float a = ((const float*)action)[idx];
  return a < p.min_w ? p.min_w : (a > p.max_w ? p.max_w : a);
}

// action_weight with the discrete table read from kernel arguments by index-compare selects (no
// per-lane load from the argument segment behind the action's own load: one HBM round trip)
__device__ __forceinline__ float action_weight_sel(const SimParams& p, const void* action,
                                                   int dtype, size_t idx) {
  if (p.action_type == 0) {
    int64_t a = (dtype == 1) ? ((const int64_t*)action)[idx]
                             : (int64_t)((const int32_t*)action)[idx];
    if (a < 0) a += p.num_discrete;  // python negative indexing
    if (a < 0) a = 0;
    if (a >= p.num_discrete) a = p.num_discrete - 1;
    float w = p.dw[0];
#pragma unroll
    for (int k = 1; k < 8; ++k) w = a == k ? p.dw[k] : w;
    return w;
  }
  const float a = ((const float*)action)[idx];
  return a < p.min_w ? p.min_w : (a > p.max_w ? p.max_w : a);
}

// Waves per workgroup of dynamics_kernel.  Every wave runs a long, issue-bound event loop, so a
// SIMD holding two waves finishes twice as late.  With one-wave workgroups the dispatcher stacked
// some CUs (up to 6 fit by LDS) while others had room: at 65536 x 4 (1024 waves on 1024 SIMDs) the
// kernel lasted 1.42x the mean wave lifetime (rocprofv3 SQ_WAVE_CYCLES vs duration), and capping
// the CUs at 4 workgroups cut it 0.308 -> 0.266 ms.  Here one workgroup is 4 waves whose LDS
// (> half a CU's 160 KiB) admits one workgroup per CU: its waves land on the CU's 4 SIMDs.
// MAXS = 16 (44 KiB per wave) takes 2 waves per workgroup.
template <int MAXS>
constexpr int kDynWaves = MAXS <= 8 ? 4 : 2;

// MODE is a template parameter so step and reset launches are separate kernels in profiles.
// POLICY and TRACE (arrival source) are template parameters: each combination gets its own
// straight-line event loop.
template <int MAXS, int MODE, int POLICY, bool TRACE>
__global__ void __launch_bounds__(64 * kDynWaves<MAXS>)
    dynamics_kernel(DevState st, SimParams p, const void* action, int action_dtype,
                    int32_t* assign_out, const uint8_t* reset_mask) {
  constexpr int mode = MODE;
  const uint32_t b = blockIdx.x * (64u * kDynWaves<MAXS>) + threadIdx.x;
  const int wv = (int)(threadIdx.x >> 6);
  __shared__ int2 qwin[kDynWaves<MAXS>][(MAXS * Win<MAXS>::WL + 1) * 64];  // + scratch slots
  __shared__ int32_t fields[kDynWaves<MAXS>][F_NUM * MAXS * 64];
  __shared__ uint32_t chgw[kDynWaves<MAXS>][MAXS * 4 * 64];
  const Lds l{qwin[wv], fields[wv], (int)(threadIdx.x & 63u), chgw[wv]};
  if (b >= (uint32_t)p.B) return;
  const int S = p.S;
  LaneState<MAXS> L;
  L.gid = p.env_id_offset + b;

  if (mode == kModeReset && reset_mask != nullptr && reset_mask[b] == 0) return;
  float w[MAXS];
  auto reset_in = [&]() {  // a new episode (env.py:186-213): its first arrival, empty servers
    L.episode = st.episode[b] + 1u;
    L.clock = 0u;
    L.dropped = 0u;
    L.arr_idx = 0u;
    draw_arrival<MAXS>(st, p, L, 0);
    trace_prefetch<MAXS>(st, p, L);
    clear_servers<MAXS>(p, L, l);
    if (p.leak)  // a new episode: no lost flows yet (n_flow_on_mode VPP)
      for (int s = 0; s < S; ++s) st.lost_on[b * (uint32_t)S + (uint32_t)s] = 0u;
#pragma unroll
    for (int s = 0; s < MAXS; ++s) w[s] = 1.0f;
  };
  auto load_in = [&]() {  // the env and its servers from HBM, the step's weights
    L.episode = st.episode[b];
    L.clock = st.clock[b];
    L.dropped = st.dropped[b];
    L.arr_idx = st.arr_idx[b];
    L.next_arr = st.next_arr[b];
    L.next_work = st.next_work[b];
    L.u2 = st.next_u2[b];
    L.u3 = st.next_u3[b];
    trace_prefetch<MAXS>(st, p, L);
    load_servers<MAXS>(st, p, L, b, l);
#pragma unroll
    for (int s = 0; s < MAXS; ++s)
      w[s] = (s < S) ? action_weight(p, action, action_dtype, (size_t)b * S + (size_t)s) : 1.0f;
  };
  auto reset_out = [&](int32_t ep_step) {
    st.ep_step[b] = ep_step;
    st.ep_return[b] = 0.0;
#pragma unroll
    for (int s = 0; s < MAXS; ++s) fld<MAXS>(l, F_ASSIGNED, s) = 0;  // not the warm-up's
  };
  if constexpr (mode == kModeStep) {
    load_in();
    sim_step<MAXS, POLICY, TRACE>(st, p, L, b, w, l);
  } else if constexpr (mode == kModeReset) {
    reset_in();
    for (int k = 0; k < p.warmup_steps; ++k) sim_step<MAXS, POLICY, TRACE>(st, p, L, b, w, l);
    reset_out(0);
  } else {  // kModeStepNR: an env done last step resets in place of stepping (ep_step = -1)
    if (st.ep_step[b] >= p.max_steps) {
      reset_in();
      for (int k = 0; k < p.warmup_steps; ++k) sim_step<MAXS, POLICY, TRACE>(st, p, L, b, w, l);
      reset_out(-1);
    } else {
      load_in();
      sim_step<MAXS, POLICY, TRACE>(st, p, L, b, w, l);
    }
  }
  store_servers<MAXS>(st, p, L, b, l, mode == kModeReset ? nullptr : assign_out);
  st.episode[b] = L.episode;
  st.clock[b] = L.clock;
  st.dropped[b] = L.dropped;
  st.arr_idx[b] = L.arr_idx;
  st.next_arr[b] = L.next_arr;
  st.next_work[b] = L.next_work;
  st.next_u2[b] = L.u2;
  st.next_u3[b] = L.u3;
}

// ================================================================ wave-level helpers (wave64)

__device__ __forceinline__ uint32_t shfl_xor_u32(uint32_t v, int m) {
  return (uint32_t)__shfl_xor((int)v, m, 64);
}
__device__ __forceinline__ uint32_t shfl_up_u32(uint32_t v, int d) {
  return (uint32_t)__shfl_up((int)v, (unsigned)d, 64);
}
__device__ __forceinline__ uint32_t shfl_u32(uint32_t v, int src) {
  return (uint32_t)__shfl((int)v, src, 64);
}
__device__ __forceinline__ uint32_t readlane_u32(uint32_t v, int lane) {
  return (uint32_t)__builtin_amdgcn_readlane((int)v, lane);
}

// Lane exchanges inside a 16-lane DPP row, VALU only (no LDS crossbar):
//   xor 1 / xor 2: quad_perm [1,0,3,2] / [2,3,0,1];  xor 8: row_ror:8;
//   xor 4: row_shl:4 (lane i reads i+4) for lanes with bit 2 clear, row_shr:4 (reads i-4) else.
template <int CTRL>
__device__ __forceinline__ uint32_t dpp_u32(uint32_t v) {
  return (uint32_t)__builtin_amdgcn_update_dpp((int)v, (int)v, CTRL, 0xF, 0xF, false);
}
template <int M>
__device__ __forceinline__ uint32_t xor_lane_u32(uint32_t v, int lane) {
  if constexpr (M == 1) return dpp_u32<0xB1>(v);
  else if constexpr (M == 2) return dpp_u32<0x4E>(v);
  else if constexpr (M == 4) {
    const uint32_t up = dpp_u32<0x104>(v), dn = dpp_u32<0x114>(v);
    return (lane & 4) ? dn : up;
  } else if constexpr (M == 3) return dpp_u32<0x1B>(v);   // quad_perm [3,2,1,0]
  else if constexpr (M == 7) return dpp_u32<0x141>(v);     // row_half_mirror
  else if constexpr (M == 8) return dpp_u32<0x128>(v);
  else return shfl_xor_u32(v, M);
}
// The same exchanges for code where every lane of the row is active (sort networks, the full-
// reservoir observe path): mov_dpp with bound_ctrl and full masks has no tied "old" operand, so
// the DPP move writes a fresh register instead of a copy + in-place move (one VALU op, not two).
template <int CTRL>
__device__ __forceinline__ uint32_t dppz_u32(uint32_t v) {
  return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, CTRL, 0xF, 0xF, true);
}
template <int M>
__device__ __forceinline__ uint32_t xor_lane_z(uint32_t v, int lane) {
  if constexpr (M == 1) return dppz_u32<0xB1>(v);
  else if constexpr (M == 2) return dppz_u32<0x4E>(v);
  else if constexpr (M == 4) {  // lanes whose row_shl/row_shr source is out of the row select the other
    const uint32_t up = dppz_u32<0x104>(v), dn = dppz_u32<0x114>(v);
    return (lane & 4) ? dn : up;
  } else if constexpr (M == 3) return dppz_u32<0x1B>(v);
  else if constexpr (M == 7) return dppz_u32<0x141>(v);
  else if constexpr (M == 8) return dppz_u32<0x128>(v);
  else return shfl_xor_u32(v, M);
}
template <int M>
__device__ __forceinline__ float xor_f32_z(float v, int lane) {
  return __uint_as_float(xor_lane_z<M>(__float_as_uint(v), lane));
}
template <int M>
__device__ __forceinline__ double xor_f64_z(double v, int lane) {
  const uint32_t lo = xor_lane_z<M>((uint32_t)__double2loint(v), lane);
  const uint32_t hi = xor_lane_z<M>((uint32_t)__double2hiint(v), lane);
  return __hiloint2double((int)hi, (int)lo);
}
template <int M>
__device__ __forceinline__ float xor_lane_f32(float v, int lane) {
  return __uint_as_float(xor_lane_u32<M>(__float_as_uint(v), lane));
}
template <int M>
__device__ __forceinline__ double xor_lane_f64(double v, int lane) {
  const uint32_t lo = xor_lane_u32<M>((uint32_t)__double2loint(v), lane);
  const uint32_t hi = xor_lane_u32<M>((uint32_t)__double2hiint(v), lane);
  return __hiloint2double((int)hi, (int)lo);
}
__device__ __forceinline__ float xor_lane(float v, int lane, int m) {
  return m == 1 ? xor_lane_f32<1>(v, lane) : m == 2 ? xor_lane_f32<2>(v, lane) : xor_lane_f32<4>(v, lane);
}
__device__ __forceinline__ double xor_lane(double v, int lane, int m) {
  return m == 1 ? xor_lane_f64<1>(v, lane) : m == 2 ? xor_lane_f64<2>(v, lane) : xor_lane_f64<4>(v, lane);
}

__device__ __forceinline__ uint32_t wave_max_u32(uint32_t v, int lane) {
  uint32_t o;
  o = xor_lane_u32<1>(v, lane); v = o > v ? o : v;
  o = xor_lane_u32<2>(v, lane); v = o > v ? o : v;
  o = xor_lane_u32<4>(v, lane); v = o > v ? o : v;
  o = xor_lane_u32<8>(v, lane); v = o > v ? o : v;
  o = shfl_xor_u32(v, 16); v = o > v ? o : v;
  o = shfl_xor_u32(v, 32); v = o > v ? o : v;
  return v;
}

// numpy pairwise summation (numpy/_core/src/umath/loops_utils.h.src, n <= 128) by a group of 8
// lanes (j = lane & 7): n < 8 -> sequential sum from 0; else 8 strided accumulators r[j] (same
// per-accumulator order as numpy's unrolled loop), combined ((r0+r1)+(r2+r3))+((r4+r5)+(r6+r7))
// by three xor-shuffles (IEEE addition is commutative, so every lane of the group gets the same
// bits), then the n % 8 tail in order.  `term(i)` returns element i.
template <typename T, typename F>
__device__ __forceinline__ T pairwise8(int n, int j, F term) {
  if (n < 8) {
    T r = (T)0;
    for (int i = 0; i < n; ++i) r += term(i);
    return r;
  }
  const int m8 = n - (n % 8);
  T acc = term(j);
  for (int i = 8 + j; i < m8; i += 8) acc += term(i);
  const int lane = j;  // only bit 2 of the lane index is consulted (lane & 4 == j & 4)
  T t = acc + xor_lane(acc, lane, 1);
  t = t + xor_lane(t, lane, 2);
  t = t + xor_lane(t, lane, 4);
  for (int i = m8; i < n; ++i) t += term(i);
  return t;
}

// Two pairwise sums over the same index walk (each in numpy's order on its own): `term(i, b)`
// returns element i of the first and stores element i of the second in b.
template <typename T, typename F>
__device__ __forceinline__ T pairwise8x2(int n, int j, T& second, F term) {
  if (n < 8) {
    T r = (T)0, q = (T)0;
    for (int i = 0; i < n; ++i) {
      T bi;
      r += term(i, bi);
      q += bi;
    }
    second = q;
    return r;
  }
  const int m8 = n - (n % 8);
  T bacc;
  T acc = term(j, bacc);
  for (int i = 8 + j; i < m8; i += 8) {
    T bi;
    acc += term(i, bi);
    bacc += bi;
  }
  const int lane = j;
  T t = acc + xor_lane(acc, lane, 1), u = bacc + xor_lane(bacc, lane, 1);
  t = t + xor_lane(t, lane, 2);
  u = u + xor_lane(u, lane, 2);
  t = t + xor_lane(t, lane, 4);
  u = u + xor_lane(u, lane, 4);
  for (int i = m8; i < n; ++i) {
    T bi;
    t += term(i, bi);
    u += bi;
  }
  second = u;
  return t;
}

// ================================================================ features of one env

// LDS image of one env's reservoirs during observe (one wave per env, 64-thread blocks).
// Rows are padded to KP = 136 dwords: row r starts at bank 8r (mod 32), so the 8 lanes x 8
// groups of a sort pass (lane t of group g reads slot 8e + t of row g) and the 8-lane pairwise
// groups hit distinct banks.
constexpr int KP = K + 8;

// Scratch of one chunk of up to 4 servers (observe_kernel gives every chunk of an env its own wave
// and scratch, so the per-wave LDS footprint -- and the occupancy -- is the same at every S).
constexpr int kObsChunk = 4;

struct ObsScratch {
  static constexpr int MAXS = kObsChunk;
  uint32_t vals[2 * MAXS][KP];  // reservoir r = 2s (fct) / 2s+1 (duration), slot order; then
                                // sorted, transposed: sorted position p at (p & 15) * 8 + (p >> 4)
  float wts[MAXS][KP];          // decay weights of server s (shared by its two reservoirs)
  int n[2 * MAXS];             // valid slots per reservoir
  float mean[2 * MAXS], sd[2 * MAXS], md[2 * MAXS], p90[2 * MAXS], p90d[2 * MAXS];
  double swt[MAXS], svw[2 * MAXS];
  uint8_t perm[8][K];           // two-pass sort: slot at each position after the first pass
};

// Key-only sort of 128 keys held by the 8 lanes of a group (sorted index 16 t + e), all-ascending
// "flip" form of the bitonic network: the first step of the merge of size k pairs i with
// i ^ (k - 1), the following steps pair i with i ^ j, and every pair leaves its minimum at the
// lower index -- no step depends on a direction bit.  In-register pairs are one v_min + one v_max;
// a cross-lane step fetches the partner's key by DPP and keeps med3(key, partner, lower ? 0 : ~0).
template <int M, bool FLIP>
__device__ __forceinline__ void cross_step_keys(uint32_t (&key)[16], int t, int lowbit) {
  const uint32_t bound = (t & lowbit) ? 0xFFFFFFFFu : 0u;
  uint32_t pk[16];
#pragma unroll
  for (int e = 0; e < 16; ++e) pk[e] = xor_lane_z<M>(key[FLIP ? (e ^ 15) : e], t);
#pragma unroll
  for (int e = 0; e < 16; ++e) {
    const uint32_t a = key[e], b = pk[e];
    const uint32_t mn = a < b ? a : b, mx = a < b ? b : a;
    const uint32_t hi = mx < bound ? mx : bound;
    key[e] = mn > hi ? mn : hi;  // med3(a, b, bound)
  }
}

__device__ __forceinline__ void inreg_steps_keys(uint32_t (&key)[16], int kflip, int jtop) {
  if (kflip) {
#pragma unroll
    for (int e = 0; e < 16; ++e) {
      const int f = e ^ (kflip - 1);
      if (f > e) {
        const uint32_t a = key[e], b = key[f];
        key[e] = a < b ? a : b;
        key[f] = a < b ? b : a;
      }
    }
  }
#pragma unroll
  for (int j = jtop; j > 0; j >>= 1) {
#pragma unroll
    for (int e = 0; e < 16; ++e) {
      const int f = e ^ j;
      if (f > e) {
        const uint32_t a = key[e], b = key[f];
        key[e] = a < b ? a : b;
        key[f] = a < b ? b : a;
      }
    }
  }
}

// Ascending sort of a lane's 16 keys by Green's 60-comparator, 10-layer network (Knuth TAOCP
// 5.3.4; checked for all 2^16 0-1 inputs) instead of the 80 comparators of the bitonic stages
// k = 2..16: any network that sorts the lane's keys ascending leaves the same keys.
__device__ __forceinline__ void sort16_keys(uint32_t (&key)[16]) {
  constexpr int8_t net[60][2] = {
      {0, 13}, {1, 12}, {2, 15}, {3, 14}, {4, 8},  {5, 6},   {7, 11},  {9, 10},
      {0, 5},  {1, 7},  {2, 9},  {3, 4},  {6, 13}, {8, 14},  {10, 15}, {11, 12},
      {0, 1},  {2, 3},  {4, 5},  {6, 8},  {7, 9},  {10, 11}, {12, 13}, {14, 15},
      {0, 2},  {1, 3},  {4, 10}, {5, 11}, {6, 7},  {8, 9},   {12, 14}, {13, 15},
      {1, 2},  {3, 12}, {4, 6},  {5, 7},  {8, 10}, {9, 11},  {13, 14},
      {1, 4},  {2, 6},  {5, 8},  {7, 10}, {9, 13}, {11, 14},
      {2, 4},  {3, 6},  {9, 12}, {11, 13},
      {3, 5},  {6, 8},  {7, 9},  {10, 12},
      {3, 4},  {5, 6},  {7, 8},  {9, 10}, {11, 12},
      {6, 7},  {8, 9}};
#pragma unroll
  for (int c = 0; c < 60; ++c) {
    const uint32_t a = key[net[c][0]], b = key[net[c][1]];
    key[net[c][0]] = a < b ? a : b;
    key[net[c][1]] = a < b ? b : a;
  }
}

__device__ __forceinline__ void bitonic128_keys_g8(uint32_t (&key)[16], int t) {
  sort16_keys(key);                      // k = 2 .. 16 (each lane's 16 keys ascending)
  cross_step_keys<1, true>(key, t, 1);   // k = 32
  inreg_steps_keys(key, 0, 8);
  cross_step_keys<3, true>(key, t, 2);   // k = 64
  cross_step_keys<1, false>(key, t, 1);
  inreg_steps_keys(key, 0, 8);
  cross_step_keys<7, true>(key, t, 4);   // k = 128
  cross_step_keys<2, false>(key, t, 2);
  cross_step_keys<1, false>(key, t, 1);
  inreg_steps_keys(key, 0, 8);
}

// Reservoir sample -> float seconds.  Simulator reservoirs hold integer microseconds (US); the
// stateless features API hands in float bits.
template <bool US>
__device__ __forceinline__ float sample_value(uint32_t raw) {
  if constexpr (US) return (float)(int32_t)raw * 1.0e-6f;  // signed: lost-FIN guesses (lost_fct)
  else return __uint_as_float(raw);
}


// p90 of a full reservoir (numpy 'linear', float32 virtual index (K - 1) * 0.9f): sorted
// positions 114 and 115, both in lane 7 of the sorting group (sorted position 16 t + e).
constexpr int kP90Lo = (K - 1) * 9 / 10;
static_assert(kP90Lo == 114 && (kP90Lo & 15) != 15, "p90 pair inside one lane");

// observe_chunk with every value in registers, for simulator state whose chunk (<= 4 servers) has
// n >= 8 samples in each reservoir and every sample below kPackLimit (FULL: n = K, the steady
// state; else n in [8, K), the first steps of an episode).  Lane (g, j), g = 2 u + r, owns
// reservoir r (0 fct, 1 duration) of server s_base + u and holds its slots 8 e + j, e = 0..15 --
// numpy's pairwise accumulator j (reservoir.py:143-155) over the slots below m8 = n - n % 8; the
// tail slots [m8, n) are added in order after the accumulators are combined.  The two groups of a
// server (lanes 16 u .. 16 u + 15, one DPP row) compute half of the decay weights each and swap
// halves by row_ror:8.  LDS holds the 2^-48 fixed-point weights by slot (gathered after the sort;
// 0 for empty slots) and, when n < K, the tail values and the sorted keys for the p90 pair.  Same
// operations in the same order as the general path, so the same bits.
template <bool INC, bool FULL>
__device__ __forceinline__ void observe_chunk_regs(const DevState& st, const SimParams& p, size_t b,
                                                   int s_base, int S, int n_in, ObsScratch& sc,
                                                   float* obs_out, int lane) {
  const size_t srow = b * (size_t)p.S + (size_t)s_base;
  const int g = lane >> 3, j = lane & 7, u = g >> 1, r = g & 1;
  const bool act = u < S;
  const size_t sb = srow + (size_t)(act ? u : 0);
  const int n = FULL ? K : n_in;  // this group's sample count
  const int m8 = FULL ? K : n - (n & 7);
  // values of reservoir r (the 8-B record is {fct, ts}; the duration reservoir is the duration
  // plane when the handle has one, else the fct words again); timestamps of the half of the slots
  // whose weights this group computes, 8 (q + 8 r) + j -- the pair's other group reads the other
  // half, and the newest timestamp is a max over the 16 lanes of the pair
  const uint32_t* rec = reinterpret_cast<const uint32_t*>(st.res + sb * K + (size_t)j);
  const bool dplane = r == 1 && st.res_dur != nullptr;
  const uint32_t* vb = dplane ? st.res_dur + sb * K + (size_t)j : rec;
  const uint32_t vstep = dplane ? 8u : 16u;
  uint32_t key[16], th[8];
#pragma unroll
  for (int e = 0; e < 16; ++e) key[e] = vb[vstep * (uint32_t)e];
  const uint32_t* rts = rec + 1 + 128 * r;
#pragma unroll
  for (int q = 0; q < 8; ++q) {
    th[q] = rts[16 * q];
    if constexpr (!FULL) th[q] = 8 * (q + 8 * r) + j < n ? th[q] : 0u;  // empty slots: stale words
  }
  uint32_t tmax = 0;
#pragma unroll
  for (int q = 0; q < 8; ++q) tmax = th[q] > tmax ? th[q] : tmax;
  uint32_t o = xor_lane_z<1>(tmax, lane);
  tmax = o > tmax ? o : tmax;
  o = xor_lane_z<2>(tmax, lane);
  tmax = o > tmax ? o : tmax;
  o = xor_lane_z<4>(tmax, lane);
  tmax = o > tmax ? o : tmax;
  o = xor_lane_z<8>(tmax, lane);
  tmax = o > tmax ? o : tmax;

  // decay weights: group r computes slots 8 (q + 8 r) + j, q < 8, swaps halves with its partner
  float wh[8], w[16];
  uint64_t* wfix = reinterpret_cast<uint64_t*>(&sc.vals[0][0]) + u * K;  // [4][K] u64
#pragma unroll
  for (int q = 0; q < 8; ++q) {
    const int slot = 8 * (q + 8 * r) + j;
    wh[q] = lb_exp2f((float)(tmax - th[q]) * p.decay_c);
    if constexpr (!FULL) wh[q] = slot < n ? wh[q] : 0.0f;
    if (act) wfix[slot] = (uint64_t)(wh[q] * 281474976710656.0f);
  }
#pragma unroll
  for (int q = 0; q < 8; ++q) {
    const float pw = __uint_as_float(xor_lane_z<8>(__float_as_uint(wh[q]), lane));
    w[q] = r ? pw : wh[q];
    w[q + 8] = r ? wh[q] : pw;
  }

  // numpy-order sums (pairwise8 / pairwise8x2): accumulator j over e (terms past m8 are +0: every
  // term is >= 0, so adding +0 changes no bit), xor-combine, then the tail
  float vf[16];
#pragma unroll
  for (int e = 0; e < 16; ++e) vf[e] = sample_value<true>(key[e]);
  auto in_acc = [&](int e) { return FULL || 8 * e + j < m8; };
  float acc = vf[0];
#pragma unroll
  for (int e = 1; e < 16; ++e) acc += in_acc(e) ? vf[e] : 0.0f;
  acc = acc + xor_f32_z<1>(acc, lane);
  acc = acc + xor_f32_z<2>(acc, lane);
  acc = acc + xor_f32_z<4>(acc, lane);
  double svw = (double)vf[0] * (double)w[0], sw = (double)w[0];
#pragma unroll
  for (int e = 1; e < 16; ++e) {
    const double wi = (double)w[e];
    // a product of two floats is exact in double, so fma(v, w, svw) rounds exactly as numpy's
    // product-then-add: one f64 op instead of two
    svw = in_acc(e) ? fma((double)vf[e], wi, svw) : svw;
    sw += in_acc(e) ? wi : 0.0;
  }
  svw = svw + xor_f64_z<1>(svw, lane);
  sw = sw + xor_f64_z<1>(sw, lane);
  svw = svw + xor_f64_z<2>(svw, lane);
  sw = sw + xor_f64_z<2>(sw, lane);
  svw = svw + xor_f64_z<4>(svw, lane);
  sw = sw + xor_f64_z<4>(sw, lane);
  float* tail_v = reinterpret_cast<float*>(&sc.wts[0][0]) + g * 16;  // [8 groups][8] tail values
  float* tail_w = reinterpret_cast<float*>(&sc.perm[0][0]) + g * 16;  // [8 groups][8] tail weights
  int ntail = 0;
  if constexpr (!FULL) {  // slots [m8, n) are lanes 0 .. n - m8 - 1 at e = m8 / 8: through LDS
    ntail = n - m8;
    const int et = m8 >> 3;
#pragma unroll
    for (int e = 0; e < 16; ++e)
      if (e == et) {
        tail_v[j] = vf[e];
        tail_w[j] = w[e];
      }
    wave_sync();
    for (int k = 0; k < ntail; ++k) {
      const float tv = tail_v[k], tw = tail_w[k];
      acc += tv;
      svw = fma((double)tv, (double)tw, svw);
      sw += (double)tw;
    }
  }
  const float mean = acc / (float)n;
  float ss;
  {
    float dv = vf[0] - mean;
    ss = dv * dv;
#pragma unroll
    for (int e = 1; e < 16; ++e) {
      dv = vf[e] - mean;
      ss += in_acc(e) ? dv * dv : 0.0f;
    }
  }
  ss = ss + xor_f32_z<1>(ss, lane);
  ss = ss + xor_f32_z<2>(ss, lane);
  ss = ss + xor_f32_z<4>(ss, lane);
  if constexpr (!FULL) {
    for (int k = 0; k < ntail; ++k) {
      const float dv = tail_v[k] - mean;
      ss += dv * dv;
    }
  }
  const float sd = sqrtf(ss / (float)n);
  const float md = (float)(svw / sw);

  // order statistics: one key-only sort of (us << 7 | slot), empty slots last
#pragma unroll
  for (int e = 0; e < 16; ++e) {
    key[e] = (key[e] << 7) | (uint32_t)(8 * e + j);
    if constexpr (!FULL) key[e] = 8 * e + j < n ? key[e] : 0xFFFFFFFFu;
  }
  bitonic128_keys_g8(key, j);
  wave_sync();  // wfix complete
  uint64_t incl[16];
  uint64_t run = 0;
#pragma unroll
  for (int e = 0; e < 16; ++e) {
    run += wfix[key[e] & 127u];
    incl[e] = run;
    key[e] >>= 7;
  }
  uint64_t excl = 0;
#pragma unroll
  for (int dd = 1; dd < 8; dd <<= 1) {
    const uint32_t lo = (uint32_t)__shfl_up((int)(uint32_t)(run + excl), (unsigned)dd, 8);
    const uint32_t hi = (uint32_t)__shfl_up((int)(uint32_t)((run + excl) >> 32), (unsigned)dd, 8);
    if (j >= dd) excl += ((uint64_t)hi << 32) | lo;
  }
  const uint64_t tot_incl = run + excl;
  const uint32_t tlo = (uint32_t)__shfl((int)(uint32_t)tot_incl, (lane & ~7) | 7, 64);
  const uint32_t thi = (uint32_t)__shfl((int)(uint32_t)(tot_incl >> 32), (lane & ~7) | 7, 64);
  const uint64_t thr = ((((uint64_t)thi << 32) | tlo) * 9u + 9u) / 10u;
  const uint64_t thr_lane = thr > excl ? thr - excl : 0u;
  // the first e with incl[e] >= thr_lane holds this lane's smallest such key (keys ascend with
  // e): a min instead of a register-indexed read; past the last position: position 127.  The
  // crossing is always at a filled position (empty slots add no weight).
  uint32_t cand = 0xFFFFFFFFu;
#pragma unroll
  for (int e = 0; e < 16; ++e) {
    const uint32_t c = incl[e] >= thr_lane ? key[e] : 0xFFFFFFFFu;
    cand = c < cand ? c : cand;
  }
  const bool crosses = incl[15] >= thr_lane;
  const uint64_t m = __ballot(crosses);
  const uint32_t gm = (uint32_t)(m >> (lane & ~7)) & 0xFFu;
  const int tstar = gm ? __builtin_ctz(gm) : 7;
  cand = crosses ? cand : key[15];
  const float p90d = sample_value<true>(shfl_u32(cand, (lane & ~7) | tstar));
  // p90 (reservoir.py:144, numpy 2 'linear' in float32): virtual index (n - 1) * 0.9f; at n = K
  // sorted positions kP90Lo, kP90Lo + 1 of lane 7, else read back from LDS
  float p90;
  {
    const float hidx = (float)(n - 1) * 0.9f;
    const float fl = floorf(hidx);
    const float gg = hidx - fl;
    float va, vb;
    if constexpr (FULL) {
      va = sample_value<true>(key[kP90Lo & 15]);
      vb = sample_value<true>(key[(kP90Lo & 15) + 1]);
    } else {
      wave_sync();  // every gather from wfix done: reuse sc.vals for the sorted keys
      uint32_t* srt = &sc.vals[g][0];
#pragma unroll
      for (int e = 0; e < 16; ++e) srt[16 * j + e] = key[e];
      wave_sync();
      const int lo = (int)fl;
      va = sample_value<true>(srt[lo]);
      vb = sample_value<true>(srt[lo + 1 < n ? lo + 1 : lo]);
    }
    const float diff = vb - va;
    p90 = (gg >= 0.5f) ? (vb - diff * (1.0f - gg)) : (va + diff * gg);
    if constexpr (FULL) p90 = __uint_as_float(shfl_u32(__float_as_uint(p90), (lane & ~7) | 7));
  }
  // row of server u: lane j < 5 of group r writes feature j of reservoir r; lane 5 of the fct
  // group writes n_flow_on
  if (act) {
    const size_t so = srow + (size_t)u;
    if (j < 5) {
      const float v = j == 0 ? mean : j == 1 ? p90 : j == 2 ? sd : j == 3 ? md : p90d;
      obs_out[(s_base + u) * NF + 1 + 5 * r + j] = v;
      st.fcache[so * 10 + (size_t)(5 * r + j)] = v;
    } else if (j == 5 && r == 0) {
      obs_out[(s_base + u) * NF] = n_flow_on(st, so);
    }
  }
  wave_sync();
}

// Chooses observe_chunk_regs for a chunk of simulator state: every reservoir with n >= 8 samples
// and every sample below kPackLimit (else false: the general path; reservoirs with n < 8 sum
// sequentially in numpy, samples >= 2^25 - 1 us need the two-pass sort).  FULL (all n = K, the
// steady state) is a wave-uniform choice.
// rc / hcw: res_count and hc of the lane's server s_base + (lane >> 4), loaded by the caller
// together with the written-slot masks (one round trip for the three).
template <bool INC>
__device__ __forceinline__ bool observe_chunk_full(const DevState& st, const SimParams& p, size_t b,
                                                   int s_base, int S, ObsScratch& sc,
                                                   float* obs_out, int lane, uint32_t rc,
                                                   uint32_t hcw) {
  const bool act = (lane >> 4) < S;
  const int n = rc < (uint32_t)K ? (int)rc : K;
  // a reservoir with fewer than 8 samples, or one that ever stored a sample >= kPackLimit since it
  // was emptied (the sticky kHcBig flag the dynamics set): the general path
  if (__any(act && (n < 8 || (hcw & kHcBig) != 0u))) return false;
  const bool full = !__any(act && n < K);
  if (full) observe_chunk_regs<INC, true>(st, p, b, s_base, S, K, sc, obs_out, lane);
  else observe_chunk_regs<INC, false>(st, p, b, s_base, S, n, sc, obs_out, lane);
  return true;
}

// The 11-column observation rows (features.py:256-286) of servers [s_base, s_base + S), S <= 4,
// of env b into obs_out.  Slot-order sums follow numpy exactly (reservoir.py:143-155); order
// statistics come from the sorted keys (reservoir.py:144, 165-196).
// INC (step mode with state): a chunk none of whose reservoirs this step's dynamics wrote
// (DevState::chg all zero) takes its features from DevState::fcache instead of recomputing them;
// every computed chunk refreshes the cache (US: reset and step modes).  A reset (also the one
// inside a next-step auto-reset step) marks slot 0 of every server written, so a reset env never
// takes the previous episode's cached features, with no reset flag to load here.
// REGS = false: the general path only -- observe_rows_paired's fallback for rows the register
// path cannot take (one copy of the code instead of two more register-path instantiations: fewer
// SGPR / VGPR spills in observe_pair_kernel, 131 -> 125 us at 65536 x 4, 241 -> 229 us at
// 65536 x 8, profiles/r05f/; LBSIM_OBS_PAIR_FALLBACK_REGS=1 restores the full observe_chunk).
// The general path of observe_chunk (LDS image of the reservoirs) for servers [s_base, s_base +
// S) of env b.  Split handles (lost-FIN, DevState::res_count_dur) give the duration reservoir its
// own count and timestamps, hence its own decay weights: reservoir r then uses weight row r (S <= 2
// per call), else the server's row r >> 1.
template <bool US, bool SPLIT>
__device__ __forceinline__ void observe_chunk_general(const DevState& st, const SimParams& p,
                                                      size_t b, int s_base, int S, ObsScratch& sc,
                                                      float* obs_out, int lane) {
  const size_t srow = b * (size_t)p.S + (size_t)s_base;  // first (env, server) of the chunk
  const int R = 2 * S;
  const int g = lane >> 3, j = lane & 7;
  const bool split = US && SPLIT && st.res_count_dur != nullptr;
  const int wsh = split ? 0 : 1;  // reservoir r's weight row: r >> wsh
  // ---- phase 1: reservoirs into LDS, decay weights relative to each server's newest sample.
  //      Loads of 4 servers are issued before any is consumed (memory-level parallelism).
  for (int s0 = 0; s0 < S; s0 += 4) {
    uint32_t f[4][2], d[4][2], t[4][2], td[4][2];
    int nn[4];
    int nd[4];  // the duration reservoir's count (split handles; else nn)
#pragma unroll
    for (int u = 0; u < 4; ++u) {  // the counts first: one round trip, then every slot load
      const int s = s0 + u;
      const uint32_t rcl = st.res_count[srow + (size_t)(s < S ? s : 0)];  // branch-free loads
      const uint32_t rcd = split ? st.res_count_dur[srow + (size_t)(s < S ? s : 0)] : rcl;
      const uint32_t rc = s < S ? rcl : 0u;
      const uint32_t rd = s < S ? rcd : 0u;
      nn[u] = rc < (uint32_t)K ? (int)rc : K;
      nd[u] = rd < (uint32_t)K ? (int)rd : K;
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int s = s0 + u;
      const size_t sb = srow + (size_t)(s < S ? s : 0);
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const int slot = lane + 64 * h;
        const bool v = slot < nn[u];
        if constexpr (US) {  // simulator: one 8-B record per slot (+ the duration plane)
          const bool dplane = st.res_dur != nullptr;
          const uint2 rec = v ? st.res[sb * K + slot] : make_uint2(0u, 0u);
          if (split) {  // the duration reservoir's own {us, ts} records
            const bool vd = slot < nd[u];
            const uint2 dr = vd ? reinterpret_cast<const uint2*>(st.res_dur)[sb * K + slot]
                                : make_uint2(0u, 0u);
            d[u][h] = dr.x;
            td[u][h] = dr.y;
          } else {
            // (the plane's load must not wait for the record: both issued, then the select)
            const uint32_t dw = (v && dplane) ? st.res_dur[sb * K + slot] : 0u;
            d[u][h] = dplane ? dw : rec.x;
            td[u][h] = rec.y;
          }
          f[u][h] = rec.x;
          t[u][h] = rec.y;
        } else {  // features API: one value array serves as both "fct" and "duration"
          f[u][h] = v ? st.feat_vals[sb * K + slot] : 0u;
          d[u][h] = f[u][h];
          t[u][h] = v ? st.feat_ts[sb * K + slot] : 0u;
          td[u][h] = t[u][h];
        }
      }
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int s = s0 + u;
      if (s < S) {
        const uint32_t newest = wave_max_u32(t[u][0] > t[u][1] ? t[u][0] : t[u][1], lane);
        // split: the duration reservoir's weights from its own timestamps (weight row 2 s + 1)
        const uint32_t newd =
            split ? wave_max_u32(td[u][0] > td[u][1] ? td[u][0] : td[u][1], lane) : 0u;
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          const int slot = lane + 64 * h;
          sc.vals[2 * s][slot] = f[u][h];
          sc.vals[2 * s + 1][slot] = d[u][h];
          sc.wts[split ? 2 * s : s][slot] =
              slot < nn[u] ? lb_exp2f((float)(newest - t[u][h]) * p.decay_c) : 0.0f;
          if (split)
            sc.wts[2 * s + 1][slot] =
                slot < nd[u] ? lb_exp2f((float)(newd - td[u][h]) * p.decay_c) : 0.0f;
        }
        if (lane == 0) {
          sc.n[2 * s] = nn[u];
          sc.n[2 * s + 1] = nd[u];
        }
      }
    }
  }
  wave_sync();

  // ---- phase 2: numpy-order sums, one job per 8-lane group
  for (int job0 = 0; job0 < R; job0 += 8) {  // float32 means
    const int r = job0 + g;
    const int n = r < R ? sc.n[r] : 0;
    const uint32_t* a = sc.vals[r < R ? r : 0];
    const float sum = pairwise8<float>(n, j, [&](int i) { return sample_value<US>(a[i]); });
    if (j == 0 && r < R) sc.mean[r] = n > 0 ? sum / (float)n : 0.0f;
  }
  for (int job0 = 0; job0 < R; job0 += 8) {  // float64 sum v*w and sum w, one job per reservoir
    const int r = job0 + g;
    const int n = r < R ? sc.n[r] : 0;
    const uint32_t* a = sc.vals[r < R ? r : 0];
    const float* w = sc.wts[r < R ? r >> wsh : 0];
    double sw;
    const double svw = pairwise8x2<double>(n, j, sw, [&](int i, double& wi) {
      wi = (double)w[i];
      return (double)sample_value<US>(a[i]) * wi;
    });
    if (j == 0 && r < R) {
      sc.svw[r] = svw;
      // the two reservoirs of a server share w (split handles: each its own)
      if (split || (r & 1) == 0) sc.swt[r >> wsh] = sw;
    }
  }
  wave_sync();
  for (int job0 = 0; job0 < R; job0 += 8) {  // float32 sum (v - mean)^2
    const int r = job0 + g;
    const int n = r < R ? sc.n[r] : 0;
    const uint32_t* a = sc.vals[r < R ? r : 0];
    const float m = r < R ? sc.mean[r] : 0.0f;
    const float ss = pairwise8<float>(n, j, [&](int i) {
      const float dv = sample_value<US>(a[i]) - m;
      return dv * dv;
    });
    if (j == 0 && r < R) {
      sc.sd[r] = n > 0 ? sqrtf(ss / (float)n) : 0.0f;
      sc.md[r] = n > 0 ? (float)(sc.svw[r] / sc.swt[r >> wsh]) : 0.0f;
    }
  }
  wave_sync();

  // ---- phase 3: order statistics, 8 reservoirs per pass (one per 8-lane group)
  for (int r0 = 0; r0 < R; r0 += 8) {
    const int r = r0 + g;
    const bool act = r < R;
    const int rr = act ? r : 0;
    const int n = act ? sc.n[r] : 0;
    const float* wrow = sc.wts[rr >> wsh];
    uint32_t* vrow = sc.vals[rr];
    // any initial placement sorts to the same keys; ties only permute equal keys, which changes
    // neither p90 nor the weighted p90 (exact integer cumsums), so load strided (bank-free)
    uint32_t key[16];
    uint32_t pay[16];  // float weight bits of sorted element e
    uint32_t vmax = 0;
#pragma unroll
    for (int e = 0; e < 16; ++e) {
      const int slot = 8 * e + j;
      key[e] = slot < n ? vrow[slot] : 0u;
      vmax = key[e] > vmax ? key[e] : vmax;
    }
    // Key-only sorts of (sample << 7 | slot).  One pass when every sample of the wave's 8
    // reservoirs is below 2^25 - 1 (simulator samples in us: flows under 33 s); otherwise, and
    // always for float bits, an LSD pair of passes: low 16 bits then (high 16 bits << 7 | rank
    // after the first pass), which orders by the full 32-bit sample.  Wave-uniform branch.
    const bool one = US && !__any(vmax >= kPackLimit);
#pragma unroll
    for (int e = 0; e < 16; ++e) {
      const int slot = 8 * e + j;
      key[e] = slot < n ? (((one ? key[e] : (key[e] & 0xFFFFu)) << 7) | (uint32_t)slot) : 0xFFFFFFFFu;
    }
    bitonic128_keys_g8(key, j);
    if (one) {
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        const bool v = 16 * j + e < n;
        pay[e] = v ? __float_as_uint(wrow[key[e] & 127u]) : 0u;
        key[e] = v ? key[e] >> 7 : 0xFFFFFFFFu;
      }
    } else {
      uint8_t* perm = sc.perm[g];  // slot at each position of the first pass
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        const int pos = 16 * j + e;
        const uint32_t slot = key[e] & 127u;
        if (pos < n) perm[pos] = (uint8_t)slot;
        // simulator samples are signed us (lost-FIN guesses can be negative): the high half
        // with its sign bit flipped orders them as int32
        const uint32_t hi = (vrow[slot] ^ (US ? 0x80000000u : 0u)) >> 16;
        key[e] = pos < n ? ((hi << 7) | (uint32_t)pos) : 0xFFFFFFFFu;
      }
      bitonic128_keys_g8(key, j);
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        const bool v = 16 * j + e < n;
        const int slot = v ? perm[key[e] & 127u] : 0;
        pay[e] = v ? __float_as_uint(wrow[slot]) : 0u;
        key[e] = v ? vrow[slot] : 0xFFFFFFFFu;
      }
    }
    // decay-weighted p90: cumulative 2^-48 fixed-point weight in sorted order, first position
    // with 10 * cum >= 9 * total (searchsorted 'left' of 0.9 * cumsum[-1])
    uint64_t incl[16];
    uint64_t run = 0;
#pragma unroll
    for (int e = 0; e < 16; ++e) {
      run += (uint64_t)(__uint_as_float(pay[e]) * 281474976710656.0f);
      incl[e] = run;
    }
    uint64_t excl = 0;  // sum of the totals of lanes t' < t of this group (exact integers)
#pragma unroll
    for (int dd = 1; dd < 8; dd <<= 1) {
      const uint32_t lo = (uint32_t)__shfl_up((int)(uint32_t)(run + excl), (unsigned)dd, 8);
      const uint32_t hi = (uint32_t)__shfl_up((int)(uint32_t)((run + excl) >> 32), (unsigned)dd, 8);
      if (j >= dd) excl += ((uint64_t)hi << 32) | lo;
    }
    // (the loop above is an inclusive scan of lane totals written as run + excl; excl now holds
    //  the exclusive prefix)
    const uint64_t tot_incl = run + excl;
    const uint32_t tlo = (uint32_t)__shfl((int)(uint32_t)tot_incl, (lane & ~7) | 7, 64);
    const uint32_t thi = (uint32_t)__shfl((int)(uint32_t)(tot_incl >> 32), (lane & ~7) | 7, 64);
    // 10 c >= 9 T  <=>  c >= ceil(9 T / 10) for integers (T < 2^55, so 9 T fits)
    const uint64_t thr = ((((uint64_t)thi << 32) | tlo) * 9u + 9u) / 10u;
    const uint64_t thr_lane = thr > excl ? thr - excl : 0u;  // this lane's share of the threshold
    int fe = 0;  // first e with excl + incl[e] >= thr (incl is non-decreasing): count of those below
#pragma unroll
    for (int e = 0; e < 16; ++e) fe += incl[e] < thr_lane ? 1 : 0;
    const uint64_t m = __ballot(fe < 16);
    const uint32_t gm = (uint32_t)(m >> (lane & ~7)) & 0xFFu;
    const int tstar = gm ? __builtin_ctz(gm) : 7;
    const int fstar = __shfl(fe, (lane & ~7) | tstar, 64);
    const int pd = 16 * tstar + (fstar < 16 ? fstar : 15);
    // sorted keys back into LDS (slot-order values are no longer needed)
#pragma unroll
    for (int e = 0; e < 16; ++e)
      if (act) sc.vals[rr][e * 8 + j] = key[e];  // sorted position 16 j + e, transposed
    wave_sync();
    if (j == 0 && act) {
      float p90 = 0.0f, p90d = 0.0f;
      if (n > 0) {
        // numpy 2 'linear' (float32): virtual index (n - 1) * float32(0.9), _lerp
        const float hidx = (float)(n - 1) * 0.9f;
        const float fl = floorf(hidx);
        const int lo = (int)fl;
        const float gg = hidx - fl;
        auto sorted = [&](int pos) { return sample_value<US>(sc.vals[r][(pos & 15) * 8 + (pos >> 4)]); };
        const float va = sorted(lo);
        const float vb = sorted(lo + 1 < n ? lo + 1 : lo);
        const float diff = vb - va;
        p90 = (gg >= 0.5f) ? (vb - diff * (1.0f - gg)) : (va + diff * gg);
        p90d = sorted(pd);
      }
      sc.p90[r] = p90;
      sc.p90d[r] = p90d;
    }
    wave_sync();
  }

  // ---- observation rows: [n_flow_on, fct x5, duration x5]
  for (int e = lane; e < S * NF; e += 64) {
    const int s = e / NF, c = e - s * NF;
    float v;
    if (c == 0) {
      v = n_flow_on(st, srow + (size_t)s);
    } else {
      const int r = 2 * s + (c >= 6 ? 1 : 0);
      const int f = (c - 1) % 5;
      v = f == 0 ? sc.mean[r] : f == 1 ? sc.p90[r] : f == 2 ? sc.sd[r] : f == 3 ? sc.md[r] : sc.p90d[r];
      if constexpr (US) st.fcache[(srow + (size_t)s) * 10 + (size_t)(c - 1)] = v;
    }
    obs_out[s_base * NF + e] = v;
  }
  wave_sync();
}


// SPLIT = false: the caller never sees a split (lost-FIN) handle -- the paired observe and the
// one-wave-per-env forms -- and the split code is compiled out of it.
template <bool US, bool INC, bool REGS = true, bool SPLIT = true>
__device__ __forceinline__ void observe_chunk(const DevState& st, const SimParams& p, size_t b,
                                              int s_base, int S, ObsScratch& sc, float* obs_out,
                                              int lane) {
  const size_t srow = b * (size_t)p.S + (size_t)s_base;  // first (env, server) of the chunk
  // the register path's decision words, issued with the written-slot masks (no round trip of
  // their own after the unchanged-chunk test)
  uint32_t rc = 0u, hcw = 0u;
  if constexpr (US) {
    const size_t usb = srow + (size_t)((lane >> 4) < S ? (lane >> 4) : 0);
    rc = st.res_count[usb];
    hcw = st.hc[usb];
  }
  if constexpr (INC) {
    const uint32_t w = lane < 4 * S ? st.chg[(srow + (size_t)(lane >> 2)) * 4 + (lane & 3)] : 0u;
    if (!__any(w != 0u)) {  // no reservoir of the chunk changed: the cached features
      for (int e = lane; e < S * NF; e += 64) {
        const int s = e / NF, c = e - s * NF;
        obs_out[s_base * NF + e] = c == 0 ? n_flow_on(st, srow + (size_t)s)
                                          : st.fcache[(srow + (size_t)s) * 10 + (size_t)(c - 1)];
      }
      wave_sync();
      return;
    }
  }
  if constexpr (US && REGS) {  // (not for split handles: their reservoirs differ in count and ts)
    if (st.res_count_dur == nullptr &&
        observe_chunk_full<INC>(st, p, b, s_base, S, sc, obs_out, lane, rc, hcw))
      return;
  }
  // split handles: two servers (four weight rows) per pass; one call site (one inlined copy of
  // the general path: two cost observe_pair_kernel 9 more VGPR spills, 92 -> 102 us, r06f)
  const int step = (US && SPLIT && st.res_count_dur != nullptr) ? 2 : S;
#pragma clang loop unroll(disable)
  for (int h = 0; h < S; h += step)
    observe_chunk_general<US, SPLIT>(st, p, b, s_base + h, S - h < step ? S - h : step, sc,
                                     obs_out, lane);
}

// ================================================================ reward (rewards.py)

// numpy pairwise sum of n <= 16 float64 terms in one thread (term(i) = element i).
template <typename F>
__device__ __forceinline__ double pw_sum64(int n, F term) {
  if (n < 8) {
    double r = 0.0;
    for (int i = 0; i < n; ++i) r += term(i);
    return r;
  }
  double r0 = term(0), r1 = term(1), r2 = term(2), r3 = term(3);
  double r4 = term(4), r5 = term(5), r6 = term(6), r7 = term(7);
  const int m8 = n - (n % 8);
  for (int i = 8; i < m8; i += 8) {
    r0 += term(i); r1 += term(i + 1); r2 += term(i + 2); r3 += term(i + 3);
    r4 += term(i + 4); r5 += term(i + 5); r6 += term(i + 6); r7 += term(i + 7);
  }
  double res = ((r0 + r1) + (r2 + r3)) + ((r4 + r5) + (r6 + r7));
  for (int i = m8; i < n; ++i) res += term(i);
  return res;
}

// RewardFunction.compute (rewards.py:329-381) over the n values x(0..n-1): the reward field of
// the active servers (any column > 0, env.py:410-413) in server order, metric in float64.
template <typename X>
__device__ __forceinline__ double reward_values(int n, X x, int metric) {
  if (n == 0) return 0.0;
  const double eps = 1e-10;
  auto var = [&]() {
    const double mean = pw_sum64(n, x) / (double)n;
    return pw_sum64(n, [&](int i) { const double t = x(i) - mean; return t * t; }) / (double)n;
  };
  switch (metric) {
    case 0: {  // jain_fairness 21-67
      const double sv = pw_sum64(n, x);
      if (sv < eps) return 1.0;
      const double sq = pw_sum64(n, [&](int i) { const double v = x(i); return v * v; });
      if (sq < eps) return 1.0;
      const double j = (sv * sv) / ((double)n * sq);
      const double lo = 1.0 / (double)n;
      return j < lo ? lo : (j > 1.0 ? 1.0 : j);
    }
    case 1: return -var();        // variance_fairness 70-94
    case 2: return -sqrt(var());  // std_fairness 97-114
    case 3: {                     // coefficient_of_variation 117-144
      const double mean = pw_sum64(n, x) / (double)n;
      if (mean < eps) return 0.0;
      return -(sqrt(var()) / (mean + eps));
    }
    case 4: {  // max_min_fairness 147-171
      double m = x(0);
      for (int i = 1; i < n; ++i) m = x(i) > m ? x(i) : m;
      return -m;
    }
    case 5: {  // min_max_fairness 174-191
      double m = x(0);
      for (int i = 1; i < n; ++i) m = x(i) < m ? x(i) : m;
      return m;
    }
    case 6: return pw_sum64(n, [&](int i) { return log(x(i) + eps); });  // product 194-225
    case 7: {  // range_fairness 228-246
      double mx = x(0), mn = x(0);
      for (int i = 1; i < n; ++i) { mx = x(i) > mx ? x(i) : mx; mn = x(i) < mn ? x(i) : mn; }
      return -(mx - mn);
    }
    case 8: {  // gini_coefficient 249-287
      const double mean = pw_sum64(n, x) / (double)n;
      if (mean == 0.0) return 0.0;
      double ds = 0.0;
      for (int i = 0; i < n; ++i)
        for (int k = 0; k < n; ++k) ds += fabs(x(i) - x(k));
      return -(ds / ((double)(2 * n * n) * mean));
    }
    default: return 0.0;
  }
}

// reward_values' jain_fairness (rewards.py:21-67) for n <= 4 active values, straight-line: numpy's
// pairwise sum of n < 8 terms is the sequential sum from 0.0, and a term past n adds +0.0 to a
// non-negative partial sum (every load is >= 0), which changes no bit; 1 / n from a table of the
// correctly rounded quotients.
__device__ __forceinline__ double jain_upto4(int n, const float* x) {
  if (n == 0) return 0.0;
  const double eps = 1e-10;
  double sv = 0.0, sq = 0.0;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const double v = i < n ? (double)x[i] : 0.0;
    sv += v;
    sq += v * v;
  }
  if (sv < eps) return 1.0;
  if (sq < eps) return 1.0;
  const double j = (sv * sv) / ((double)n * sq);
  const double lo = n == 1 ? 1.0 : n == 2 ? 0.5 : n == 3 ? 1.0 / 3.0 : 0.25;
  return j < lo ? lo : (j > 1.0 ? 1.0 : j);
}

// Active servers of an (S, 11) row as a bit mask, one thread.
__device__ __forceinline__ uint64_t active_mask_seq(const float* obs, int S) {
  uint64_t m = 0;
  for (int s = 0; s < S; ++s) {
    bool active = false;
    for (int f = 0; f < NF; ++f) active |= obs[s * NF + f] > 0.0f;
    m |= active ? 1ull << s : 0ull;
  }
  return m;
}

// Position of the i-th set bit of m (i < popcount(m)).
__device__ __forceinline__ int nth_bit(uint64_t m, int i) {
  for (; i > 0; --i) m &= m - 1ull;
  return __builtin_ctzll(m);
}

// One thread, one (S, 11) row (the stateless lbsim_reward entry point).
__device__ double reward_of(const float* obs, int S, int metric, int field) {
  if (field < 0 || field >= NF) return 0.0;  // no value has the field (rewards.py:375-376)
  const uint64_t act = active_mask_seq(obs, S);
  return reward_values(__popcll(act),
                       [&](int i) { return (double)obs[nth_bit(act, i) * NF + field]; }, metric);
}

// ================================================================ paired observe (8 rows per wave)
//
// With the default duration sample (duration_mode AGE: both samples of a flow are tc - ta,
// DESIGN.md §3.4) and lost-FIN off, every flow's duration equals its fct, so the handle has no
// duration plane (DevState::res_dur == nullptr): a server's duration reservoir IS its fct
// reservoir slot for slot (same values, timestamps and count) and its 5 duration features equal
// its 5 fct features bit for bit.  observe_pair_kernel then computes each server's features
// once: one wave takes up to 8 consecutive (env, server) rows -- the 8 / S whole envs of S <= 8
// servers -- and lane (u, j) holds slots 8 e + j of row u (one 8-B {fct, ts} record each: a
// server's reservoir is 1 KiB), so a wave does the work observe_kernel spreads over two.  step_wave_kernel's S = 5-8 observe phase takes the same path for its env.
// Same operations in the same order as observe_chunk_regs' fct group: the same bits.

// (uint64_t)(w * 2^48) for w in [0, 1], from the f32 weight: hi = floor(x / 2^32), lo = the
// exact remainder x - hi 2^32 (x has <= 24 significant bits, so the remainder is a float), both
// truncated as the conversion truncates.
__device__ __forceinline__ uint64_t fixed48(float w) {
  const float x = w * 281474976710656.0f;
  const float hf = floorf(x * 2.3283064365386963e-10f);
  const uint32_t hi = (uint32_t)hf;
  const uint32_t lo = (uint32_t)fmaf(hf, -4294967296.0f, x);
  return ((uint64_t)hi << 32) | lo;
}

// hcw: the hc word of the lane's row (loaded with the decision words): column 0 from it, no load.
template <bool FULL>
__device__ __forceinline__ void observe_rows_paired_regs(const DevState& st, const SimParams& p,
                                                         size_t row0, int nrows, int n_in,
                                                         ObsScratch& sc, float* obs_out, int lane,
                                                         uint32_t hcw) {
  const int u = lane >> 3, j = lane & 7;
  const bool act = u < nrows;
  const size_t sb = row0 + (size_t)(act ? u : 0);
  const int n = FULL ? K : n_in;  // this row's sample count
  const int m8 = FULL ? K : n - (n & 7);
  // the record {fct, ts} of slots 8 e + j: one dwordx2 each, 8 lanes = 64 contiguous bytes
  const uint2* rec = st.res + sb * K + (size_t)j;
  uint32_t key[16], th[16];
#pragma unroll
  for (int e = 0; e < 16; ++e) {
    const uint2 r2 = rec[8 * e];
    key[e] = r2.x;
    th[e] = r2.y;
    if constexpr (!FULL) th[e] = 8 * e + j < n ? th[e] : 0u;  // empty slots: stale words
  }
  uint32_t tmax = 0;
#pragma unroll
  for (int e = 0; e < 16; ++e) tmax = th[e] > tmax ? th[e] : tmax;
  uint32_t o = xor_lane_z<1>(tmax, lane);
  tmax = o > tmax ? o : tmax;
  o = xor_lane_z<2>(tmax, lane);
  tmax = o > tmax ? o : tmax;
  o = xor_lane_z<4>(tmax, lane);
  tmax = o > tmax ? o : tmax;

  // decay weights of the lane's 16 slots; f32 copies by slot in LDS for the gather after the sort.
  // Row u at stride KP = 136 dwords: the 32 lanes of a ds_write_b32 half (rows u, u + 1, u + 2,
  // u + 3, slots 8 e + j) hit 32 distinct banks (a stride of 128 put 4 rows on every bank)
  float w[16];
  float* wf = reinterpret_cast<float*>(&sc.vals[u][0]);  // [8][KP] f32
#pragma unroll
  for (int e = 0; e < 16; ++e) {
    const int slot = 8 * e + j;
    w[e] = lb_exp2f((float)(tmax - th[e]) * p.decay_c);
    if constexpr (!FULL) w[e] = slot < n ? w[e] : 0.0f;
    if (act) wf[slot] = w[e];
  }

  // numpy-order sums, as observe_chunk_regs
  float vf[16];
#pragma unroll
  for (int e = 0; e < 16; ++e) vf[e] = sample_value<true>(key[e]);
  auto in_acc = [&](int e) { return FULL || 8 * e + j < m8; };
  float acc = vf[0];
#pragma unroll
  for (int e = 1; e < 16; ++e) acc += in_acc(e) ? vf[e] : 0.0f;
  acc = acc + xor_f32_z<1>(acc, lane);
  acc = acc + xor_f32_z<2>(acc, lane);
  acc = acc + xor_f32_z<4>(acc, lane);
  double svw = (double)vf[0] * (double)w[0], sw = (double)w[0];
#pragma unroll
  for (int e = 1; e < 16; ++e) {
    const double wi = (double)w[e];
    svw = in_acc(e) ? fma((double)vf[e], wi, svw) : svw;
    sw += in_acc(e) ? wi : 0.0;
  }
  svw = svw + xor_f64_z<1>(svw, lane);
  sw = sw + xor_f64_z<1>(sw, lane);
  svw = svw + xor_f64_z<2>(svw, lane);
  sw = sw + xor_f64_z<2>(sw, lane);
  svw = svw + xor_f64_z<4>(svw, lane);
  sw = sw + xor_f64_z<4>(sw, lane);
  float* tail_v = reinterpret_cast<float*>(&sc.wts[0][0]) + u * 16;  // [8 rows][8] tail values
  float* tail_w = reinterpret_cast<float*>(&sc.perm[0][0]) + u * 16;  // [8 rows][8] tail weights
  int ntail = 0;
  if constexpr (!FULL) {
    ntail = n - m8;
    const int et = m8 >> 3;
#pragma unroll
    for (int e = 0; e < 16; ++e)
      if (e == et) {
        tail_v[j] = vf[e];
        tail_w[j] = w[e];
      }
    wave_sync();
    for (int k = 0; k < ntail; ++k) {
      const float tv = tail_v[k], tw = tail_w[k];
      acc += tv;
      svw = fma((double)tv, (double)tw, svw);
      sw += (double)tw;
    }
  }
  const float mean = acc / (float)n;
  float ss;
  {
    float dv = vf[0] - mean;
    ss = dv * dv;
#pragma unroll
    for (int e = 1; e < 16; ++e) {
      dv = vf[e] - mean;
      ss += in_acc(e) ? dv * dv : 0.0f;
    }
  }
  ss = ss + xor_f32_z<1>(ss, lane);
  ss = ss + xor_f32_z<2>(ss, lane);
  ss = ss + xor_f32_z<4>(ss, lane);
  if constexpr (!FULL) {
    for (int k = 0; k < ntail; ++k) {
      const float dv = tail_v[k] - mean;
      ss += dv * dv;
    }
  }
  const float sd = sqrtf(ss / (float)n);
  const float md = (float)(svw / sw);

  // order statistics: one key-only sort of (us << 7 | slot), empty slots last
#pragma unroll
  for (int e = 0; e < 16; ++e) {
    key[e] = (key[e] << 7) | (uint32_t)(8 * e + j);
    if constexpr (!FULL) key[e] = 8 * e + j < n ? key[e] : 0xFFFFFFFFu;
  }
  bitonic128_keys_g8(key, j);
  wave_sync();  // wf complete
  uint64_t incl[16];
  uint64_t run = 0;
#pragma unroll
  for (int e = 0; e < 16; ++e) {
    run += fixed48(wf[key[e] & 127u]);
    incl[e] = run;
    key[e] >>= 7;
  }
  uint64_t excl = 0;
#pragma unroll
  for (int dd = 1; dd < 8; dd <<= 1) {
    const uint32_t lo = (uint32_t)__shfl_up((int)(uint32_t)(run + excl), (unsigned)dd, 8);
    const uint32_t hi = (uint32_t)__shfl_up((int)(uint32_t)((run + excl) >> 32), (unsigned)dd, 8);
    if (j >= dd) excl += ((uint64_t)hi << 32) | lo;
  }
  const uint64_t tot_incl = run + excl;
  const uint32_t tlo = (uint32_t)__shfl((int)(uint32_t)tot_incl, (lane & ~7) | 7, 64);
  const uint32_t thi = (uint32_t)__shfl((int)(uint32_t)(tot_incl >> 32), (lane & ~7) | 7, 64);
  const uint64_t thr = ((((uint64_t)thi << 32) | tlo) * 9u + 9u) / 10u;
  const uint64_t thr_lane = thr > excl ? thr - excl : 0u;
  uint32_t cand = 0xFFFFFFFFu;
#pragma unroll
  for (int e = 0; e < 16; ++e) {
    const uint32_t c = incl[e] >= thr_lane ? key[e] : 0xFFFFFFFFu;
    cand = c < cand ? c : cand;
  }
  const bool crosses = incl[15] >= thr_lane;
  const uint64_t m = __ballot(crosses);
  const uint32_t gm = (uint32_t)(m >> (lane & ~7)) & 0xFFu;
  const int tstar = gm ? __builtin_ctz(gm) : 7;
  cand = crosses ? cand : key[15];
  const float p90d = sample_value<true>(shfl_u32(cand, (lane & ~7) | tstar));
  float p90;
  {
    const float hidx = (float)(n - 1) * 0.9f;
    const float fl = floorf(hidx);
    const float gg = hidx - fl;
    float va, vb;
    if constexpr (FULL) {
      va = sample_value<true>(key[kP90Lo & 15]);
      vb = sample_value<true>(key[(kP90Lo & 15) + 1]);
    } else {
      wave_sync();  // every gather from wf done: reuse sc.vals for the sorted keys
      uint32_t* srt = &sc.vals[u][0];
#pragma unroll
      for (int e = 0; e < 16; ++e) srt[16 * j + e] = key[e];
      wave_sync();
      const int lo = (int)fl;
      va = sample_value<true>(srt[lo]);
      vb = sample_value<true>(srt[lo + 1 < n ? lo + 1 : lo]);
    }
    const float diff = vb - va;
    p90 = (gg >= 0.5f) ? (vb - diff * (1.0f - gg)) : (va + diff * gg);
    if constexpr (FULL) p90 = __uint_as_float(shfl_u32(__float_as_uint(p90), (lane & ~7) | 7));
  }
  // row u: lane j < 5 writes feature j to both column groups (fct 1-5, duration 6-10); lane 5
  // writes n_flow_on
  if (act) {
    if (j < 5) {
      const float v = j == 0 ? mean : j == 1 ? p90 : j == 2 ? sd : j == 3 ? md : p90d;
      obs_out[u * NF + 1 + j] = v;
      obs_out[u * NF + 6 + j] = v;
      st.fcache[sb * 10 + (size_t)j] = v;
      st.fcache[sb * 10 + (size_t)(5 + j)] = v;
    } else if (j == 5) {
      uint32_t nfo = hcw >> 16;  // n_flow_on (n_flow_on_mode VPP: + the lost-FIN flows)
      if (st.lost_on != nullptr)
        nfo += __hip_atomic_load(st.lost_on + sb, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      obs_out[u * NF] = (float)nfo;
    }
  }
  wave_sync();
}

// Rows of envs [b0, b0 + nenv) (nenv * S <= 8) into obs_out (their (S, 11) rows back to back).
// INC: unchanged rows take their cached features unless some env was reset by this step (nr:
// next-step auto-reset is on; its ep_step words are loaded with the decision words); rows
// the register path cannot take (n < 8, a sample >= kPackLimit) go through observe_chunk per env.
#ifndef LBSIM_OBS_PAIR_FALLBACK_REGS
#define LBSIM_OBS_PAIR_FALLBACK_REGS 0
#endif
template <bool INC>
__device__ __forceinline__ void observe_rows_paired(const DevState& st, const SimParams& p,
                                                    size_t b0, int nenv, ObsScratch& sc,
                                                    float* obs_out, int lane) {
  const int S = p.S, nrows = nenv * S;
  const size_t row0 = b0 * (size_t)S;
  const int u = lane >> 3;
  const bool act = u < nrows;
  const size_t usb = row0 + (size_t)(act ? u : 0);
  const uint32_t rc = st.res_count[usb];
  const uint32_t hcw = st.hc[usb];
  if constexpr (INC) {
    const uint32_t w = lane < 4 * nrows ? st.chg[(row0 + (size_t)(lane >> 2)) * 4 + (lane & 3)] : 0u;
    // one round trip for the decision words (a reset env's rows are marked written: no reset flag)
    if (!__any(w != 0u)) {  // no reservoir of the rows changed: the cached features
      for (int e = lane; e < nrows * NF; e += 64) {
        const int s = e / NF, c = e - s * NF;
        obs_out[e] = c == 0 ? n_flow_on(st, row0 + (size_t)s)
                            : st.fcache[(row0 + (size_t)s) * 10 + (size_t)(c - 1)];
      }
      wave_sync();
      return;
    }
  }
  const int n = rc < (uint32_t)K ? (int)rc : K;
  if (!__any(act && (n < 8 || (hcw & kHcBig) != 0u))) {
    if (!__any(act && n < K))
      observe_rows_paired_regs<true>(st, p, row0, nrows, K, sc, obs_out, lane, hcw);
    else
      observe_rows_paired_regs<false>(st, p, row0, nrows, n, sc, obs_out, lane, hcw);
    return;
  }
  for (int e = 0; e < nenv; ++e) {
    for (int s0 = 0; s0 < S; s0 += kObsChunk)
      observe_chunk<true, INC, LBSIM_OBS_PAIR_FALLBACK_REGS != 0, false>(
          st, p, b0 + (size_t)e, s0, S - s0 < kObsChunk ? S - s0 : kObsChunk, sc,
          obs_out + e * S * NF, lane);
  }
}

// Rows [s0, s0 + 8) of env b of a wide env (S a multiple of 8, S >= 16): the paired register
// path of observe_rows_paired over one wave's 8 rows, written to obs_env + s0 * NF; the rows the
// register path cannot take go through the two 4-server observe_chunk calls.
template <bool INC>
__device__ __forceinline__ void observe_rows_paired_wide(const DevState& st, const SimParams& p,
                                                         size_t b, int s0, ObsScratch& sc,
                                                         float* obs_env, int lane) {
  const size_t row0 = b * (size_t)p.S + (size_t)s0;
  const size_t usb = row0 + (size_t)(lane >> 3);
  float* obs_out = obs_env + s0 * NF;
  const uint32_t rc = st.res_count[usb];
  const uint32_t hcw = st.hc[usb];
  if constexpr (INC) {
    const uint32_t w = lane < 32 ? st.chg[(row0 + (size_t)(lane >> 2)) * 4 + (lane & 3)] : 0u;
    if (!__any(w != 0u)) {  // none of the 8 reservoirs changed: the cached features
      for (int e = lane; e < 8 * NF; e += 64) {
        const int s = e / NF, c = e - s * NF;
        obs_out[e] = c == 0 ? n_flow_on(st, row0 + (size_t)s)
                            : st.fcache[(row0 + (size_t)s) * 10 + (size_t)(c - 1)];
      }
      wave_sync();
      return;
    }
  }
  const int n = rc < (uint32_t)K ? (int)rc : K;
  if (!__any(n < 8 || (hcw & kHcBig) != 0u)) {
    if (!__any(n < K)) observe_rows_paired_regs<true>(st, p, row0, 8, K, sc, obs_out, lane, hcw);
    else observe_rows_paired_regs<false>(st, p, row0, 8, n, sc, obs_out, lane, hcw);
    return;
  }
  for (int c = s0; c < s0 + 8; c += kObsChunk)
    observe_chunk<true, INC, LBSIM_OBS_PAIR_FALLBACK_REGS != 0, false>(st, p, b, c, kObsChunk, sc,
                                                                 obs_env, lane);
}

// ================================================================ observe (one wave = one env)

struct ObsOutputs {
  float* obs;
  float* reward;
  uint8_t* done;
  float* raw_obs;
  int32_t* ep_len;
  double* ep_ret;
  // problem-05 facade (multi_agent_env.py:152-188, 240-258): per-agent observations [B, A, 4k +
  // 7S] of the returned rows, and the global state [B, 4S + 10]
  float* agent_obs;
  float* state;
  int num_agents, servers_per_agent;
  // one-env handles: the step's completion word (lbsim_step_outputs_t::done_word), stored after
  // every other output with a system-scope release (observe_outputs)
  uint32_t* done_word;
  uint32_t done_value;
};

// One wave per 4-server chunk (kObsChunk), all chunks of an env in one workgroup: S = 4 -> one
// wave, 8 -> 2, 16 -> 4, 64 -> 16.  Each wave computes its chunk in its own ObsScratch (dynamic
// LDS, nw * sizeof(ObsScratch) bytes at launch) with wave-level ordering only; the workgroup meets
// once, then wave 0 computes the reward and every wave writes outputs.  5 waves per SIMD at every
// S (96 VGPRs): the work per wave is the same chunk whatever S is.
template <int MAXS>
constexpr int kObsWavesPerEnv = MAXS <= kObsChunk ? 1 : MAXS / kObsChunk;

// The reward, episode bookkeeping and output rows of env b once its (S, 11) rows are in s_obs
// (rewards.py:290-381, env.py:261-281, env.py:450-470): threads tid < 64 (one wave) compute the
// reward, all nthr threads write the rows.
template <int MAXS, int MODE, bool FAC>
__device__ __forceinline__ void observe_outputs(const DevState& st, const SimParams& p,
                                                const ObsOutputs& out, size_t b,
                                                float* s_obs, float* s_act, int tid, int nthr) {
  const int S = p.S;
  // active servers (any column > 0): lane s of wave 0 scans its row, one ballot; their
  // reward-field values compacted into s_act in server order
  if (tid < 64) {
    const int lane = tid;
    bool act = false;
    if (lane < S)
      for (int f = 0; f < NF; ++f) act |= s_obs[lane * NF + f] > 0.0f;
    const uint64_t act_mask = __ballot(act);
    const bool fok = p.reward_field >= 0 && p.reward_field < NF;
    if (act && fok) s_act[__popcll(act_mask & ((1ull << lane) - 1ull))] = s_obs[lane * NF + p.reward_field];
    wave_sync();
    if (MODE == kModeStep && lane == 0) {
      const int na = __popcll(act_mask);
      double r = 0.0;
      // reset by this step (next-step auto-reset, ep_step = -1): reward 0, episode step 0, not done
      const int32_t es0 = st.ep_step[b];
      const bool fresh = p.next_reset && es0 < 0;
      if (fok && !fresh) {
        // (compile-time for observe_kernel<4>; fused G = 8 with S <= 4 at run time)
        if ((MAXS <= kObsChunk || S <= kObsChunk) && p.reward_metric == 0)
          r = jain_upto4(na, s_act);
        else
          r = reward_values(na, [&](int i) { return (double)s_act[i]; }, p.reward_metric);
      }
      out.reward[b] = (float)r;
      const int32_t es = es0 + 1;  // -1 + 1 = 0 for a fresh env
      const double er = st.ep_return[b] + r;  // 0 + 0
      st.ep_step[b] = es;
      st.ep_return[b] = er;
      out.done[b] = (uint8_t)(es >= p.max_steps ? 1 : 0);
      if (out.ep_len != nullptr) out.ep_len[b] = es;
      if (out.ep_ret != nullptr) out.ep_ret[b] = er;
    }
  }

  const int nobs = S * NF;
  float* orow = out.obs + b * (size_t)nobs;
  // FAC: the launch writes the problem-05 facade rows (a separate instantiation, so the plain
  // step carries none of that code)
  const bool facade = FAC && (out.agent_obs != nullptr || out.state != nullptr);
  if (out.raw_obs != nullptr)
    for (int e = tid; e < nobs; e += nthr) out.raw_obs[b * (size_t)nobs + e] = s_obs[e];
  if (p.normalize) {  // env.py:460-468, float64 running statistics
    const int32_t cnt = st.norm_count[b] + 1;
    for (int e = tid; e < nobs; e += nthr) {
      const size_t gi = b * (size_t)nobs + (size_t)e;
      const double o = (double)s_obs[e];
      double m = st.norm_mean[gi];
      const double sdv = st.norm_std[gi];
      const double delta = o - m;
      m = m + delta / (double)cnt;
      const double delta2 = o - m;
      double v = (sdv * sdv * (double)(cnt - 1) + delta * delta2) / (double)cnt;
      v = v > 1e-8 ? v : 1e-8;
      const double ns = sqrt(v);
      st.norm_mean[gi] = m;
      st.norm_std[gi] = ns;
      const float r = (float)((o - m) / (ns + 1e-8));
      orow[e] = r;
      if (facade) s_obs[e] = r;  // the returned rows, for the facade gather below (same thread)
    }
    if (tid == 0) st.norm_count[b] = cnt;
  } else {
    for (int e = tid; e < nobs; e += nthr) orow[e] = s_obs[e];
  }
  if (facade) {
    if (nthr == 64) wave_sync();
    else __syncthreads();  // block-uniform
    const int A = out.num_agents, k = out.servers_per_agent, D = 4 * k + 7 * S;
    if (out.agent_obs != nullptr) {  // agent a: flat[4 a k, 4 (a+1) k) ++ flat[4 S:]
      float* ao = out.agent_obs + b * (size_t)A * (size_t)D;
      for (int e = tid; e < A * D; e += nthr) {
        const int a = e / D, j = e - a * D;
        ao[e] = s_obs[j < 4 * k ? 4 * k * a + j : 4 * S + (j - 4 * k)];
      }
    }
    if (out.state != nullptr) {  // get_state: zeros ... then step / max_steps, num_agents
      const int sd = 4 * S + 10;
      float* so = out.state + b * (size_t)sd;
      for (int e = tid; e < sd - 2; e += nthr) so[e] = 0.0f;
      if (tid == 0) {
        // the episode step after this step (written by this thread above), or 0 after a reset
        // (the reset dynamics launch zeroed it)
        const int32_t es = st.ep_step[b];
        so[sd - 2] = (float)es / (float)p.max_steps;
        so[sd - 1] = (float)A;
      }
    }
  }
  if (out.done_word != nullptr) {  // one-env handles: the completion word, after every output
    if (nthr == 64) wave_sync();
    else __syncthreads();  // block-uniform
    __threadfence_system();
    if (tid == 0)
      __hip_atomic_store(out.done_word, out.done_value, __ATOMIC_RELEASE,
                         __HIP_MEMORY_SCOPE_SYSTEM);
  }
}

template <int MAXS, int MODE, bool FAC>
__global__ void __launch_bounds__(64 * kObsWavesPerEnv<MAXS>, 5)
    observe_kernel(DevState st, SimParams p, ObsOutputs out, const uint8_t* reset_mask) {
  constexpr int mode = MODE;
  const size_t b = blockIdx.x;
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6, nthr = blockDim.x;
  if (mode == kModeReset && reset_mask != nullptr && reset_mask[b] == 0) return;
  extern __shared__ double obs_dyn[];
  ObsScratch& sc = reinterpret_cast<ObsScratch*>(obs_dyn)[wv];
  __shared__ float s_obs[MAXS * NF];
  __shared__ float s_act[MAXS];
  const int S = p.S;
  {
    const int s0 = wv * kObsChunk;  // the launch has ceil(S / 4) waves
    observe_chunk<true, mode == kModeStep>(st, p, b, s0, S - s0 < kObsChunk ? S - s0 : kObsChunk,
                                           sc, s_obs, lane);
  }
  __syncthreads();
  observe_outputs<MAXS, MODE, FAC>(st, p, out, b, s_obs, s_act, tid, nthr);
}

// Step-mode observation when every record pairs dur == fct (observe_rows_paired): one wave per
// 8 / S whole envs (S <= 8: their 8 / S * S <= 8 consecutive rows), then each env's reward,
// episode words and outputs (observe_outputs, in env order).
// 4 waves per SIMD (128 VGPRs): with 5 (96 VGPRs) the register path spilled and the kernel ran
// 140 us against 130 us at 65536 x 4, 255 against 236 us at 65536 x 8 (profiles/r05d/).
#ifndef LBSIM_OBS_PAIR_WAVES
#define LBSIM_OBS_PAIR_WAVES 4
#endif
template <int MODE, bool FAC>
__global__ void __launch_bounds__(64, LBSIM_OBS_PAIR_WAVES)
    observe_pair_kernel(DevState st, SimParams p, ObsOutputs out) {
  __shared__ ObsScratch sc;
  __shared__ float s_obs[8 * NF];
  __shared__ float s_act[8];
  const int S = p.S, epw = 8 / S, lane = (int)threadIdx.x;
  const size_t b0 = (size_t)blockIdx.x * (size_t)epw;
  const int nenv = (size_t)p.B - b0 < (size_t)epw ? (int)((size_t)p.B - b0) : epw;
  // (loading the envs' episode words into LDS up front with global_load_lds measured 12 us slower
  // at 65536 x 4: 92.8 -> 104.5 us, profiles/r06e/)
  observe_rows_paired<MODE == kModeStep>(st, p, b0, nenv, sc, s_obs, lane);
  for (int e = 0; e < nenv; ++e) {
    observe_outputs<8, MODE, FAC>(st, p, out, b0 + (size_t)e, s_obs + e * S * NF, s_act, lane, 64);
    wave_sync();  // s_act reused by the next env
  }
}

// Step-mode observation of paired records for S = 16 (configs[4]'s 4 agents x 4 servers): one
// workgroup of two waves per env, wave w observing rows [8 w, 8 w + 8) (observe_rows_paired_wide),
// then the env's reward, episode words and outputs (observe_outputs) -- the work of
// observe_kernel<16>'s four chunk waves in two.
#ifndef LBSIM_OBS_PAIR16_WAVES
#define LBSIM_OBS_PAIR16_WAVES LBSIM_OBS_PAIR_WAVES
#endif
template <int MODE, bool FAC>
__global__ void __launch_bounds__(128, LBSIM_OBS_PAIR16_WAVES)
    observe_pair16_kernel(DevState st, SimParams p, ObsOutputs out) {
  __shared__ ObsScratch sc[2];
  __shared__ float s_obs[16 * NF];
  __shared__ float s_act[16];
  const size_t b = blockIdx.x;
  const int tid = (int)threadIdx.x, lane = tid & 63, wv = tid >> 6;
  observe_rows_paired_wide<MODE == kModeStep>(st, p, b, 8 * wv, sc[wv], s_obs, lane);
  __syncthreads();
  observe_outputs<16, MODE, FAC>(st, p, out, b, s_obs, s_act, tid, 128);
}

// The raw rows of paired-record wide envs (S > 16, a multiple of 8) for observe_rows_kernel: one
// single-wave workgroup per (env, 8-row group), as observe_chunks_kernel per 4-server chunk.
template <int MODE>
__global__ void __launch_bounds__(64, LBSIM_OBS_PAIR_WAVES)
    observe_pair_chunks_kernel(DevState st, SimParams p, ObsOutputs out, int ngroups) {
  const size_t b = blockIdx.x / (unsigned)ngroups;
  const int c = (int)(blockIdx.x - b * (unsigned)ngroups);
  __shared__ ObsScratch sc;
  observe_rows_paired_wide<MODE == kModeStep>(st, p, b, 8 * c, sc,
                                              out.obs + b * (size_t)p.S * NF, (int)threadIdx.x);
}

// Wide envs (S > 16: configs[4] read literally, 4 agents x 16 servers), in two launches instead of
// one workgroup of S / 4 waves per env.  observe_chunks_kernel: one single-wave workgroup per (env,
// chunk) computes the chunk's raw rows into out.obs; observe_rows_kernel: one wave per env reads
// the env's rows back and runs observe_outputs (reward, episode words, normalisation, facade).  A
// 16-wave workgroup holds 16 chunk scratches (125 KB of LDS: one workgroup per CU) and its waves
// wait for the slowest chunk and for the reward; single-wave chunks schedule like S <= 4 envs.
// Same routines in the same order: the same bits as observe_kernel.
template <int MODE>
__global__ void __launch_bounds__(64, 5)
    observe_chunks_kernel(DevState st, SimParams p, ObsOutputs out, const uint8_t* reset_mask,
                          int nchunks) {
  const size_t b = blockIdx.x / (unsigned)nchunks;
  const int c = (int)(blockIdx.x - b * (unsigned)nchunks);
  if (MODE == kModeReset && reset_mask != nullptr && reset_mask[b] == 0) return;
  __shared__ ObsScratch sc;
  const int S = p.S, s0 = c * kObsChunk, lane = (int)threadIdx.x;
  observe_chunk<true, MODE == kModeStep>(st, p, b, s0, S - s0 < kObsChunk ? S - s0 : kObsChunk,
                                         sc, out.obs + b * (size_t)S * NF, lane);
}

template <int MAXS, int MODE, bool FAC>
__global__ void __launch_bounds__(64)
    observe_rows_kernel(DevState st, SimParams p, ObsOutputs out, const uint8_t* reset_mask) {
  const size_t b = blockIdx.x;
  if (MODE == kModeReset && reset_mask != nullptr && reset_mask[b] == 0) return;
  __shared__ float s_obs[MAXS * NF];
  __shared__ float s_act[MAXS];
  const int lane = (int)threadIdx.x, n = p.S * NF;
  for (int e = lane; e < n; e += 64) s_obs[e] = out.obs[b * (size_t)n + (size_t)e];
  wave_sync();
  observe_outputs<MAXS, MODE, FAC>(st, p, out, b, s_obs, s_act, lane, 64);
}

// observe_kernel's work for env b by ONE wave, its chunks in sequence (fused_step_kernel's second
// phase).  Same routines, same order: the same bits.
#ifndef LBSIM_STEP_WAVE_PAIRED
#define LBSIM_STEP_WAVE_PAIRED 1
#endif
template <int MAXS>
__device__ __forceinline__ void observe_env_wave(const DevState& st, const SimParams& p,
                                                 const ObsOutputs& out, size_t b, ObsScratch& sc,
                                                 float* s_obs, float* s_act, int lane) {
  const int S = p.S;
  if constexpr (MAXS <= kObsChunk) {  // one chunk: straight-line code, no loop-carried s0
    observe_chunk<true, true, true, false>(st, p, b, 0, S, sc, s_obs, lane);
  } else if (LBSIM_STEP_WAVE_PAIRED && MAXS <= 8 && st.res_dur == nullptr) {
    // paired records: the env's S <= 8 rows in one pass (observe_rows_paired)
    observe_rows_paired<true>(st, p, b, 1, sc, s_obs, lane);
  } else {
    // rolled, with b and lane opaque per chunk: nothing derived from them is hoisted and held
    // across both chunks (step_wave_kernel<4, ..., 8>: 124 VGPRs instead of 184 B of spills/lane)
#pragma clang loop unroll(disable)
    for (int s0 = 0; s0 < S; s0 += kObsChunk) {
      size_t bb = b;
      int ln = lane;
      asm volatile("" : "+s"(bb), "+v"(ln));
      observe_chunk<true, true, true, false>(st, p, bb, s0, S - s0 < kObsChunk ? S - s0 : kObsChunk,
                                             sc, s_obs, ln);
    }
  }
  observe_outputs<MAXS, kModeStep, true>(st, p, out, b, s_obs, s_act, lane, 64);
  wave_sync();  // s_obs / s_act reused by the next env
}

// Reset-mode observation of S <= 4 envs, kObsResetEnvs envs per workgroup, one wave each (its own
// scratch; only wave-level ordering, so waves of envs outside the mask simply leave).  A masked
// reset (graph_mode's every-step auto-reset, or the eager one past max_steps) then dispatches B / 8
// workgroups instead of B: when few envs are done, the launch costs its dispatch, not B
// single-wave workgroups that each read one mask byte.
constexpr int kObsResetEnvs = 8;
static_assert(kObsResetEnvs * sizeof(ObsScratch) <= 65536, "default dynamic LDS limit");
template <bool FAC>
__global__ void __launch_bounds__(64 * kObsResetEnvs, 4)
    observe_reset_kernel(DevState st, SimParams p, ObsOutputs out, const uint8_t* reset_mask) {
  const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const size_t b = (size_t)blockIdx.x * kObsResetEnvs + (size_t)wv;
  if (b >= (size_t)p.B || (reset_mask != nullptr && reset_mask[b] == 0)) return;
  extern __shared__ double obs_dyn[];
  ObsScratch& sc = reinterpret_cast<ObsScratch*>(obs_dyn)[wv];
  __shared__ float s_obs[kObsResetEnvs][kObsChunk * NF];
  __shared__ float s_act[kObsResetEnvs][kObsChunk];
  observe_chunk<true, false>(st, p, b, 0, p.S, sc, s_obs[wv], lane);  // S <= kObsChunk: one chunk
  observe_outputs<kObsChunk, kModeReset, FAC>(st, p, out, b, s_obs[wv], s_act[wv], lane, 64);
}

}  // namespace lbk
