// lbsim_stateless.h — stateless entry-point kernels (no handle state): the observe / reward /
// alias routines of lbsim_kernels.h on caller-given inputs, problem-07's Vose tables and
// problem-05's per-agent observations.  Non-template kernels: included by lbsim_api.hip only.
#pragma once

#include "lbsim_kernels.h"

namespace lbk {

// ================================================================ stateless entry points

// Reservoir features of caller-given reservoirs: 4 reservoirs per block, each presented to
// observe_chunk as one "server" whose fct and duration arrays are both the given values.
__global__ void __launch_bounds__(64)
    features_kernel(const float* values, const uint32_t* ts, const uint32_t* counts, int64_t n,
                    float decay_c, float* out) {
  const int64_t r0 = (int64_t)blockIdx.x * 4;
  const int lane = threadIdx.x;
  __shared__ ObsScratch sc;
  __shared__ float fobs[4 * NF];
  const int S = (int)(n - r0 < 4 ? n - r0 : 4);
  DevState st{};
  st.feat_vals = reinterpret_cast<const uint32_t*>(values) + r0 * K;
  st.feat_ts = ts + r0 * K;
  st.res_count = const_cast<uint32_t*>(counts) + r0;
  __shared__ uint32_t hc0[4];
  if (lane < 4) hc0[lane] = 0;
  st.hc = hc0;
  SimParams p{};
  p.S = S;
  p.decay_c = decay_c;
  __syncthreads();
  observe_chunk<false, false>(st, p, 0, 0, S, sc, fobs, lane);
  for (int e = lane; e < S * 5; e += 64) {
    const int s = e / 5, f = e - s * 5;
    out[(r0 + s) * 5 + f] = fobs[s * NF + 1 + f];
  }
}

// ALIAS tables of caller-given weight rows, one lane per row (the per-step build of
// dynamics_kernel, exposed for the gen_alias parity test).
__global__ void __launch_bounds__(64)
    alias_tables_kernel(const float* weights, int64_t n, int S, float* odd_out,
                        int32_t* alias_out, int32_t* active_out) {
  __shared__ int32_t tabw[2 * MAX_S * 64];  // table words [f][k][lane]
  const int lane = (int)threadIdx.x;
  auto tab = [&](int f, int k) -> int32_t& { return tabw[(f * MAX_S + k) * 64 + lane]; };
  const int64_t r = (int64_t)blockIdx.x * 64 + threadIdx.x;
  if (r >= n) return;
  float w[MAX_S];
#pragma unroll
  for (int s = 0; s < MAX_S; ++s) w[s] = s < S ? weights[r * S + s] : 0.0f;
  const int na = build_alias<MAX_S>(w, S, tab);
  for (int k = 0; k < S; ++k) {
    const bool v = k < na;
    odd_out[r * S + k] = v ? __uint_as_float((uint32_t)tab(0, k)) : 1.0f;
    alias_out[r * S + k] = v ? (tab(1, k) & 0xFF) : 0;
    active_out[r * S + k] = v ? (tab(1, k) >> 8) : -1;
  }
}

// Vose alias tables of problem-07's VPP plugin (realtime-mode/problem-07-realtime-deployment/
// vpp-plugin/alias_table.h:82-158), one lane per row, in the float32 of the C: sequential sum,
// sum <= 0 (not NaN) -> identity table, prob_scaled = (f32)n * w / sum, small (< 1) / large
// stacks pushed in index order and popped from the top, the large's remainder (p_l + p_s) - 1
// (the C's double subtraction rounded to f32 is the correctly rounded f32 subtraction),
// leftovers (1, self).  prob_scaled and both stacks live in LDS [slot][lane].
__global__ void __launch_bounds__(64)
    vose_tables_kernel(const float* weights, int64_t n, int S, float* prob_out,
                       uint32_t* alias_out) {
  __shared__ float ps[MAX_S * 64];
  __shared__ uint8_t stk[2 * MAX_S * 64];  // small: [j][lane], large: [MAX_S + j][lane]
  const int lane = (int)threadIdx.x;
  const int64_t r = (int64_t)blockIdx.x * 64 + lane;
  if (r >= n) return;
  const float* w = weights + r * S;
  float* po = prob_out + r * S;
  uint32_t* ao = alias_out + r * S;
  float sum = 0.0f;
  for (int s = 0; s < S; ++s) sum = __fadd_rn(sum, w[s]);
  if (sum <= 0.0f) {
    for (int s = 0; s < S; ++s) { po[s] = 1.0f; ao[s] = (uint32_t)s; }
    return;
  }
  const float fn = (float)(uint32_t)S;
  auto small = [&](int j) -> uint8_t& { return stk[j * 64 + lane]; };
  auto large = [&](int j) -> uint8_t& { return stk[(MAX_S + j) * 64 + lane]; };
  int ns = 0, nl = 0;
  for (int s = 0; s < S; ++s) {
    const float p = __fdiv_rn(__fmul_rn(fn, w[s]), sum);
    ps[s * 64 + lane] = p;
    if (p < 1.0f) small(ns++) = (uint8_t)s;
    else large(nl++) = (uint8_t)s;
  }
  while (ns > 0 && nl > 0) {
    const int s = small(--ns), l = large(--nl);
    const float p_s = ps[s * 64 + lane];
    po[s] = p_s;
    ao[s] = (uint32_t)l;
    const float v = __fsub_rn(__fadd_rn(ps[l * 64 + lane], p_s), 1.0f);
    ps[l * 64 + lane] = v;
    if (v < 1.0f) small(ns++) = (uint8_t)l;
    else large(nl++) = (uint8_t)l;
  }
  while (ns > 0) { const int s = small(--ns); po[s] = 1.0f; ao[s] = (uint32_t)s; }
  while (nl > 0) { const int l = large(--nl); po[l] = 1.0f; ao[l] = (uint32_t)l; }
}

// alias_table_sample (alias_table.h:195-209) k times per table from the table's xorshift32
// state (:163-172): i = x1 % S, r = (f32)x2 / (f32)0xFFFFFFFF (= 2^32: an exact scaling), pick
// i if r < prob[i] else alias[i].  One lane per table; the histogram
// (alias_table_test_distribution, :221-237) in LDS [server][lane]; picks >= S (a malformed
// alias entry) are returned in idx_out but not counted.
__global__ void __launch_bounds__(64)
    vose_sample_kernel(const float* prob, const uint32_t* alias, int64_t n, int S,
                       uint32_t* state_io, int64_t k, int32_t* idx_out, uint64_t* hist_out) {
  __shared__ uint32_t hist[MAX_S * 64];
  const int lane = (int)threadIdx.x;
  const int64_t r = (int64_t)blockIdx.x * 64 + lane;
  if (r >= n) return;
  for (int s = 0; s < S; ++s) hist[s * 64 + lane] = 0;
  const float* p = prob + r * S;
  const uint32_t* a = alias + r * S;
  int32_t* io = idx_out ? idx_out + r * k : nullptr;
  uint32_t x = state_io[r];
  for (int64_t j = 0; j < k; ++j) {
    x ^= x << 13; x ^= x >> 17; x ^= x << 5;
    const uint32_t i = x % (uint32_t)S;
    x ^= x << 13; x ^= x >> 17; x ^= x << 5;
    const float u = __fmul_rn((float)x, 2.3283064365386962890625e-10f);
    const uint32_t pick = u < p[i] ? i : a[i];
    if (io) io[j] = (int32_t)pick;
    if (pick < (uint32_t)S) hist[pick * 64 + lane] += 1;
  }
  state_io[r] = x;
  if (hist_out)
    for (int s = 0; s < S; ++s) hist_out[r * S + s] = hist[s * 64 + lane];
}

// problem-05 per-agent observations (multi_agent_env.py:152-188) of n flattened (S, 11) obs:
// agent a sees 4-value slices of the flattened obs for its servers [a k, (a+1) k) -- flat
// [4 a k, 4 (a+1) k), the wrapper's `server_features_per_server = 4` -- followed by flat[4 S:].
__global__ void __launch_bounds__(256)
    agent_obs_kernel(const float* obs, int64_t n, int S, int A, int k, float* out) {
  const int D = 4 * k + 7 * S;
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n * A * D) return;
  const int64_t b = i / ((int64_t)A * D);
  const int r = (int)(i - b * A * D);
  const int a = r / D, j = r - a * D;
  const int src = j < 4 * k ? 4 * k * a + j : 4 * S + (j - 4 * k);
  out[i] = obs[b * S * NF + src];
}

__global__ void __launch_bounds__(256)
    reward_kernel(const float* obs, int64_t n, int S, int metric, int field, float* out) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  out[i] = (float)reward_of(obs + i * (int64_t)S * NF, S, metric, field);
}

}  // namespace lbk
