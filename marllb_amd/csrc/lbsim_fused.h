// lbsim_fused.h — one-kernel policy inference for the policy-in-the-loop rollouts (SURVEY §8f
// ranks 1-2, BASELINE configs[3] and configs[4]) on the f32-input MFMA of gfx950.
//
//   sac_actor_kernel   problem-04 PolicyNetwork.sample (networks.py:82-146): GRU(state -> H),
//                      fc1 -> F + ReLU, [fc_mean | fc_logstd] -> 2A, clamp, Philox noise, tanh.
//   qmix_policy_kernel problem-05 QMIXAgent.select_actions (qmix_agent.py:138-178) for all A agents
//                      (AgentQNetwork agent_network.py:63-87: GRU(obs -> H), fc1/fc2 -> F + ReLU,
//                      fc3 -> n_actions), epsilon-greedy, the chosen Q-values, then QMixingNetwork
//                      (mixing_network.py:78-117) on the global state -> Q_tot.
//
// One workgroup (4 waves) owns a tile of R = 16 MT envs for the whole network: activations never
// leave LDS ([R][ld] f32, ld = 4 mod 64 so the MFMA operand reads are bank-conflict free), weights
// stream from L2 in MFMA-fragment order, every GEMM is v_mfma_f32_16x16x4_f32 (exact f32 FMA
// chain, the same numerics class as the fp32 hipBLASLt path it replaces: tested to 1e-5 against
// the torch modules).  Per layer each wave accumulates its output tiles in registers, the
// workgroup barriers, then writes the activated tile back over its input (so one LDS buffer serves
// every layer).
//
// Packed weight layout (marllb_amd/policies.py `pack_linear`): a torch Linear weight W [N, K] is
// zero-padded to [16 NT, 16 KB] and stored as P[nt][kb][lane][s] = W[16 nt + (lane & 15)]
// [16 kb + 4 (lane >> 4) + s]: for k-step s of block kb, lane l feeds A[row l&15][k = l>>4] and
// B[k = l>>4][col l&15] of the 16x16x4 MFMA with the same permuted k, so one 16-B load per lane
// per block gives the B operands of four MFMAs and one ds_read_b128 per M-tile the A operands.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

#include "lbsim_math.h"

namespace lbk {

typedef float f4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ f4 splat4(float v) { return f4{v, v, v, v}; }

// Timing diagnostic only (wrong results): LBSIM_EXP_L1W=1 makes every k-block past the first two
// re-read one of the tile's first two weight blocks: fewer distinct weight bytes, the same stream
// of weight requests (a CU's ~24 waves' blocks still overflow its L1; profiles/r06k/).
#if LBSIM_EXP_L1W
#define LBSIM_EXP_WBLK(n) ((n) & 1)
#else
#define LBSIM_EXP_WBLK(n) (n)
#endif

// Timing diagnostic only (LBSIM_EXP_PHASES=1, pol.o of an A/B build): lane 0 of wave 0 of every
// gridDim / 64-th workgroup records the 100 MHz clock at the kernel's phase boundaries into
// lbsim_exp_ts[sample][phase] (read by lbsim_exp_phase_read, tools/policy_phases.py).
#if LBSIM_EXP_PHASES
__device__ unsigned long long lbsim_exp_ts[64 * 16];
#define LB_PHASE(i)                                                                        \
  do {                                                                                      \
    const unsigned st_ = gridDim.x >= 64u ? gridDim.x / 64u : 1u;                           \
    if (threadIdx.x == 0 && blockIdx.x % st_ == 0u && blockIdx.x / st_ < 64u)               \
      lbsim_exp_ts[(blockIdx.x / st_) * 16u + (i)] = __builtin_amdgcn_s_memrealtime();     \
  } while (0)
#else
#define LB_PHASE(i) \
  do {              \
  } while (0)
#endif

__device__ __forceinline__ float sigmoid_f(float x) { return 1.0f / (1.0f + expf(-x)); }

// acc[m] += X[rows 16m .. 16m+15, cols col0 .. col0 + 16 nkb) . W^T for one 16-column output tile
// whose packed k-blocks start at wp.  Software-pipelined: B fragments two blocks ahead (L2
// latency), A fragments one block ahead (LDS latency); the clamped tail re-reads the last block.
template <int MT>
__device__ __forceinline__ void mma_tile(f4 (&acc)[MT], const float* lds, int ld, int col0,
                                         const f4* __restrict__ wp, int nkb, int lane, f4 b0,
                                         f4 b1) {
  const float* arow = lds + (lane & 15) * ld + col0 + 4 * (lane >> 4);
  f4 a[MT];
#pragma unroll
  for (int m = 0; m < MT; ++m) a[m] = *(const f4*)(arow + m * 16 * ld);
  for (int kb = 0; kb < nkb; ++kb) {
    const int n2 = kb + 2 < nkb ? kb + 2 : nkb - 1;
    const int n1 = kb + 1 < nkb ? kb + 1 : nkb - 1;
    const f4 b2 = wp[LBSIM_EXP_WBLK(n2) * 64 + lane];
    f4 an[MT];
#pragma unroll
    for (int m = 0; m < MT; ++m) an[m] = *(const f4*)(arow + m * 16 * ld + n1 * 16);
#pragma unroll
    for (int s = 0; s < 4; ++s)
#pragma unroll
      for (int m = 0; m < MT; ++m)
        acc[m] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[m][s], b0[s], acc[m], 0, 0, 0);
#pragma unroll
    for (int m = 0; m < MT; ++m) a[m] = an[m];
    b0 = b1;
    b1 = b2;
  }
}
template <int MT>
__device__ __forceinline__ void mma_tile(f4 (&acc)[MT], const float* lds, int ld, int col0,
                                         const f4* __restrict__ wp, int nkb, int lane) {
  mma_tile<MT>(acc, lds, ld, col0, wp, nkb, lane, wp[lane], wp[(nkb > 1 ? 64 : 0) + lane]);
}

// The first two k-blocks' B fragments of NB tiles, loaded ahead of mma_multi: a caller issues
// them before the barrier that precedes the layer, so their L2 latency overlaps the wait.
template <int NB>
struct BPrime {
  f4 b0[NB], b1[NB];
};
template <int NB>
__device__ __forceinline__ BPrime<NB> mma_prime(const f4* const (&wp)[NB], int nkb, int lane) {
  BPrime<NB> bp;
#pragma unroll
  for (int j = 0; j < NB; ++j) {
    bp.b0[j] = wp[j][lane];
    bp.b1[j] = wp[j][(nkb > 1 ? 64 : 0) + lane];
  }
  return bp;
}

// NB output tiles over the same input columns in one pipelined loop: the A fragments are read
// once per block for all of them, and NB x MT independent accumulator chains keep the MFMA pipe
// busy even at MT = 1 (a single chain waits out the 40-cycle dependent latency every MFMA).
template <int MT, int NB>
__device__ __forceinline__ void mma_multi(f4 (&acc)[NB][MT], const float* lds, int ld, int col0,
                                          const f4* const (&wp)[NB], int nkb, int lane,
                                          const BPrime<NB>& bp) {
  const float* arow = lds + (lane & 15) * ld + col0 + 4 * (lane >> 4);
  f4 b0[NB], b1[NB];
#pragma unroll
  for (int j = 0; j < NB; ++j) {
    b0[j] = bp.b0[j];
    b1[j] = bp.b1[j];
  }
  f4 a[MT];
#pragma unroll
  for (int m = 0; m < MT; ++m) a[m] = *(const f4*)(arow + m * 16 * ld);
  for (int kb = 0; kb < nkb; ++kb) {
    const int n2 = kb + 2 < nkb ? kb + 2 : nkb - 1;
    const int n1 = kb + 1 < nkb ? kb + 1 : nkb - 1;
    f4 b2[NB];
#pragma unroll
    for (int j = 0; j < NB; ++j) b2[j] = wp[j][LBSIM_EXP_WBLK(n2) * 64 + lane];
    f4 an[MT];
#pragma unroll
    for (int m = 0; m < MT; ++m) an[m] = *(const f4*)(arow + m * 16 * ld + n1 * 16);
#pragma unroll
    for (int s = 0; s < 4; ++s)
#pragma unroll
      for (int j = 0; j < NB; ++j)
#pragma unroll
        for (int m = 0; m < MT; ++m)
          acc[j][m] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[m][s], b0[j][s], acc[j][m], 0, 0, 0);
#pragma unroll
    for (int m = 0; m < MT; ++m) a[m] = an[m];
#pragma unroll
    for (int j = 0; j < NB; ++j) {
      b0[j] = b1[j];
      b1[j] = b2[j];
    }
  }
}
template <int MT, int NB>
__device__ __forceinline__ void mma_multi(f4 (&acc)[NB][MT], const float* lds, int ld, int col0,
                                          const f4* const (&wp)[NB], int nkb, int lane) {
  mma_multi<MT, NB>(acc, lds, ld, col0, wp, nkb, lane, mma_prime<NB>(wp, nkb, lane));
}

// Dense layer, accumulate phase: wave w owns output tiles nt = w, w + WS, ... < ntiles (WS = the
// waves sharing the layer), all in one mma_multi pass (a wave with fewer tiles recomputes the last
// one; dense_store skips it).
template <int MT, int NTW, int WS = 4>
__device__ __forceinline__ void dense_acc(f4 (&acc)[NTW][MT], const float* lds, int ld, int col0,
                                          const float* __restrict__ w, int nkb, int ntiles,
                                          const float* __restrict__ bias, int wave, int lane) {
  const f4* wp[NTW];
#pragma unroll
  for (int j = 0; j < NTW; ++j) {
    const int nt = wave + WS * j < ntiles ? wave + WS * j : ntiles - 1;
    wp[j] = (const f4*)w + (size_t)nt * nkb * 64;
    const float bv = bias[nt * 16 + (lane & 15)];
#pragma unroll
    for (int m = 0; m < MT; ++m) acc[j][m] = splat4(bv);
  }
  mma_multi<MT, NTW>(acc, lds, ld, col0, wp, nkb, lane);
}

// A narrow output (<= 2 tiles: the SAC heads, the Q-values) with K split over the 4 waves: wave w
// runs the k-blocks [w nkb / 4, (w + 1) nkb / 4) of every M-tile, the partial tiles meet in LDS
// scratch ([4][nt][R][16]) and the workgroup sums them: dst[r * dld + c] = bias[c] + sum, c <
// ncols.  Contains a barrier; the caller barriers again before reading dst.
template <int MT>
__device__ __forceinline__ void splitk_out(const float* lds, int ld, const float* __restrict__ w,
                                           const float* __restrict__ bias, int nkb, int nt,
                                           float* scratch, float* dst, int dld, int ncols,
                                           int wave, int lane) {
  constexpr int R = 16 * MT;
  const int k0 = wave * nkb / 4, k1 = (wave + 1) * nkb / 4;
  for (int t = 0; t < nt; ++t) {
    f4 acc[MT];
#pragma unroll
    for (int m = 0; m < MT; ++m) acc[m] = splat4(0.0f);
    if (k1 > k0)
      mma_tile<MT>(acc, lds, ld, k0 * 16, (const f4*)w + ((size_t)t * nkb + k0) * 64, k1 - k0,
                   lane);
#pragma unroll
    for (int m = 0; m < MT; ++m)
#pragma unroll
      for (int i = 0; i < 4; ++i)
        scratch[((wave * nt + t) * R + m * 16 + 4 * (lane >> 4) + i) * 16 + (lane & 15)] =
            acc[m][i];
  }
  __syncthreads();
  for (int e = threadIdx.x; e < R * ncols; e += blockDim.x) {
    const int r = e / ncols, c = e - r * ncols, t = c >> 4, cc = c & 15;
    float v = bias[c];
#pragma unroll
    for (int q = 0; q < 4; ++q) v += scratch[((q * nt + t) * R + r) * 16 + cc];
    dst[r * dld + c] = v;
  }
}

// splitk_out for a 32-row tile (MT = 2): wave w runs M-tile w >> 1 over the k-blocks of half
// (w & 1), so the scratch holds two partials per row ([2][nt][32][16]) instead of four -- the
// SAC tile's LDS is then 37.4 KB, four workgroups per CU where the four-partial scratch (41.5 KB)
// fit three (LBSIM_SAC_SPLIT_M).  Contains a barrier; the caller barriers again before reading dst.
__device__ __forceinline__ void splitk_out_m2(const float* lds, int ld, const float* __restrict__ w,
                                              const float* __restrict__ bias, int nkb, int nt,
                                              float* scratch, float* dst, int dld, int ncols,
                                              int wave, int lane) {
  constexpr int R = 32;
  const int m = wave >> 1, kh = wave & 1;
  const int k0 = kh * nkb / 2, k1 = (kh + 1) * nkb / 2;
  for (int t = 0; t < nt; ++t) {
    f4 acc[1] = {splat4(0.0f)};
    if (k1 > k0)
      mma_tile<1>(acc, lds + m * 16 * ld, ld, k0 * 16, (const f4*)w + ((size_t)t * nkb + k0) * 64,
                  k1 - k0, lane);
#pragma unroll
    for (int i = 0; i < 4; ++i)
      scratch[((kh * nt + t) * R + m * 16 + 4 * (lane >> 4) + i) * 16 + (lane & 15)] = acc[0][i];
  }
  __syncthreads();
  for (int e = threadIdx.x; e < R * ncols; e += blockDim.x) {
    const int r = e / ncols, c = e - r * ncols, t = c >> 4, cc = c & 15;
    float v = bias[c];
#pragma unroll
    for (int q = 0; q < 2; ++q) v += scratch[((q * nt + t) * R + r) * 16 + cc];
    dst[r * dld + c] = v;
  }
}

// Dense layer, store phase (after a barrier): out[row][col0 + 16 nt + c] = act(acc, 16 nt + c).
template <int MT, int NTW, class Act, int WS = 4>
__device__ __forceinline__ void dense_store(const f4 (&acc)[NTW][MT], float* lds, int ld, int col0,
                                            int ntiles, int wave, int lane, Act act) {
#pragma unroll
  for (int j = 0; j < NTW; ++j) {
    const int nt = wave + WS * j;
    if (nt < ntiles) {
      const int c = nt * 16 + (lane & 15);
#pragma unroll
      for (int m = 0; m < MT; ++m)
#pragma unroll
        for (int i = 0; i < 4; ++i)
          lds[(m * 16 + 4 * (lane >> 4) + i) * ld + col0 + c] = act(acc[j][m][i], c);
    }
  }
}

// torch.nn.GRU cell over the tile (gate order r, z, n):
//   r = sig(x W_ir + b_ir + h W_hr + b_hr), z likewise, n = tanh(x W_in + b_in + r (h W_hn + b_hn)),
//   h' = (1 - z) n + z h,
// with x in LDS cols [0, kxp) and h in [kxp, kxp + H).  Returns h' of the wave's unit tiles in
// hn (wave w: unit tiles u = w, w + 4, ...); the caller barriers before overwriting h.
template <int MT, int H>
__device__ __forceinline__ void gru_tile(f4 (&hn)[(H / 16 + 3) / 4][MT], const float* lds, int ld,
                                         int kxp, const float* __restrict__ w_ih,
                                         const float* __restrict__ w_hh,
                                         const float* __restrict__ b_ih,
                                         const float* __restrict__ b_hh, int wave, int lane) {
  constexpr int UT = H / 16, UTW = (UT + 3) / 4, KBH = H / 16;
  const int kbx = kxp / 16;
  const f4* wi = (const f4*)w_ih;
  const f4* wh = (const f4*)w_hh;
#pragma unroll
  for (int j = 0; j < UTW; ++j) {
    const int u = wave + 4 * j;
    if (u >= UT) continue;
    const int col = u * 16 + (lane & 15);
    // g = {x W_in + b_in, r, z, h W_hn + b_hn}: the input part feeds g[0..2], the hidden part
    // g[1..3], each in one mma_multi pass sharing its A fragments
    f4 g[4][MT];
    const float bg[4] = {b_ih[2 * H + col], b_ih[col] + b_hh[col], b_ih[H + col] + b_hh[H + col],
                         b_hh[2 * H + col]};
#pragma unroll
    for (int q = 0; q < 4; ++q)
#pragma unroll
      for (int m = 0; m < MT; ++m) g[q][m] = splat4(bg[q]);
    const f4* const wx[3] = {wi + (size_t)(2 * UT + u) * kbx * 64, wi + (size_t)u * kbx * 64,
                             wi + (size_t)(UT + u) * kbx * 64};
    const f4* const wy[3] = {wh + (size_t)u * KBH * 64, wh + (size_t)(UT + u) * KBH * 64,
                             wh + (size_t)(2 * UT + u) * KBH * 64};
    mma_multi<MT, 3>(*reinterpret_cast<f4(*)[3][MT]>(&g[0]), lds, ld, 0, wx, kbx, lane);
    mma_multi<MT, 3>(*reinterpret_cast<f4(*)[3][MT]>(&g[1]), lds, ld, kxp, wy, KBH, lane);
#pragma unroll
    for (int m = 0; m < MT; ++m)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const float hp = lds[(m * 16 + 4 * (lane >> 4) + i) * ld + kxp + col];
        const float r = sigmoid_f(g[1][m][i]);
        const float z = sigmoid_f(g[2][m][i]);
        const float n = tanhf(g[0][m][i] + r * g[3][m][i]);
        hn[j][m][i] = (1.0f - z) * n + z * hp;
      }
  }
}

// Store h' into LDS cols [kxp, kxp + H) and to hidden[b, H] (row stride h_ld floats).
template <int MT, int H>
__device__ __forceinline__ void gru_store(const f4 (&hn)[(H / 16 + 3) / 4][MT], float* lds, int ld,
                                          int kxp, float* hidden, int64_t h_ld, int64_t row0,
                                          int64_t B, int wave, int lane) {
  constexpr int UT = H / 16, UTW = (UT + 3) / 4;
#pragma unroll
  for (int j = 0; j < UTW; ++j) {
    const int u = wave + 4 * j;
    if (u >= UT) continue;
    const int col = u * 16 + (lane & 15);
#pragma unroll
    for (int m = 0; m < MT; ++m)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int r = m * 16 + 4 * (lane >> 4) + i;
        lds[r * ld + kxp + col] = hn[j][m][i];
        if (row0 + r < B) hidden[(row0 + r) * h_ld + col] = hn[j][m][i];
      }
  }
}

// Stage rows [row0, row0 + R) of a [B, n] matrix (row stride src_ld) into LDS cols [col0, col0 +
// npad), zero past n, past B and (if reset_mask) for rows whose mask byte is set.  Eight elements
// per thread per pass: the eight values are loaded from clamped in-range addresses with no
// condition, then the eight mask bytes, and only then selected, so the sixteen loads are in flight
// together (a load behind each row's mask byte waited for every earlier load: one HBM round trip
// per element instead of one per pass, profiles/r06n/).
__device__ __forceinline__ void stage_rows(float* lds, int ld, int col0, const float* src,
                                           int64_t src_ld, int n, int npad, int R, int64_t row0,
                                           int64_t B, const uint8_t* reset_mask) {
  const int total = R * npad, nthr = (int)blockDim.x;
  for (int e0 = (int)threadIdx.x; e0 < total; e0 += 8 * nthr) {
    float v[8];
    int at[8];
    int64_t bc[8];
    bool ok[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int e = e0 + i * nthr;
      const int r = e / npad, c = e - r * npad;
      const int64_t b = row0 + r;
      at[i] = e < total ? r * ld + col0 + c : -1;
      ok[i] = e < total && c < n && b < B;
      bc[i] = b < B ? b : B - 1;
      v[i] = src[bc[i] * src_ld + (ok[i] ? c : 0)];
    }
    if (reset_mask != nullptr) {
      uint8_t m[8];
#pragma unroll
      for (int i = 0; i < 8; ++i) m[i] = reset_mask[bc[i]];
#pragma unroll
      for (int i = 0; i < 8; ++i) ok[i] = ok[i] && m[i] == 0;
    }
#pragma unroll
    for (int i = 0; i < 8; ++i)
      if (at[i] >= 0) lds[at[i]] = ok[i] ? v[i] : 0.0f;
  }
}

struct ReluAct {
  __device__ float operator()(float v, int) const { return v > 0.0f ? v : 0.0f; }
};

// ------------------------------------------------------------------------------ SAC-GRU actor
struct SacActorArgs {
  const float* state;     // [B, I]
  float* hidden;          // [B, H], updated in place
  const uint8_t* reset;   // [B] or null: rows whose hidden state starts from zero
  const float *w_ih, *w_hh, *b_ih, *b_hh, *w1, *b1, *wh, *bh;
  float* action;          // [B, A]
  float* log_std;         // [B, A] or null
  int64_t B;
  int I, kxp, ld, A;
  float lo, hi, scale, bias;
  int deterministic;
  uint32_t key0, key1, step;
  const uint32_t* step_dev;  // when set, the Philox step counter is *step_dev (graph replays)
};

// The SAC tile's input rows in one pass with no index division: thread t < kxp stages state
// column t, kxp <= t < kxp + H hidden column t - kxp, each for all R rows.  Every row's value is
// loaded from a clamped in-range address with no condition, then (hidden columns) every row's
// reset byte, then the selects: the R + R loads are in flight together.  (Loading each hidden value
// behind its row's reset byte made every byte load wait for all earlier loads -- R HBM round trips,
// 20 of a workgroup's 67 us, profiles/r06m/.)
template <int R, int H>
__device__ __forceinline__ void stage_sac_rows(float* lds, const SacActorArgs& p, int64_t row0) {
  const int t = threadIdx.x, kxp = p.kxp, ld = p.ld;
#if LBSIM_EXP_NOSTAGE  // timing diagnostic (wrong results): no HBM reads in the staging
  for (int c = t; c < kxp + H; c += blockDim.x)
    for (int r = 0; r < R; ++r) lds[r * ld + c] = 0.01f * (float)c;
  return;
#endif
  for (int c = t; c < kxp + H; c += blockDim.x) {
    const bool st = c < kxp;
    const bool col_ok = !st || c < p.I;
    const float* src = st ? p.state + (col_ok ? c : 0) : p.hidden + (c - kxp);
    const int64_t stride = st ? p.I : H;
    int64_t bc[R];
    float v[R];
#pragma unroll
    for (int r = 0; r < R; ++r) {
      const int64_t b = row0 + r;
      bc[r] = b < p.B ? b : p.B - 1;
      v[r] = src[bc[r] * stride];
    }
    bool keep[R];
#pragma unroll
    for (int r = 0; r < R; ++r) keep[r] = col_ok && row0 + r < p.B;
    if (!st && p.reset != nullptr) {
      uint8_t m[R];
#pragma unroll
      for (int r = 0; r < R; ++r) m[r] = p.reset[bc[r]];
#pragma unroll
      for (int r = 0; r < R; ++r) keep[r] = keep[r] && m[r] == 0;
    }
#pragma unroll
    for (int r = 0; r < R; ++r) lds[r * ld + c] = keep[r] ? v[r] : 0.0f;
  }
}

#ifndef LBSIM_SAC_WPE
#define LBSIM_SAC_WPE 1
#endif
// 1: the 32-env SAC tile's heads split their K over 2 waves per M-tile (splitk_out_m2), the LDS
// scratch halved (lbsim_api.hip sac_lds_bytes must agree)
#ifndef LBSIM_SAC_SPLIT_M
#define LBSIM_SAC_SPLIT_M 1
#endif

template <int MT, int H, int F>
__global__ void __launch_bounds__(256, LBSIM_SAC_WPE) sac_actor_kernel(SacActorArgs p) {
  const uint32_t step = p.step_dev != nullptr ? *p.step_dev : p.step;
  extern __shared__ float lds[];
  constexpr int R = 16 * MT;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int64_t row0 = (int64_t)blockIdx.x * R;
  const int ld = p.ld, kxp = p.kxp;
  LB_PHASE(0);
#if LBSIM_SAC_OLD_STAGE
  stage_rows(lds, ld, 0, p.state, p.I, p.I, kxp, R, row0, p.B, nullptr);
  stage_rows(lds, ld, kxp, p.hidden, H, H, H, R, row0, p.B, p.reset);
#else
  stage_sac_rows<R, H>(lds, p, row0);
#endif
  LB_PHASE(1);
  __syncthreads();
  LB_PHASE(2);
  {
    f4 hn[(H / 16 + 3) / 4][MT];
    gru_tile<MT, H>(hn, lds, ld, kxp, p.w_ih, p.w_hh, p.b_ih, p.b_hh, wave, lane);
    LB_PHASE(3);
    __syncthreads();
    gru_store<MT, H>(hn, lds, ld, kxp, p.hidden, H, row0, p.B, wave, lane);
  }
  __syncthreads();
  LB_PHASE(4);
  {
    constexpr int NT = F / 16, NTW = (NT + 3) / 4;
    f4 acc[NTW][MT];
    dense_acc<MT, NTW>(acc, lds, ld, kxp, p.w1, H / 16, NT, p.b1, wave, lane);
    LB_PHASE(5);
    __syncthreads();
    dense_store<MT, NTW>(acc, lds, ld, 0, NT, wave, lane, ReluAct{});
  }
  __syncthreads();
  LB_PHASE(6);
  // heads [mean | log_std] (2A <= 32 columns), K split over the waves; y over the first 2A
  // columns of the tile
  if constexpr (MT == 2 && LBSIM_SAC_SPLIT_M)
    splitk_out_m2(lds, ld, p.wh, p.bh, F / 16, (2 * p.A + 15) / 16, lds + R * ld, lds, ld,
                  2 * p.A, wave, lane);
  else
    splitk_out<MT>(lds, ld, p.wh, p.bh, F / 16, (2 * p.A + 15) / 16, lds + R * ld, lds, ld,
                   2 * p.A, wave, lane);
  __syncthreads();
  LB_PHASE(7);
  const int A = p.A;
  for (int e = threadIdx.x; e < R * A; e += blockDim.x) {
    const int r = e / A, a = e - r * A;
    const int64_t b = row0 + r;
    if (b >= p.B) continue;
    const float mean = lds[r * ld + a];
    float ls = lds[r * ld + A + a];
    ls = ls < p.lo ? p.lo : (ls > p.hi ? p.hi : ls);
    float x = mean;
    if (!p.deterministic) {  // the noise of sac_head_kernel (lbsim_nets.h), same counter
      const u32x4 d = philox4x32_10(u32x4{(uint32_t)b, step, (uint32_t)a, 3u << 24}, p.key0,
                                    p.key1);
      const float u1 = u01_open0(d.x), u2 = (float)(d.y >> 8) * 5.9604644775390625e-8f;
      const float eps = sqrtf(-2.0f * logf(u1)) * cospif(2.0f * u2);
      x = mean + expf(ls) * eps;
    }
    p.action[b * A + a] = tanhf(x) * p.scale + p.bias;
    if (p.log_std) p.log_std[b * A + a] = ls;
  }
  LB_PHASE(8);
}

// ------------------------------------------------------------------------------ QMIX policy
struct QmixArgs {
  const float* obs;       // [B, A, I]
  float* hidden;          // [B, A, H], updated in place
  const uint8_t* reset;   // [B] or null
  const float* state;     // [B, Ds]
  // agent networks, A stacked copies each: packed weights and padded biases
  const float *w_ih, *w_hh, *b_ih, *b_hh, *w1, *b1, *w2, *b2, *w3, *b3;
  // mixer: first layers [hyper_w1[0] | hyper_w2[0] | hyper_b2[0] | hyper_b1] (3 he + E rows),
  // second layers hyper_w1[2] (A E x he), hyper_w2[2] (E x he), hyper_b2[2] (1 x he, padded)
  const float *m0, *mb0, *mw1, *mbw1, *mw2, *mbw2, *mb2, *mbb2;
  int64_t* actions;         // [B, A]
  int32_t* server_actions;  // [B, A k] or null: each agent's action repeated for its k servers
  float* q_out;             // [B, A, n_actions] or null
  float* q_chosen;          // [B, A] or null
  float* q_tot;             // [B]
  int64_t B;
  int A, I, kxp, Ds, ksp, ld, n_act, k, he, E;
  int lda;  // qmix_agent_wave_kernel: row stride of a wave's own [16][lda] agent region
  int sld;  // qmix_agent_pair_kernel: row stride of its prefetched [16][sld] state rows
  float epsilon;
  uint32_t key0, key1, step;
  const uint32_t* step_dev;  // when set, the Philox step counter is *step_dev (graph replays)
};

struct QmixMixAct {
  int relu_cols;  // columns [0, relu_cols) are ReLU'd (the three hypernetwork hidden layers)
  __device__ float operator()(float v, int c) const {
    return c < relu_cols ? (v > 0.0f ? v : 0.0f) : v;
  }
};

// QMixingNetwork.forward (mixing_network.py:78-117) of the tile, by the workgroup's NW waves (4:
// qmix_policy_kernel / the wave kernel, 8: the pair kernel), after the agents: chosen[R][A] holds
// the chosen Q-values; the LDS tile [R][p.ld] is free.
// pre: the state rows already staged (qmix_agent_pair_kernel loads them at its start, so their
// HBM latency hides behind the agents), [R][pre_ld]; else they are staged here.
// With 8 waves (round 6, profiles/r06n/): every wave takes part in both GEMM layers (2 first-layer
// tiles, <= 2 second-layer tiles each instead of 4 / 3 on waves 0-3), the second layer's first
// weight blocks are requested before the first layer's barrier, and the ELU tail runs one thread
// per (row, embedding unit) with a 32-lane sum (it ran 4 threads per row on one wave: 4.1 us).
#ifndef LBSIM_MIX_PRIME
#define LBSIM_MIX_PRIME 1
#endif
// 1: the pair kernel's epsilon-greedy inside the mixer's first layer (no barrier of its own)
#ifndef LBSIM_QMIX_EPS_IN_MIXER
#define LBSIM_QMIX_EPS_IN_MIXER 1
#endif
// 1: the pair kernel's obs rows loaded straight into LDS and waited for after the GRU's hidden
// pass, which then runs first (see qmix_agent_pair_kernel)
#ifndef LBSIM_QMIX_ASYNC_OBS
#define LBSIM_QMIX_ASYNC_OBS 1
#endif
// 1: the pair kernel's first GRU weights requested after its staging loads (A/B)
#ifndef LBSIM_QMIX_PRIME_LATE
#define LBSIM_QMIX_PRIME_LATE 0
#endif
// waves per SIMD the pair kernel is built for: 4 = two 8-wave workgroups per CU (<= 128 VGPRs)
#ifndef LBSIM_QMIX_PAIR_WPE
#define LBSIM_QMIX_PAIR_WPE 4
#endif
#ifndef LBSIM_MIX_NW
#define LBSIM_MIX_NW 8
#endif
#ifndef LBSIM_MIX_TAIL
#define LBSIM_MIX_TAIL 1
#endif
struct NoOp {
  __device__ void operator()() const {}
};
template <int MT, int NW = 4, class Pre1 = NoOp>
__device__ __forceinline__ void qmix_mixer(const QmixArgs& p, float* lds, const float* chosen,
                                           int64_t row0, int wave, int lane,
                                           const float* pre = nullptr, int pre_ld = 0,
                                           Pre1 pre1 = NoOp{}) {
  static_assert(NW == 4 || NW == 8, "4- or 8-wave workgroups");
  constexpr int R = 16 * MT;
  constexpr int J1 = 16 / NW;  // first-layer tiles per wave (3 he + E <= 256 columns)
  constexpr int J2 = 16 / NW;  // second-layer tiles per wave (A E + E + 16 <= 256 columns)
  const int ld = p.ld, A = p.A;
  if (pre == nullptr) {
    stage_rows(lds, ld, 0, p.state, p.Ds, p.Ds, p.ksp, R, row0, p.B, nullptr);
    __syncthreads();
  }
  const float* x0 = pre != nullptr ? pre : lds;
  const int x0_ld = pre != nullptr ? pre_ld : ld;
  const int he = p.he, E = p.E;
  const bool mw = wave < NW;  // the mixer's GEMM waves (a larger workgroup's others only meet
                              // the barriers)
  // second layers: w1 tiles (A E / 16) from cols [0, he), w2 tiles (E / 16) from [he, 2 he),
  // b2 (one tile) from [2 he, 3 he); outputs to cols [0, A E), [A E, A E + E), A E + E
  const int n1 = A * E / 16, n2 = E / 16, ntot = n1 + n2 + 1, kb = he / 16;
  const f4* w2p[J2];
  const float* b2p[J2];
  int c2[J2];
  f4 pb0[J2], pb1[J2];
#pragma unroll
  for (int j = 0; j < J2; ++j) {
    const int t0 = wave + NW * j, t = t0 < ntot ? t0 : ntot - 1;
    const float* w;
    if (t < n1) {
      w = p.mw1, b2p[j] = p.mbw1, c2[j] = 0;
    } else if (t < n1 + n2) {
      w = p.mw2, b2p[j] = p.mbw2, c2[j] = he;
    } else {
      w = p.mb2, b2p[j] = p.mbb2, c2[j] = 2 * he;
    }
    const int tt = t < n1 ? t : (t < n1 + n2 ? t - n1 : 0);
    w2p[j] = (const f4*)w + (size_t)tt * kb * 64;
    b2p[j] += tt * 16;
    if (NW == 8 && LBSIM_MIX_PRIME && mw) {  // requested now: their latency hides behind the first layer
      pb0[j] = w2p[j][lane];
      pb1[j] = w2p[j][(kb > 1 ? 64 : 0) + lane];
    }
  }
  {
    const int nt0 = (3 * he + E) / 16;  // <= 16
    f4 acc[J1][MT];
    if (mw) dense_acc<MT, J1, NW>(acc, x0, x0_ld, 0, p.m0, p.ksp / 16, nt0, p.mb0, wave, lane);
    pre1();  // (the pair kernel's epsilon-greedy: chosen is read by the tail only)
    __syncthreads();
    if (mw) dense_store<MT, J1, QmixMixAct, NW>(acc, lds, ld, 0, nt0, wave, lane, QmixMixAct{3 * he});
  }
  __syncthreads();
  LB_PHASE(9);
  {
    f4 acc[J2][MT];
#pragma unroll
    for (int j = 0; j < J2; ++j) {
      const int t = wave + NW * j;
      if (!mw || t >= ntot) continue;
      const float bv = b2p[j][lane & 15];
#pragma unroll
      for (int m = 0; m < MT; ++m) acc[j][m] = splat4(bv);
      if (NW == 8 && LBSIM_MIX_PRIME)
        mma_tile<MT>(acc[j], lds, ld, c2[j], w2p[j], kb, lane, pb0[j], pb1[j]);
      else
        mma_tile<MT>(acc[j], lds, ld, c2[j], w2p[j], kb, lane);
    }
    __syncthreads();
#pragma unroll
    for (int j = 0; j < J2; ++j) {
      const int t = wave + NW * j;
      if (!mw || t >= ntot) continue;
      const bool is_abs = t < n1 + n2;  // |W1|, |W2| (mixing_network.py:96,105)
      const int c = t * 16 + (lane & 15);
#pragma unroll
      for (int m = 0; m < MT; ++m)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const float v = acc[j][m][i];
          lds[(m * 16 + 4 * (lane >> 4) + i) * ld + c] = is_abs ? fabsf(v) : v;
        }
    }
  }
  __syncthreads();
  LB_PHASE(10);
  // tail: hidden_e = elu(b1_e + sum_a q_a |w1[a E + e]|), Q_tot = sum_e hidden_e |w2_e| + b2
  const int b1c = 3 * he, w2c = A * E, b2c = A * E + E;
  if (LBSIM_MIX_TAIL && NW * 64 == R * 32 && E == 32) {
    // one thread per (row, unit): rows r = tid / 32 of the wave's two halves, a 32-lane sum
    const int r = (int)threadIdx.x >> 5, u = (int)threadIdx.x & 31;
    const float* row = lds + r * ld;
    float h = 0.0f;
    for (int a = 0; a < A; ++a) h += chosen[r * A + a] * row[a * E + u];
    h += row[b1c + u];
    h = h > 0.0f ? h : expm1f(h);
    float acc = h * row[w2c + u];
    acc += __shfl_xor(acc, 16);
    acc += __shfl_xor(acc, 8);
    acc += __shfl_xor(acc, 4);
    acc += __shfl_xor(acc, 2);
    acc += __shfl_xor(acc, 1);
    if (u == 0 && row0 + r < p.B) p.q_tot[row0 + r] = acc + row[b2c];
    return;
  }
  // 4 threads per row, E / 4 embedding units each, combined by shuffles (R * 4 is a multiple of
  // 64, so every wave is either fully inside the loop or fully outside it)
  for (int e0 = threadIdx.x; e0 < R * 4; e0 += blockDim.x) {
    const int r = e0 >> 2, part = e0 & 3;
    const float* row = lds + r * ld;
    float acc = 0.0f;
    for (int u = part * (E / 4); u < (part + 1) * (E / 4); ++u) {
      float h = 0.0f;
      for (int a = 0; a < A; ++a) h += chosen[r * A + a] * row[a * E + u];
      h += row[b1c + u];
      h = h > 0.0f ? h : expm1f(h);
      acc += h * row[w2c + u];
    }
    acc += __shfl_xor(acc, 1);
    acc += __shfl_xor(acc, 2);
    if (part == 0 && row0 + r < p.B) p.q_tot[row0 + r] = acc + row[b2c];
  }
}

template <int MT, int H, int F>
__global__ void __launch_bounds__(256) qmix_policy_kernel(QmixArgs p) {
  const uint32_t step = p.step_dev != nullptr ? *p.step_dev : p.step;
  extern __shared__ float lds[];
  constexpr int R = 16 * MT;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int64_t row0 = (int64_t)blockIdx.x * R;
  const int ld = p.ld, kxp = p.kxp, A = p.A, NQ = p.n_act;
  float* qv = lds + R * ld;         // [A][R][16]
  float* chosen = qv + A * R * 16;  // [R][A]
  float* scratch = chosen + R * A;  // [4][R][16] split-K partials
  const size_t s_ih = (size_t)3 * H * kxp, s_hh = (size_t)3 * H * H;
  constexpr int NT = F / 16, NTW = (NT + 3) / 4;
  for (int a = 0; a < A; ++a) {
    stage_rows(lds, ld, 0, p.obs + (size_t)a * p.I, (int64_t)A * p.I, p.I, kxp, R, row0, p.B,
               nullptr);
    stage_rows(lds, ld, kxp, p.hidden + (size_t)a * H, (int64_t)A * H, H, H, R, row0, p.B,
               p.reset);
    __syncthreads();
    {
      f4 hn[(H / 16 + 3) / 4][MT];
      gru_tile<MT, H>(hn, lds, ld, kxp, p.w_ih + a * s_ih, p.w_hh + a * s_hh,
                      p.b_ih + a * 3 * H, p.b_hh + a * 3 * H, wave, lane);
      __syncthreads();
      gru_store<MT, H>(hn, lds, ld, kxp, p.hidden + (size_t)a * H, (int64_t)A * H, row0, p.B,
                       wave, lane);
    }
    __syncthreads();
    {
      f4 acc[NTW][MT];
      dense_acc<MT, NTW>(acc, lds, ld, kxp, p.w1 + (size_t)a * F * H, H / 16, NT, p.b1 + a * F,
                         wave, lane);
      __syncthreads();
      dense_store<MT, NTW>(acc, lds, ld, 0, NT, wave, lane, ReluAct{});
    }
    __syncthreads();
    {
      f4 acc[NTW][MT];
      dense_acc<MT, NTW>(acc, lds, ld, 0, p.w2 + (size_t)a * F * F, F / 16, NT, p.b2 + a * F,
                         wave, lane);
      __syncthreads();
      dense_store<MT, NTW>(acc, lds, ld, 0, NT, wave, lane, ReluAct{});
    }
    __syncthreads();
    // fc3 -> Q-values (n_actions <= 16: one output tile), K split over the waves
    splitk_out<MT>(lds, ld, p.w3 + (size_t)a * 16 * F, p.b3 + a * 16, F / 16, 1, scratch,
                   qv + a * R * 16, 16, 16, wave, lane);
    __syncthreads();
  }
  // epsilon-greedy (qmix_agent.py:153-164): argmax (first maximum, as torch.argmax), explore with
  // probability epsilon to a uniform action; Philox counter (row, step, agent, 4 << 24)
  for (int e = threadIdx.x; e < R * A; e += blockDim.x) {
    const int r = e / A, a = e - r * A;
    const int64_t b = row0 + r;
    const float* q = qv + (a * R + r) * 16;
    int g = 0;
    for (int j = 1; j < NQ; ++j)
      if (q[j] > q[g]) g = j;
    const u32x4 d = philox4x32_10(u32x4{(uint32_t)b, step, (uint32_t)a, 4u << 24}, p.key0,
                                  p.key1);
    const float u = (float)(d.x >> 8) * 5.9604644775390625e-8f;  // [0, 1)
    const int act = u < p.epsilon ? (int)(((uint64_t)d.y * (uint32_t)NQ) >> 32) : g;
    chosen[r * A + a] = q[act];
    if (b < p.B) {
      p.actions[b * A + a] = act;
      if (p.server_actions)
        for (int j = 0; j < p.k; ++j) p.server_actions[(b * A + a) * p.k + j] = act;
      if (p.q_out)
        for (int j = 0; j < NQ; ++j) p.q_out[(b * A + a) * NQ + j] = q[j];
      if (p.q_chosen) p.q_chosen[b * A + a] = q[act];
    }
  }
  qmix_mixer<MT>(p, lds, chosen, row0, wave, lane);
}

// The same step with one WAVE per agent (agents w, w + 4, ...) over a 16-env tile: each wave runs
// its agent's whole network in its own LDS region [16][lda] with no workgroup barrier between
// layers, every layer's tiles in mma_multi passes (the GRU's three gates per unit tile, fc1 / fc2
// four tiles at a time); the workgroup meets once, for the mixer.
template <int H, int F>
__global__ void __launch_bounds__(256) qmix_agent_wave_kernel(QmixArgs p) {
  const uint32_t step = p.step_dev != nullptr ? *p.step_dev : p.step;
  extern __shared__ float lds[];
  constexpr int R = 16, UT = H / 16, NT = F / 16;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int64_t row0 = (int64_t)blockIdx.x * R;
  const int lda = p.lda, kxp = p.kxp, A = p.A, NQ = p.n_act;
  float* mine = lds + wave * R * lda;
  float* qv = lds + 4 * R * lda;    // [A][R][16]
  float* chosen = qv + A * R * 16;  // [R][A]
  const int kbx = kxp / 16;
  for (int a = wave; a < A; a += 4) {
    for (int e = lane; e < R * kxp; e += 64) {  // obs rows of agent a, zero padded
      const int r = e / kxp, c = e - r * kxp;
      const int64_t b = row0 + r;
      mine[r * lda + c] = (c < p.I && b < p.B) ? p.obs[(b * A + a) * p.I + c] : 0.0f;
    }
    for (int e = lane; e < R * H; e += 64) {  // hidden rows (zeros for reset envs)
      const int r = e / H, c = e - r * H;
      const int64_t b = row0 + r;
      const bool live = b < p.B && !(p.reset && p.reset[b]);
      mine[r * lda + kxp + c] = live ? p.hidden[(b * A + a) * H + c] : 0.0f;
    }
    wave_sync();
    const f4* wi = (const f4*)(p.w_ih + (size_t)a * 3 * H * kxp);
    const f4* wh = (const f4*)(p.w_hh + (size_t)a * 3 * H * H);
    const float* bi = p.b_ih + a * 3 * H;
    const float* bh = p.b_hh + a * 3 * H;
    f4 hn[UT][1];
#pragma unroll
    for (int u = 0; u < UT; ++u) {
      const int col = u * 16 + (lane & 15);
      f4 g[4][1];
      g[0][0] = splat4(bi[2 * H + col]);
      g[1][0] = splat4(bi[col] + bh[col]);
      g[2][0] = splat4(bi[H + col] + bh[H + col]);
      g[3][0] = splat4(bh[2 * H + col]);
      const f4* const wx[3] = {wi + (size_t)(2 * UT + u) * kbx * 64, wi + (size_t)u * kbx * 64,
                               wi + (size_t)(UT + u) * kbx * 64};
      const f4* const wy[3] = {wh + (size_t)u * UT * 64, wh + (size_t)(UT + u) * UT * 64,
                               wh + (size_t)(2 * UT + u) * UT * 64};
      mma_multi<1, 3>(*reinterpret_cast<f4(*)[3][1]>(&g[0]), mine, lda, 0, wx, kbx, lane);
      mma_multi<1, 3>(*reinterpret_cast<f4(*)[3][1]>(&g[1]), mine, lda, kxp, wy, UT, lane);
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const float hp = mine[(4 * (lane >> 4) + i) * lda + kxp + col];
        const float r = sigmoid_f(g[1][0][i]);
        const float z = sigmoid_f(g[2][0][i]);
        const float n = tanhf(g[0][0][i] + r * g[3][0][i]);
        hn[u][0][i] = (1.0f - z) * n + z * hp;
      }
    }
    wave_sync();
#pragma unroll
    for (int u = 0; u < UT; ++u)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int r = 4 * (lane >> 4) + i, col = u * 16 + (lane & 15);
        mine[r * lda + kxp + col] = hn[u][0][i];
        if (row0 + r < p.B) p.hidden[((row0 + r) * A + a) * H + col] = hn[u][0][i];
      }
    wave_sync();
    // fc1 (H -> F) then fc2 (F -> F), ReLU, four output tiles per mma_multi pass
#pragma unroll
    for (int layer = 0; layer < 2; ++layer) {
      const int col0 = layer == 0 ? kxp : 0, nkb = layer == 0 ? H / 16 : F / 16;
      const float* w = layer == 0 ? p.w1 + (size_t)a * F * H : p.w2 + (size_t)a * F * F;
      const float* bias = (layer == 0 ? p.b1 : p.b2) + a * F;
      f4 acc[NT][1];
#pragma unroll
      for (int t0 = 0; t0 < NT; t0 += 4) {
        const f4* wp[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          wp[j] = (const f4*)w + (size_t)(t0 + j) * nkb * 64;
          acc[t0 + j][0] = splat4(bias[(t0 + j) * 16 + (lane & 15)]);
        }
        mma_multi<1, 4>(*reinterpret_cast<f4(*)[4][1]>(&acc[t0]), mine, lda, col0, wp, nkb, lane);
      }
      wave_sync();
#pragma unroll
      for (int t = 0; t < NT; ++t)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const float v = acc[t][0][i];
          mine[(4 * (lane >> 4) + i) * lda + t * 16 + (lane & 15)] = v > 0.0f ? v : 0.0f;
        }
      wave_sync();
    }
    // fc3 -> Q-values (<= 16 actions: one tile)
    {
      f4 q[1] = {splat4(p.b3[a * 16 + (lane & 15)])};
      mma_tile<1>(q, mine, lda, 0, (const f4*)(p.w3 + (size_t)a * 16 * F), NT, lane);
#pragma unroll
      for (int i = 0; i < 4; ++i) qv[(a * R + 4 * (lane >> 4) + i) * 16 + (lane & 15)] = q[0][i];
    }
    wave_sync();
    if (lane < R) {  // epsilon-greedy for (env lane, agent a), as qmix_policy_kernel
      const int r = lane;
      const int64_t b = row0 + r;
      const float* q = qv + (a * R + r) * 16;
      int g = 0;
      for (int j = 1; j < NQ; ++j)
        if (q[j] > q[g]) g = j;
      const u32x4 d = philox4x32_10(u32x4{(uint32_t)b, step, (uint32_t)a, 4u << 24}, p.key0,
                                    p.key1);
      const float u = (float)(d.x >> 8) * 5.9604644775390625e-8f;
      const int act = u < p.epsilon ? (int)(((uint64_t)d.y * (uint32_t)NQ) >> 32) : g;
      chosen[r * A + a] = q[act];
      if (b < p.B) {
        p.actions[b * A + a] = act;
        if (p.server_actions)
          for (int j = 0; j < p.k; ++j) p.server_actions[(b * A + a) * p.k + j] = act;
        if (p.q_out)
          for (int j = 0; j < NQ; ++j) p.q_out[(b * A + a) * NQ + j] = q[j];
        if (p.q_chosen) p.q_chosen[b * A + a] = q[act];
      }
    }
    wave_sync();
  }
  __syncthreads();
  qmix_mixer<1>(p, lds, chosen, row0, wave, lane);
}

// The same step with TWO waves per agent (A = 4: eight waves, 16-env tiles): wave 2a + h owns half
// of agent a's output tiles in every layer (GRU unit tiles u = h, h + 2, ...; fc1 / fc2 tiles
// [h NT/2, (h+1) NT/2); fc3's k-blocks split in halves and summed), so 8192 envs give 4096 waves --
// four per SIMD instead of two to hide the MFMA and L2 latency.  The pair shares the agent's LDS
// region; every layer boundary is a workgroup barrier (all agents run the same layer sequence).
template <int H, int F>
__global__ void __launch_bounds__(512, LBSIM_QMIX_PAIR_WPE) qmix_agent_pair_kernel(QmixArgs p) {
  const uint32_t step = p.step_dev != nullptr ? *p.step_dev : p.step;
  extern __shared__ float lds[];
  constexpr int R = 16, UT = H / 16, NT = F / 16;
  static_assert(UT % 2 == 0 && NT % 8 == 0, "tiles split in halves of 4-tile passes");
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int a = wave >> 1, h = wave & 1;
  const int64_t row0 = (int64_t)blockIdx.x * R;
  const int lda = p.lda, kxp = p.kxp, A = p.A, NQ = p.n_act;
  LB_PHASE(0);
  float* mine = lds + a * R * lda;
  float* qv = lds + 4 * R * lda;    // [A][R][16]
  float* chosen = qv + A * R * 16;  // [R][A]
  float* part = chosen + R * A;     // [A][R][16] fc3 partials of the h = 1 waves
  float* pre = part + A * R * 16;   // [R][p.sld] the mixer's state rows, staged now (sld > 0)
  const int kbx = kxp / 16;
  const int t2 = lane + 64 * h;     // the pair's 128 threads
  const f4* wi = (const f4*)(p.w_ih + (size_t)a * 3 * H * kxp);
  const f4* wh = (const f4*)(p.w_hh + (size_t)a * 3 * H * H);
  auto gru_wx = [&](int u, const f4* (&wx)[3]) {
    wx[0] = wi + (size_t)(2 * UT + u) * kbx * 64;
    wx[1] = wi + (size_t)u * kbx * 64;
    wx[2] = wi + (size_t)(UT + u) * kbx * 64;
  };
  // the first GRU pass's weights, the epsilon-greedy draw (independent of the network) and the
  // mixer's state rows go out first: their latency hides behind the staging
  BPrime<3> bp_gru;
  auto gru_wy = [&](int u, const f4* (&wy)[3]) {
    wy[0] = wh + (size_t)u * UT * 64;
    wy[1] = wh + (size_t)(UT + u) * UT * 64;
    wy[2] = wh + (size_t)(2 * UT + u) * UT * 64;
  };
  if (!LBSIM_QMIX_PRIME_LATE) {
    const f4* wx[3];
    if (LBSIM_QMIX_ASYNC_OBS) gru_wy(h, wx);  // the hidden pass runs first
    else gru_wx(h, wx);
    bp_gru = mma_prime<3>(wx, LBSIM_QMIX_ASYNC_OBS ? UT : kbx, lane);
  }
  u32x4 eps_d{};
  if (h == 0 && lane < R)
    eps_d = philox4x32_10(u32x4{(uint32_t)(row0 + lane), step, (uint32_t)a, 4u << 24}, p.key0,
                          p.key1);
  // one round of 512 workgroups: the staging's HBM latency is exposed, so every thread issues all
  // its loads -- obs column t2 of the 16 rows (kxp <= 128), hidden column t2 mod H of 16 H / 128
  // rows and their reset bytes, the mixer's state rows -- before any LDS store: values from
  // clamped in-range addresses with no condition, selects at the stores (one HBM round trip; the
  // three loops one after the other waited out three, and a hidden load behind its row's reset byte
  // waited for every earlier load, profiles/r06m/ r06n/)
  static_assert(128 % H == 0 && R * H % 128 == 0, "hidden staging: whole rows per thread group");
  constexpr int RH = R * H / 128;  // hidden rows per thread
  // LBSIM_QMIX_ASYNC_OBS: the obs rows go straight into LDS (global_load_lds, no VGPRs) when a
  // row is whole 64-column blocks (I == kxp, a multiple of 64, <= 128: 4 x 4's 128), and are waited
  // for only before the GRU's input pass -- the hidden pass runs first, on the hidden rows staged
  // below, while the obs rows (2/3 of the 27.6 MB burst at 8192 x 16) are still arriving
  const bool obs_async = LBSIM_QMIX_ASYNC_OBS && p.I == kxp && kxp % 64 == 0 && kxp <= 128;
  if (obs_async) {
    typedef __attribute__((address_space(1))) void gvoid;
    typedef __attribute__((address_space(3))) void lvoid;
    const int nq = kxp / 64;
#pragma unroll
    for (int i = 0; i < R / 2; ++i) {  // wave h: rows 8 h .. 8 h + 7
      const int r = h * (R / 2) + i;
      const int64_t b = row0 + r, bc = b < p.B ? b : p.B - 1;
      for (int q = 0; q < nq; ++q)
        __builtin_amdgcn_global_load_lds(
            (gvoid*)(p.obs + (bc * A + a) * p.I + q * 64 + lane),
            (lvoid*)(mine + r * lda + q * 64), 4, 0, 0);
    }
  }
  const bool obs1 = kxp <= 128 && !obs_async;  // one obs column per thread (else the loop below)
  const bool ocol = t2 < p.I;
  float vo[R];
  if (obs1) {
#pragma unroll
    for (int r = 0; r < R; ++r) {
      const int64_t b = row0 + r, bc = b < p.B ? b : p.B - 1;
      vo[r] = p.obs[(bc * A + a) * p.I + (ocol ? t2 : 0)];
    }
  }
  const int hc = t2 % H, rh0 = (t2 / H) * RH;
  float vh[RH];
  int64_t bch[RH];
#pragma unroll
  for (int i = 0; i < RH; ++i) {
    const int64_t b = row0 + rh0 + i;
    bch[i] = b < p.B ? b : p.B - 1;
    vh[i] = p.hidden[(bch[i] * A + a) * H + hc];
  }
  // the mixer's state rows (up to 3 elements per thread), stored to LDS with the rest
  constexpr int NSR = 3;
  const bool pre3 = p.sld > 0 && R * p.ksp <= NSR * 512;
  const int tid = (int)threadIdx.x, tots = pre3 ? R * p.ksp : 0;
  float vs[NSR];
  int sat[NSR];
#pragma unroll
  for (int k = 0; k < NSR; ++k) {
    const int e = tid + 512 * k, r = e / p.ksp, c = e - r * p.ksp;
    const int64_t b = row0 + r, bc = b < p.B ? b : p.B - 1;
    const bool ok = e < tots && c < p.Ds && b < p.B;
    sat[k] = e < tots ? (ok ? r * p.sld + c : -(r * p.sld + c) - 1) : INT32_MIN;
    vs[k] = p.state[bc * p.Ds + (ok ? c : 0)];
  }
  if (LBSIM_QMIX_PRIME_LATE) {  // the weights after the HBM rows (every workgroup reads the same
    const f4* wx[3];            // lines: L2-channel hot spots)
    if (LBSIM_QMIX_ASYNC_OBS) gru_wy(h, wx);
    else gru_wx(h, wx);
    bp_gru = mma_prime<3>(wx, LBSIM_QMIX_ASYNC_OBS ? UT : kbx, lane);
  }
  // the reset bytes last: their compares (hoisted into the branch) wait for every load above,
  // which are all in flight by then -- one HBM round trip for the whole staging
  bool keep[RH];
#pragma unroll
  for (int i = 0; i < RH; ++i) keep[i] = row0 + rh0 + i < p.B;
  if (p.reset != nullptr) {
    uint8_t m[RH];
#pragma unroll
    for (int i = 0; i < RH; ++i) m[i] = p.reset[bch[i]];
#pragma unroll
    for (int i = 0; i < RH; ++i) keep[i] = keep[i] && m[i] == 0;
  }
  if (obs_async) {
    // (rows past B read the last env's row: their outputs are never stored)
  } else if (obs1) {
    if (t2 < kxp)
#pragma unroll
      for (int r = 0; r < R; ++r) mine[r * lda + t2] = (ocol && row0 + r < p.B) ? vo[r] : 0.0f;
  } else {
    for (int c = t2; c < kxp; c += 128) {  // obs rows of agent a, zero padded (kxp > 128)
      const bool col_ok = c < p.I;
      float v[R];
#pragma unroll
      for (int r = 0; r < R; ++r) {
        const int64_t b = row0 + r, bc = b < p.B ? b : p.B - 1;
        v[r] = p.obs[(bc * A + a) * p.I + (col_ok ? c : 0)];
      }
#pragma unroll
      for (int r = 0; r < R; ++r) mine[r * lda + c] = (col_ok && row0 + r < p.B) ? v[r] : 0.0f;
    }
  }
#pragma unroll
  for (int i = 0; i < RH; ++i) mine[(rh0 + i) * lda + kxp + hc] = keep[i] ? vh[i] : 0.0f;
#pragma unroll
  for (int k = 0; k < NSR; ++k)
    if (sat[k] != INT32_MIN) pre[sat[k] >= 0 ? sat[k] : -sat[k] - 1] = sat[k] >= 0 ? vs[k] : 0.0f;
  if (p.sld > 0 && !pre3) stage_rows(pre, p.sld, 0, p.state, p.Ds, p.Ds, p.ksp, R, row0, p.B, nullptr);
  LB_PHASE(1);
  __syncthreads();
  LB_PHASE(2);
  const float* bi = p.b_ih + a * 3 * H;
  const float* bh = p.b_hh + a * 3 * H;
  f4 hn[UT / 2][1];
#pragma unroll
  for (int uu = 0; uu < UT / 2; ++uu) {
    const int u = h + 2 * uu;
    const int col = u * 16 + (lane & 15);
    f4 g[4][1];
    g[0][0] = splat4(bi[2 * H + col]);
    g[1][0] = splat4(bi[col] + bh[col]);
    g[2][0] = splat4(bi[H + col] + bh[H + col]);
    g[3][0] = splat4(bh[2 * H + col]);
    const f4* wx[3];
    gru_wx(u, wx);
    const f4* wy[3];
    gru_wy(u, wy);
    if (LBSIM_QMIX_ASYNC_OBS) {  // hidden part first (r, z, n_h), then the input part
      mma_multi<1, 3>(*reinterpret_cast<f4(*)[3][1]>(&g[1]), mine, lda, kxp, wy, UT, lane,
                      uu == 0 ? bp_gru : mma_prime<3>(wy, UT, lane));
      if (uu == 0 && obs_async) {  // the obs rows landed in LDS, every wave's
        __builtin_amdgcn_s_waitcnt(kWaitVmcnt0);
        __syncthreads();
      }
      mma_multi<1, 3>(*reinterpret_cast<f4(*)[3][1]>(&g[0]), mine, lda, 0, wx, kbx, lane);
    } else {
      mma_multi<1, 3>(*reinterpret_cast<f4(*)[3][1]>(&g[0]), mine, lda, 0, wx, kbx, lane,
                      uu == 0 ? bp_gru : mma_prime<3>(wx, kbx, lane));
      mma_multi<1, 3>(*reinterpret_cast<f4(*)[3][1]>(&g[1]), mine, lda, kxp, wy, UT, lane);
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const float hp = mine[(4 * (lane >> 4) + i) * lda + kxp + col];
      const float r = sigmoid_f(g[1][0][i]);
      const float z = sigmoid_f(g[2][0][i]);
      const float n = tanhf(g[0][0][i] + r * g[3][0][i]);
      hn[uu][0][i] = (1.0f - z) * n + z * hp;
    }
  }
  // fc1 / fc2: this wave's NT / 2 = 4 tiles of a layer in one mma_multi pass; a layer's first
  // weights are requested before the barrier that precedes it
  static_assert(NT / 2 == 4, "one four-tile pass per layer");
  auto fc_wp = [&](int layer, const f4* (&wp)[4]) {
    const float* w = layer == 0 ? p.w1 + (size_t)a * F * H : p.w2 + (size_t)a * F * F;
    const int nkb = layer == 0 ? H / 16 : F / 16;
#pragma unroll
    for (int j = 0; j < 4; ++j) wp[j] = (const f4*)w + (size_t)(h * (NT / 2) + j) * nkb * 64;
  };
  BPrime<4> bp_fc;
  {
    const f4* wp[4];
    fc_wp(0, wp);
    bp_fc = mma_prime<4>(wp, H / 16, lane);
  }
  LB_PHASE(3);
  __syncthreads();  // both halves have read the old hidden state
#pragma unroll
  for (int uu = 0; uu < UT / 2; ++uu)
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int r = 4 * (lane >> 4) + i, col = (h + 2 * uu) * 16 + (lane & 15);
      mine[r * lda + kxp + col] = hn[uu][0][i];
      if (row0 + r < p.B) p.hidden[((row0 + r) * A + a) * H + col] = hn[uu][0][i];
    }
  __syncthreads();
  LB_PHASE(4);
#pragma unroll
  for (int layer = 0; layer < 2; ++layer) {  // fc1 (H -> F) then fc2 (F -> F), ReLU
    const int col0 = layer == 0 ? kxp : 0, nkb = layer == 0 ? H / 16 : F / 16;
    const float* bias = (layer == 0 ? p.b1 : p.b2) + a * F;
    f4 acc[4][1];
    const f4* wp[4];
    fc_wp(layer, wp);
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[j][0] = splat4(bias[(h * (NT / 2) + j) * 16 + (lane & 15)]);
    mma_multi<1, 4>(acc, mine, lda, col0, wp, nkb, lane, bp_fc);
    if (layer == 0) {
      const f4* wn[4];
      fc_wp(1, wn);
      bp_fc = mma_prime<4>(wn, F / 16, lane);
    }
    __syncthreads();
#pragma unroll
    for (int t = 0; t < 4; ++t)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const float v = acc[t][0][i];
        mine[(4 * (lane >> 4) + i) * lda + (h * (NT / 2) + t) * 16 + (lane & 15)] =
            v > 0.0f ? v : 0.0f;
      }
    __syncthreads();
    LB_PHASE(5 + layer);
  }
  // fc3 -> Q-values (<= 16 actions: one tile), k-blocks [h NT/2, (h+1) NT/2); the halves meet in LDS
  {
    f4 q[1] = {splat4(h == 0 ? p.b3[a * 16 + (lane & 15)] : 0.0f)};
    mma_tile<1>(q, mine, lda, h * (NT / 2) * 16,
                (const f4*)(p.w3 + (size_t)a * 16 * F) + (size_t)h * (NT / 2) * 64, NT / 2, lane);
    if (h == 1)
#pragma unroll
      for (int i = 0; i < 4; ++i) part[(a * R + 4 * (lane >> 4) + i) * 16 + (lane & 15)] = q[0][i];
    __syncthreads();
    if (h == 0)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int o = (a * R + 4 * (lane >> 4) + i) * 16 + (lane & 15);
        qv[o] = q[0][i] + part[o];
      }
  }
  __syncthreads();
  LB_PHASE(7);
  // epsilon-greedy for (env lane, agent a), as qmix_policy_kernel.  Its results (chosen) are read
  // only by the mixer's tail, so it runs inside the mixer's first layer, after that layer's GEMM
  // and before its barrier (LBSIM_QMIX_EPS_IN_MIXER; it had a barrier interval of its own)
  auto eps_greedy = [&]() {
    if (h == 0 && lane < R) {
      const int r = lane;
      const int64_t b = row0 + r;
      const float* q = qv + (a * R + r) * 16;
      int g = 0;
      for (int j = 1; j < NQ; ++j)
        if (q[j] > q[g]) g = j;
      const u32x4 d = eps_d;  // drawn at the start
      const float u = (float)(d.x >> 8) * 5.9604644775390625e-8f;
      const int act = u < p.epsilon ? (int)(((uint64_t)d.y * (uint32_t)NQ) >> 32) : g;
      chosen[r * A + a] = q[act];
      if (b < p.B) {
        p.actions[b * A + a] = act;
        if (p.server_actions)
          for (int j = 0; j < p.k; ++j) p.server_actions[(b * A + a) * p.k + j] = act;
        if (p.q_out)
          for (int j = 0; j < NQ; ++j) p.q_out[(b * A + a) * NQ + j] = q[j];
        if (p.q_chosen) p.q_chosen[b * A + a] = q[act];
      }
    }
  };
  if (!LBSIM_QMIX_EPS_IN_MIXER) {
    eps_greedy();
    __syncthreads();
  }
  LB_PHASE(8);
  if (LBSIM_QMIX_EPS_IN_MIXER)
    qmix_mixer<1, LBSIM_MIX_NW>(p, lds, chosen, row0, wave, lane, p.sld > 0 ? pre : nullptr,
                                p.sld, eps_greedy);
  else
    qmix_mixer<1, LBSIM_MIX_NW>(p, lds, chosen, row0, wave, lane, p.sld > 0 ? pre : nullptr,
                                p.sld);
  LB_PHASE(11);
}

}  // namespace lbk
