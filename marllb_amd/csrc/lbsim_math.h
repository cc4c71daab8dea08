// lbsim_math.h — bit-reproducible scalar math for the gfx950 kernels.
//
// Every function here is written with plain IEEE-754 binary32/binary64 +,-,*,/, explicit fma and
// integer ops only, and the whole library is compiled with -ffp-contract=off, so a kernel lane produces the
// same bits as oracle/lbsim_oracle.c (gcc, -ffp-contract=off) for the same inputs.  That is what
// makes the server-assignment indices and every integer state word bit-exact against the oracle
// (DESIGN.md §3.1).  No hardware transcendental (v_exp_f32/v_log_f32) is used on the state path.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace lbk {

// Orders one wave's LDS accesses (scratch private to a wave): a compiler fence and a wave
// barrier.  A wave's LDS instructions execute in issue order, so no s_barrier (which would meet the
// other waves of a multi-wave workgroup) and no counter wait are needed.
__device__ __forceinline__ void wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// ---------------------------------------------------------------- Philox4x32-10 (Salmon et al.
// SC'11, "Parallel random numbers: as easy as 1, 2, 3").  Counter-based: the draw for
// (env, episode, stream, index) is a pure function, so no RNG state is stored per env.
struct u32x4 {
  uint32_t x, y, z, w;
};

__device__ __forceinline__ u32x4 philox4x32_10(u32x4 c, uint32_t k0, uint32_t k1) {
  constexpr uint32_t M0 = 0xD2511F53u, M1 = 0xCD9E8D57u;
  constexpr uint32_t W0 = 0x9E3779B9u, W1 = 0xBB67AE85u;
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    // one 32x32->64 multiply per product (v_mad_u64_u32) instead of mul_hi + mul_lo
    const uint64_t p0 = (uint64_t)M0 * c.x;
    const uint64_t p1 = (uint64_t)M1 * c.z;
    c = u32x4{(uint32_t)(p1 >> 32) ^ c.y ^ k0, (uint32_t)p1, (uint32_t)(p0 >> 32) ^ c.w ^ k1,
              (uint32_t)p0};
    k0 += W0;
    k1 += W1;
  }
  return c;
}

// RNG streams (counter word w bits 24..31); see DESIGN.md §3.2.
constexpr uint32_t kStreamArrival = 1u;
constexpr uint32_t kStreamReservoir = 2u;

// Uniform in (0, 1]: 24 high bits + 1, scaled by 2^-24 (exact in binary32).
__device__ __forceinline__ float u01_open0(uint32_t r) {
  return (float)((r >> 8) + 1u) * 5.9604644775390625e-8f;
}

__device__ __forceinline__ float as_f32(uint32_t u) { return __uint_as_float(u); }
__device__ __forceinline__ uint32_t as_u32(float f) { return __float_as_uint(f); }

// Natural log for x in [2^-24, 1], no division: x = m 2^e with m folded into [sqrt(1/2), sqrt(2)],
// ln m = log1p(f), f = m - 1, by the Cephes single-precision logf polynomial (Moshier; max relative
// error over every k 2^-24, k = 1..2^24: 8.2e-8) in fmaf Horner form -- an explicit fma is
// correctly rounded on the GPU (v_fma_f32) and in C (fmaf), so both sides get the same bits.
__device__ __forceinline__ float lb_logf(float x) {
  const uint32_t b = as_u32(x);
  int e = (int)(b >> 23) - 127;
  float m = as_f32((b & 0x007fffffu) | 0x3f800000u);
  if (m > 1.41421354f) { m = m * 0.5f; e = e + 1; }
  const float f = m - 1.0f;  /* exact */
  const float z = f * f;
  float p = 7.0376836292e-2f;
  p = fmaf(p, f, -1.1514610310e-1f);
  p = fmaf(p, f, 1.1676998740e-1f);
  p = fmaf(p, f, -1.2420140846e-1f);
  p = fmaf(p, f, 1.4249322787e-1f);
  p = fmaf(p, f, -1.6668057665e-1f);
  p = fmaf(p, f, 2.0000714765e-1f);
  p = fmaf(p, f, -2.4999993993e-1f);
  p = fmaf(p, f, 3.3333331174e-1f);
  float y = (p * f) * z;
  y = fmaf(-0.5f, z, y);
  const float fe = (float)e;  /* ln 2 = 0.693359375 - 2.12194440e-4 (Cephes split) */
  float r = fmaf(fe, -2.12194440e-4f, y);
  r = r + f;
  return fmaf(fe, 0.693359375f, r);
}

// 2^x for x <= 0 (x < -60 -> 0): x = n + f, n = floor(x + 1/2), f in [-1/2, 1/2), degree-7
// Taylor of e^(f ln2) (truncation error < 6e-9) in fmaf Horner form, times 2^n.
__device__ __forceinline__ float lb_exp2f(float x) {
  // branch-free: x < -60 selects 0 at the end (the polynomial of a clamped x is discarded)
  const bool under = x < -60.0f;
  x = under ? 0.0f : x;
  const float fl = floorf(x + 0.5f);  /* exact for |x| <= 60 */
  const int n = (int)fl;
  const float f = x - fl;             /* exact, in [-0.5, 0.5) */
  float p = 1.52527336e-5f;
  p = fmaf(p, f, 1.54035297e-4f);
  p = fmaf(p, f, 1.33335581e-3f);
  p = fmaf(p, f, 9.61812911e-3f);
  p = fmaf(p, f, 5.55041086e-2f);
  p = fmaf(p, f, 0.240226507f);
  p = fmaf(p, f, 0.693147182f);
  p = fmaf(p, f, 1.0f);
  const float r = p * as_f32((uint32_t)(n + 127) << 23);
  return under ? 0.0f : r;
}

// floor(r64 * n / 2^64) for n <= 2^32: uniform integer in [0, n) (Lemire multiply-shift, 64-bit
// source, bias <= n / 2^64).  Used for Algorithm R's j = randint(0, count + 1).
__device__ __forceinline__ uint64_t mulhi64_by_u33(uint32_t r_hi, uint32_t r_lo, uint64_t n) {
  const uint64_t a = (uint64_t)r_hi * n;
  const uint64_t b = ((uint64_t)r_lo * n) >> 32;
  return (a + b) >> 32;
}

}  // namespace lbk
