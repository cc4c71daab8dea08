// Micro-benchmark: cycles per instruction of the integer multiplies Philox4x32-10 is built from
// (v_mad_u64_u32, v_mul_hi_u32 / v_mul_lo_u32, v_mul_u32_u24) and of whole Philox blocks, one
// wave alone on its SIMD, dependent chains vs independent ones.  Prints one JSON line.
//   hipcc -O3 --offload-arch=gfx950 -o tools/ubench_mul tools/ubench_mul.hip && ./tools/ubench_mul
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

constexpr int N = 4096;
constexpr uint32_t M0 = 0xD2511F53u, M1 = 0xCD9E8D57u;

struct U4 { uint32_t x, y, z, w; };

__device__ __forceinline__ U4 philox(U4 c, uint32_t k0, uint32_t k1) {
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    const uint64_t p0 = (uint64_t)M0 * c.x;
    const uint64_t p1 = (uint64_t)M1 * c.z;
    c = U4{(uint32_t)__builtin_amdgcn_bitop3_b32((uint32_t)(p1 >> 32), c.y, k0, 0x96), (uint32_t)p1,
           (uint32_t)__builtin_amdgcn_bitop3_b32((uint32_t)(p0 >> 32), c.w, k1, 0x96), (uint32_t)p0};
    k0 += 0x9E3779B9u;
    k1 += 0xBB67AE85u;
  }
  return c;
}

template <int V>
__global__ void __launch_bounds__(64) bench(uint32_t* out, uint32_t seed, long long* cyc) {
  uint32_t a = seed + threadIdx.x, b = a * 3u + 1u, c = a * 5u + 7u, d = a * 11u + 13u;
  const long long t0 = clock64();
  for (int i = 0; i < N; ++i) {
    if constexpr (V == 0) {  // dependent v_mad_u64_u32 (through the high word)
      const uint64_t p = (uint64_t)M0 * a;
      a = (uint32_t)(p >> 32) ^ (uint32_t)p;
    } else if constexpr (V == 1) {  // 4 independent v_mad_u64_u32 chains
      const uint64_t p = (uint64_t)M0 * a, q = (uint64_t)M0 * b, r = (uint64_t)M0 * c,
                     s = (uint64_t)M0 * d;
      a = (uint32_t)(p >> 32) ^ (uint32_t)p;
      b = (uint32_t)(q >> 32) ^ (uint32_t)q;
      c = (uint32_t)(r >> 32) ^ (uint32_t)r;
      d = (uint32_t)(s >> 32) ^ (uint32_t)s;
    } else if constexpr (V == 2) {  // 4 independent v_mul_hi_u32
      a = __umulhi(a, M0) + i;
      b = __umulhi(b, M0) + i;
      c = __umulhi(c, M0) + i;
      d = __umulhi(d, M0) + i;
    } else if constexpr (V == 3) {  // 4 independent v_mul_lo_u32
      a = a * M0 + (uint32_t)i;
      b = b * M0 + (uint32_t)i;
      c = c * M0 + (uint32_t)i;
      d = d * M0 + (uint32_t)i;
    } else if constexpr (V == 4) {  // 4 independent v_mul_u32_u24
      a = __umul24(a, 0x511F53u) + i;
      b = __umul24(b, 0x511F53u) + i;
      c = __umul24(c, 0x511F53u) + i;
      d = __umul24(d, 0x511F53u) + i;
    } else if constexpr (V == 5) {  // 4 independent v_xad (add + xor) : plain VALU reference
      a = (a ^ b) + 0x9E3779B9u;
      b = (b ^ c) + 0x3u;
      c = (c ^ d) + 0x5u;
      d = (d ^ a) + 0x7u;
    } else if constexpr (V == 6) {  // one Philox block per iteration (counter from the chain)
      const U4 r = philox(U4{a, b, c, d}, seed, seed * 7u);
      a = r.x; b = r.y; c = r.z; d = r.w;
    } else if constexpr (V == 7) {  // two independent Philox blocks per iteration, interleaved
      const U4 r = philox(U4{a, b, 1u, 2u}, seed, seed * 7u);
      const U4 s = philox(U4{c, d, 3u, 4u}, seed, seed * 7u);
      a = r.x ^ r.z; b = r.y ^ r.w; c = s.x ^ s.z; d = s.y ^ s.w;
    }
  }
  const long long t1 = clock64();
  out[blockIdx.x * 64 + threadIdx.x] = a ^ b ^ c ^ d;
  if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

template <int V>
double run(uint32_t* out, long long* cyc, int blocks) {
  hipLaunchKernelGGL(bench<V>, dim3(blocks), dim3(64), 0, 0, out, 1u, cyc);
  hipDeviceSynchronize();
  hipLaunchKernelGGL(bench<V>, dim3(blocks), dim3(64), 0, 0, out, 2u, cyc);
  hipDeviceSynchronize();
  long long h[2048];
  hipMemcpy(h, cyc, sizeof(long long) * blocks, hipMemcpyDeviceToHost);
  double s = 0;
  for (int i = 0; i < blocks; ++i) s += (double)h[i];
  return s / blocks / N;
}

int main() {
  uint32_t* out;
  long long* cyc;
  hipMalloc(&out, 2048 * 64 * 4);
  hipMalloc(&cyc, 2048 * 8);
  const char* names[] = {"mad64_dep", "mad64_x4", "mulhi_x4", "mullo_x4", "mul24_x4", "xoradd_x4",
                         "philox1", "philox2_interleaved"};
  double r1[8], r2[8];
  // 1 wave on the chip, then 2048 waves (2 per SIMD on 1024 SIMDs): clock64 ticks per iteration
  r1[0] = run<0>(out, cyc, 1); r1[1] = run<1>(out, cyc, 1); r1[2] = run<2>(out, cyc, 1);
  r1[3] = run<3>(out, cyc, 1); r1[4] = run<4>(out, cyc, 1); r1[5] = run<5>(out, cyc, 1);
  r1[6] = run<6>(out, cyc, 1); r1[7] = run<7>(out, cyc, 1);
  r2[0] = run<0>(out, cyc, 2048); r2[1] = run<1>(out, cyc, 2048); r2[2] = run<2>(out, cyc, 2048);
  r2[3] = run<3>(out, cyc, 2048); r2[4] = run<4>(out, cyc, 2048); r2[5] = run<5>(out, cyc, 2048);
  r2[6] = run<6>(out, cyc, 2048); r2[7] = run<7>(out, cyc, 2048);
  printf("{\"unit\": \"clock64 ticks per loop iteration\", \"one_wave\": {");
  for (int v = 0; v < 8; ++v) printf("%s\"%s\": %.2f", v ? ", " : "", names[v], r1[v]);
  printf("}, \"two_waves_per_simd\": {");
  for (int v = 0; v < 8; ++v) printf("%s\"%s\": %.2f", v ? ", " : "", names[v], r2[v]);
  printf("}}\n");
  return 0;
}
