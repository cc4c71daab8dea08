// Micro-benchmark: VALU issue cost per instruction class on gfx950, with 1, 2, 4 and 8 waves per
// SIMD (grids of 1024 * k single-wave workgroups on 256 CUs), independent accumulator chains
// (throughput) and one dependent chain (latency).  Calibrates the simulator kernels' VALU
// accounting (SQ_INSTS_VALU per op class -> SIMD cycles).  One JSON line per case:
//   {"op", "waves_per_simd", "chains", "cyc_per_inst_wave" (median over waves, s_memtime
//    cycles per instruction of one wave), "simd_cyc_per_inst" (= cyc_per_inst_wave / k: issue
//    cycles the SIMD spends per instruction when k waves share it)}
//   hipcc -O3 --offload-arch=gfx950 -o tools/ubench_valu tools/ubench_valu.hip
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#include <algorithm>
#include <vector>

constexpr int ITER = 256;  // loop trips; each trip issues UNROLL x CH instructions of the class
constexpr int UNROLL = 8;

template <int OP, int CH>
__global__ void __launch_bounds__(64) bench(uint32_t* sink, long long* cyc, uint32_t seed) {
  const uint32_t l = threadIdx.x + seed;
  uint32_t u[CH];
  float f[CH];
  double d[CH];
#pragma unroll
  for (int c = 0; c < CH; ++c) {
    u[c] = l * (2u * c + 3u) + 7u;
    f[c] = (float)(l + c) * 1e-3f;
    d[c] = (double)(l + c) * 1e-3;
  }
  const float fa = 1.0001f + (float)seed * 1e-9f, fb = 1e-7f;
  const double da = 1.0000001 + (double)seed * 1e-12, db = 1e-9;
  const long long t0 = clock64();
  for (int i = 0; i < ITER; ++i) {
#pragma unroll
    for (int k = 0; k < UNROLL; ++k) {
#pragma unroll
      for (int c = 0; c < CH; ++c) {
        if constexpr (OP == 0) {  // v_add_u32
          asm volatile("v_add_u32 %0, %0, %1" : "+v"(u[c]) : "v"(l));
        } else if constexpr (OP == 1) {  // v_fma_f32
          asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(f[c]) : "v"(fa), "v"(fb));
        } else if constexpr (OP == 2) {  // v_fma_f64
          asm volatile("v_fma_f64 %0, %0, %1, %2" : "+v"(d[c]) : "v"(da), "v"(db));
        } else if constexpr (OP == 3) {  // v_add_f64
          asm volatile("v_add_f64 %0, %0, %1" : "+v"(d[c]) : "v"(db));
        } else if constexpr (OP == 4) {  // v_mad_u64_u32 (the Philox / Algorithm R multiply)
          uint64_t p;
          asm volatile("v_mad_u64_u32 %0, vcc, %1, %2, 0" : "=v"(p) : "v"(u[c]), "v"(l) : "vcc");
          u[c] = (uint32_t)p ^ (uint32_t)(p >> 32);
        } else if constexpr (OP == 5) {  // v_med3_u32 (the sort's cross-lane compare-exchange)
          asm volatile("v_med3_u32 %0, %0, %1, %2" : "+v"(u[c]) : "v"(l), "v"(seed));
        } else if constexpr (OP == 6) {  // DPP row move (reductions), via the builtin: hazards kept
          u[c] = (uint32_t)__builtin_amdgcn_mov_dpp((int)u[c], 0x141, 0xF, 0xF, true) + 1u;
        } else if constexpr (OP == 7) {  // v_exp_f32 (transcendental)
          asm volatile("v_exp_f32 %0, %0" : "+v"(f[c]));
        } else if constexpr (OP == 8) {  // v_cvt_f64_f32 (the decay-weight upcasts)
          asm volatile("v_cvt_f64_f32 %0, %1" : "=v"(d[c]) : "v"(f[c]));
          asm volatile("v_cvt_f32_f64 %0, %1" : "=v"(f[c]) : "v"(d[c]));
        } else if constexpr (OP == 9) {  // v_lshlrev_b64 (64-bit shifts of the fixed-point sums)
          uint64_t x = ((uint64_t)u[c] << 32) | l;
          asm volatile("v_lshlrev_b64 %0, 1, %0" : "+v"(x));
          u[c] = (uint32_t)x ^ (uint32_t)(x >> 32);
        } else if constexpr (OP == 10) {  // v_mul_f64
          asm volatile("v_mul_f64 %0, %0, %1" : "+v"(d[c]) : "v"(da));
        }
      }
    }
  }
  const long long t1 = clock64();
  uint32_t x = 0;
#pragma unroll
  for (int c = 0; c < CH; ++c) x ^= u[c] ^ __float_as_uint(f[c]) ^ (uint32_t)__double_as_longlong(d[c]);
  sink[blockIdx.x * 64 + threadIdx.x] = x;
  if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

// instructions per trip of the class (ops 4, 8, 9 issue helper VALU too: counted separately)
const char* kName[] = {"v_add_u32", "v_fma_f32", "v_fma_f64", "v_add_f64", "v_mad_u64_u32+xor",
                       "v_med3_u32", "v_mov_dpp+add", "v_exp_f32", "v_cvt_f64_f32+v_cvt_f32_f64",
                       "v_lshlrev_b64+pack", "v_mul_f64"};

template <int OP, int CH>
void run(uint32_t* sink, long long* cyc, int cus) {
  for (int k : {1, 2, 4, 8}) {
    const int blocks = cus * 4 * k;
    hipLaunchKernelGGL((bench<OP, CH>), dim3(blocks), dim3(64), 0, 0, sink, cyc, 1u);
    hipDeviceSynchronize();
    hipLaunchKernelGGL((bench<OP, CH>), dim3(blocks), dim3(64), 0, 0, sink, cyc, 2u);
    hipDeviceSynchronize();
    std::vector<long long> h(blocks);
    hipMemcpy(h.data(), cyc, sizeof(long long) * blocks, hipMemcpyDeviceToHost);
    std::sort(h.begin(), h.end());
    const double per = (double)h[blocks / 2] / ((double)ITER * UNROLL * CH);
    printf("{\"op\": \"%s\", \"waves_per_simd\": %d, \"chains\": %d, \"cyc_per_inst_wave\": %.3f, "
           "\"simd_cyc_per_inst\": %.3f}\n",
           kName[OP], k, CH, per, per / k);
  }
}

template <int OP>
void op(uint32_t* sink, long long* cyc, int cus) {
  run<OP, 8>(sink, cyc, cus);  // throughput
  run<OP, 1>(sink, cyc, cus);  // latency (one dependent chain)
}

int main() {
  int cus = 0;
  hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
  uint32_t* sink;
  long long* cyc;
  hipMalloc(&sink, (size_t)cus * 4 * 8 * 64 * 4);
  hipMalloc(&cyc, (size_t)cus * 4 * 8 * 8);
  op<0>(sink, cyc, cus);
  op<1>(sink, cyc, cus);
  op<2>(sink, cyc, cus);
  op<3>(sink, cyc, cus);
  op<4>(sink, cyc, cus);
  op<5>(sink, cyc, cus);
  op<6>(sink, cyc, cus);
  op<7>(sink, cyc, cus);
  op<8>(sink, cyc, cus);
  op<9>(sink, cyc, cus);
  op<10>(sink, cyc, cus);
  hipFree(sink);
  hipFree(cyc);
  return 0;
}
