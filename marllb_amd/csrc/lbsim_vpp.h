// lbsim_vpp.h — the VPP LB plugin's shared-memory view of the simulator.
//
// The live data plane (src/vpp/lb) keeps, per application server (AS), two raw reservoirs of
// 128 (t, v) f32 pairs -- flow completion time and flow duration, `reservoir_as_t`
// (src/vpp/lb/shm.h:35-37) -- and the agent side (src/lb/shm_proxy.py:518-543, process_reservoir)
// turns them into 5 features each, in float64 over ALL 128 bins:
//     mean(v), percentile(v, 90), std(v), mean(v * 0.9^(ts - t)), percentile(v * 0.9^(ts - t), 90)
// (the "upstream" feature semantics; problem-01's reservoir.py, which the env's own observation
// follows, decays the weights instead).
//
//   vpp_export_kernel    simulator state -> that wire view: per (env, server) the 2 x 128 (t, v)
//                        pairs (reservoir_mode ALGR: slots >= min(count, 128) as the zeros of
//                        VPP's fresh shm; VPP: every bin as stored), the server's n_flow_on and
//                        the frame timestamp of each env.
//   vpp_features_kernel  process_reservoir on n raw reservoirs, one wave each: numpy's pairwise
//                        sums (pairwise8), its std and its 'linear' percentile, so everything but
//                        the f64 pow of the decay factor is bit-identical to numpy.
#pragma once

#include "lbsim_kernels.h"

namespace lbk {

// numpy 'linear' percentile of 128 sorted values at q = 0.9: virtual index (n - 1) q = 114.3, gamma
// the f64 fraction, _lerp(a, b, t) = a + (b - a) t for t < 0.5 (numpy/lib/_function_base_impl.py).
constexpr int kVppN = 128;
constexpr int kVppP90Lo = 114;

// Order-preserving u64 key of a double (finite values; -0 just below +0, then turned back).
__device__ __forceinline__ uint64_t f64_key(double x) {
  const uint64_t b = (uint64_t)__double_as_longlong(x);
  return (b >> 63) ? ~b : (b | 0x8000000000000000ull);
}
__device__ __forceinline__ double key_f64(uint64_t k) {
  return __longlong_as_double((long long)((k >> 63) ? (k & 0x7FFFFFFFFFFFFFFFull) : ~k));
}

// Ascending bitonic sort of 128 u64 keys in LDS by one wave (64 compare-exchange pairs a stage).
__device__ __forceinline__ void bitonic128_lds_u64(uint64_t* key, int lane) {
  for (int k = 2; k <= kVppN; k <<= 1) {
    for (int j = k >> 1; j > 0; j >>= 1) {
      const int i = (lane / j) * 2 * j + (lane % j), l = i + j;
      const bool up = (i & k) == 0;
      const uint64_t a = key[i], b = key[l];
      if ((a > b) == up) {
        key[i] = b;
        key[l] = a;
      }
      __syncthreads();
    }
  }
}

// process_reservoir (shm_proxy.py:518-543) of reservoir r: tv[r][128] (t, v) f32 pairs, frame time
// ts[r / res_per_ts] f32 -> out[r][5] f64 {avg, 90, std, avg_decay, 90_decay}.
__global__ void __launch_bounds__(64)
    vpp_features_kernel(const float2* tv, const float* ts, int64_t res_per_ts, int64_t n,
                        double decay, double* out) {
  __shared__ double val[kVppN], vdec[kVppN];
  __shared__ uint64_t key[kVppN];
  const int64_t r = blockIdx.x;
  const int lane = (int)threadIdx.x, j = lane & 7;
  if (r >= n) return;
  const double now = (double)ts[r / res_per_ts];  // Python float of the frame's f32 ts
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const int i = lane + 64 * h;
    const float2 p = tv[r * kVppN + i];
    const double v = (double)p.y;
    val[i] = v;
    vdec[i] = v * pow(decay, now - (double)p.x);  // np.multiply(v, np.power(0.9, ts - t))
  }
  __syncthreads();
  // np.mean / np.std: pairwise sum, true_divide by n; std over (v - mean)^2
  const double mean = pairwise8<double>(kVppN, j, [&](int i) { return val[i]; }) / (double)kVppN;
  const double ss = pairwise8<double>(kVppN, j, [&](int i) {
    const double x = val[i] - mean;
    return x * x;
  });
  const double sd = sqrt(ss / (double)kVppN);
  const double meand = pairwise8<double>(kVppN, j, [&](int i) { return vdec[i]; }) / (double)kVppN;
  const double vi = (double)(kVppN - 1) * 0.9;  // 114.3 (numpy: (n - 1) * quantiles)
  const double gamma = vi - (double)kVppP90Lo;
  double p90[2];
#pragma unroll
  for (int q = 0; q < 2; ++q) {
    const double* src = q == 0 ? val : vdec;
    key[lane] = f64_key(src[lane]);
    key[lane + 64] = f64_key(src[lane + 64]);
    __syncthreads();
    bitonic128_lds_u64(key, lane);
    const double a = key_f64(key[kVppP90Lo]), b = key_f64(key[kVppP90Lo + 1]);
    const double d = b - a;
    p90[q] = a + d * gamma;  // gamma < 0.5: the add branch of _lerp
    __syncthreads();
  }
  if (lane == 0) {
    double* o = out + r * 5;
    o[0] = mean;
    o[1] = p90[0];
    o[2] = sd;
    o[3] = meand;
    o[4] = p90[1];
  }
}

// One wave per (env, server) of envs [e0, e0 + n): the server's reservoirs as VPP's raw
// reservoir_as_t (t = sample timestamp in seconds, v = sample in seconds, f32; slots past
// min(count, 128) zero), its n_flow_on, and (server 0) the env's frame time clock * dt in seconds.
__global__ void __launch_bounds__(64)
    vpp_export_kernel(DevState st, SimParams p, int64_t e0, int64_t n, float2* tv_out,
                      int32_t* nflow_out, float* ts_out) {
  const int64_t pair = blockIdx.x;
  const int S = p.S, lane = (int)threadIdx.x;
  if (pair >= n * S) return;
  const int64_t e = pair / S;
  const int s = (int)(pair - e * S);
  const size_t b = (size_t)(e0 + e), sb = b * (size_t)S + (size_t)s;
  // reservoir_mode VPP: every bin as stored (zeroed at reset: VPP's shm); ALGR: the first
  // min(count, 128).  Split handles (lost-FIN): the duration reservoir's own count and timestamps.
  const bool split = st.res_count_dur != nullptr;
  const uint32_t c = st.res_count[sb];
  const uint32_t cd = split ? st.res_count_dur[sb] : c;
  const int cnt = p.res_vpp ? K : (c < (uint32_t)K ? (int)c : K);
  const int cntd = p.res_vpp ? K : (cd < (uint32_t)K ? (int)cd : K);
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const int i = lane + 64 * h;
    float t = 0.0f, fv = 0.0f, td = 0.0f, dv = 0.0f;
    if (i < cnt) {
      const uint2 rec = st.res[sb * K + (size_t)i];
      t = (float)((double)rec.y * 1e-3);
      fv = sample_value<true>(rec.x);
      if (!split) {
        td = t;
        dv = st.res_dur != nullptr ? sample_value<true>(st.res_dur[sb * K + (size_t)i]) : fv;
      }
    }
    if (split && i < cntd) {
      const uint2 dr = reinterpret_cast<const uint2*>(st.res_dur)[sb * K + (size_t)i];
      td = (float)((double)dr.y * 1e-3);
      dv = sample_value<true>(dr.x);
    }
    tv_out[(pair * 2 + 0) * kVppN + i] = make_float2(t, fv);
    tv_out[(pair * 2 + 1) * kVppN + i] = make_float2(td, dv);
  }
  if (lane == 0) {
    if (nflow_out != nullptr) nflow_out[pair] = (int32_t)n_flow_on(st, sb);
    if (s == 0 && ts_out != nullptr)
      ts_out[e] = (float)((double)st.clock[b] * (double)p.dt_us * 1e-6);
  }
}

}  // namespace lbk
