// lbsim_nets.h — fused elementwise kernels of the on-GPU policies.
//
// The GEMMs of the GRU + MLP networks (problem-04 PolicyNetwork networks.py:19-151, problem-05
// AgentQNetwork agent_network.py:13-92) go to hipBLASLt; everything between them is fused here so a
// policy step is GEMM, GEMM, gru_gates, GEMM (+ReLU epilogue), GEMM, head -- instead of MIOpen's
// generic RNN path (≈ 20 tensor-op launches per step at configs[3]).
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

#include "lbsim_math.h"

namespace lbk {

__device__ __forceinline__ float sigmoidf_(float x) { return 1.0f / (1.0f + expf(-x)); }

// PyTorch GRU cell (torch.nn.GRU, gate order r, z, n):
//   r = σ(gi_r + gh_r), z = σ(gi_z + gh_z), n = tanh(gi_n + r ⊙ gh_n), h' = (1 − z) ⊙ n + z ⊙ h
// gi = x W_ih^T + b_ih and gh = h W_hh^T + b_hh come from the two GEMMs, [B, 3H] row-major.
__global__ void __launch_bounds__(256)
    gru_gates_kernel(const float* gi, const float* gh, const float* h, float* h_out, int64_t B,
                     int H) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= B * H) return;
  const int64_t b = i / H;
  const int u = (int)(i - b * H);
  const float* a = gi + b * 3 * H;
  const float* c = gh + b * 3 * H;
  const float r = sigmoidf_(a[u] + c[u]);
  const float z = sigmoidf_(a[H + u] + c[H + u]);
  const float n = tanhf(a[2 * H + u] + r * c[2 * H + u]);
  h_out[i] = (1.0f - z) * n + z * h[i];
}

// SAC actor head (networks.py:98-146): y = [B, 2A] = [mean | log_std_raw];
// log_std = clamp(raw, lo, hi); deterministic: tanh(mean); else tanh(mean + exp(log_std) ε),
// ε ~ N(0,1) from Philox4x32-10 (counter = (b, step, a, stream 3)) by Box–Muller; then
// action = tanh(·) * scale + bias.  Also writes the clamped log_std (log-prob needs it).
__global__ void __launch_bounds__(256)
    sac_head_kernel(const float* y, int64_t B, int A, float lo, float hi, float scale, float bias,
                    int deterministic, uint32_t key0, uint32_t key1, uint32_t step,
                    float* action, float* log_std_out) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= B * A) return;
  const int64_t b = i / A;
  const int a = (int)(i - b * A);
  const float mean = y[b * 2 * A + a];
  float ls = y[b * 2 * A + A + a];
  ls = ls < lo ? lo : (ls > hi ? hi : ls);
  float x = mean;
  if (!deterministic) {
    const u32x4 d = philox4x32_10(u32x4{(uint32_t)b, step, (uint32_t)a, 3u << 24}, key0, key1);
    const float u1 = u01_open0(d.x), u2 = (float)(d.y >> 8) * 5.9604644775390625e-8f;
    const float eps = sqrtf(-2.0f * logf(u1)) * cospif(2.0f * u2);
    x = mean + expf(ls) * eps;
  }
  action[i] = tanhf(x) * scale + bias;
  if (log_std_out) log_std_out[i] = ls;
}

// QMIX mixing tail (mixing_network.py:96-116) per env, after the hypernetwork GEMMs:
//   hidden_e = elu(b1_e + sum_a q_a |w1_(a,e)|),  Q_tot = sum_e hidden_e |w2_e| + b2
// with w1 = hyper_w1(state) [B, A*E] (viewed (A, E)), b1 [B, E], w2 [B, E], b2 [B] (strided).
__global__ void __launch_bounds__(256)
    qmix_tail_kernel(const float* q, const float* w1, int64_t w1_ld, const float* b1,
                     int64_t b1_ld, const float* w2, int64_t w2_ld, const float* b2,
                     int64_t b2_ld, int64_t B, int A, int E, float* q_tot) {
  const int64_t b = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= B) return;
  float acc = 0.0f;
  for (int e = 0; e < E; ++e) {
    float h = 0.0f;
    for (int a = 0; a < A; ++a) h += q[b * A + a] * fabsf(w1[b * w1_ld + a * E + e]);
    h += b1[b * b1_ld + e];
    h = h > 0.0f ? h : expm1f(h);  // F.elu, alpha = 1
    acc += h * fabsf(w2[b * w2_ld + e]);
  }
  q_tot[b] = acc + b2[b * b2_ld];
}

}  // namespace lbk
