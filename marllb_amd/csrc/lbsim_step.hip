// lbsim_step.hip — the fused step: one launch per step runs a wave's dynamics and then observes the
// same envs ("fused step").
//
// fused_step_kernel<G, MAXS, POLICY, TRACE>: one 64-lane workgroup = the 64 / G envs of one
// dynamics wave (dyn_group_wave, lbsim_dyn_group.h).  Phase 1 steps them; a workgroup barrier makes
// the wave's state writes visible to its own loads (L1 shared by the workgroup); phase 2 observes
// them one env after the other with observe_env_wave (every chunk of an env by this wave).  The
// dynamics LDS and the observe scratch share one union.  Compared with the two launches:
//   - no dynamics -> observe kernel boundary: a wave whose envs finish their event loops early
//     starts observing while slower waves still simulate (the latency-bound event loop leaves VALU
//     issue slots that the VALU-bound observe fills) instead of the whole chip draining first;
//   - the reservoir records observe reads were written microseconds earlier by the same CU: L2
//     hits instead of a second HBM pass over the state.
// Same routines in the same order per env, so the same bits as the two-launch step (tested).
#include "lbsim_internal.h"
#include "lbsim_dyn_group.h"

namespace lbk {
namespace {

template <int G, int MAXS, int POLICY, bool TRACE>
__global__ void __launch_bounds__(64)
    fused_step_kernel(DevState st, SimParams p, const void* action, int action_dtype,
                      int32_t* assign_out, ObsOutputs out) {
  __shared__ union {
    DynGroupLds<POLICY> dyn;
    ObsScratch obs;
  } L;
  __shared__ float s_obs[MAXS * NF];
  __shared__ float s_act[MAXS];
  const int lane = (int)threadIdx.x;
  dyn_group_wave<G, kModeStep, POLICY, TRACE>(st, p, action, action_dtype, assign_out, nullptr,
                                              blockIdx.x, lane, L.dyn);
  __syncthreads();  // state stores complete and visible to this workgroup; LDS reused below
  constexpr int EPW = 64 / G;
  for (int i = 0; i < EPW; ++i) {
    const size_t b = (size_t)blockIdx.x * EPW + (size_t)i;
    if (b >= (size_t)p.B) break;
    observe_env_wave<MAXS>(st, p, out, b, L.obs, s_obs, s_act, lane);
  }
}

template <int G, int POLICY>
void launch_g(const LaunchCtx& L, const void* action, int dtype, int32_t* assign,
              const ObsOutputs& o, hipStream_t s) {
  constexpr int MAXS = G < 4 ? 4 : G;
  const dim3 block(64), grid((unsigned)((L.B + 64 / G - 1) / (64 / G)));
  if (L.prm.trace)
    hipLaunchKernelGGL((fused_step_kernel<G, MAXS, POLICY, true>), grid, block, 0, s, L.st, L.prm,
                       action, dtype, assign, o);
  else
    hipLaunchKernelGGL((fused_step_kernel<G, MAXS, POLICY, false>), grid, block, 0, s, L.st,
                       L.prm, action, dtype, assign, o);
}

template <int G>
void launch_pol(const LaunchCtx& L, const void* action, int dtype, int32_t* assign,
                const ObsOutputs& o, hipStream_t s) {
  switch (L.prm.policy) {
    case LBSIM_POLICY_SED: launch_g<G, 0>(L, action, dtype, assign, o, s); break;
    case LBSIM_POLICY_SED2: launch_g<G, 1>(L, action, dtype, assign, o, s); break;
    case LBSIM_POLICY_LSQ: launch_g<G, 2>(L, action, dtype, assign, o, s); break;
    case LBSIM_POLICY_LSQ2: launch_g<G, 3>(L, action, dtype, assign, o, s); break;
    default: launch_g<G, 4>(L, action, dtype, assign, o, s); break;
  }
}

}  // namespace

bool launch_fused_step(const LaunchCtx& L, int group_lanes, const void* action, int dtype,
                       int32_t* assign, const ObsOutputs& o, hipStream_t s) {
  switch (group_lanes) {
    case 2: launch_pol<2>(L, action, dtype, assign, o, s); return true;
    case 4: launch_pol<4>(L, action, dtype, assign, o, s); return true;
    case 8: launch_pol<8>(L, action, dtype, assign, o, s); return true;
    case 16: launch_pol<16>(L, action, dtype, assign, o, s); return true;
    default: return false;  // S > 16: the two-launch step
  }
}

}  // namespace lbk
