// lbsim_step.hip — the fused steps: one launch per step runs a wave's dynamics and then observes
// the same envs ("fused step").  step_wave_kernel (one wave per env, the default
// for small S <= 4 batches) is below; fused_step_kernel (server-per-lane groups, opt-in):
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
#include "lbsim_dyn_wave.h"


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

// The small-batch step (dyn_wave_fits: S <= 8, at most 4 envs per SIMD): one wave per env steps it
// (dyn_wave_env) and then observes it (observe_env_wave: one chunk for S <= 4, two for 5-8), so the
// step is ONE launch and each env's observation runs as soon as its own event loop ends, while
// slower envs still simulate.  Same routines, same order: the same bits as the two launches.
// OCC waves per SIMD.  2: batches of at most 2 envs per SIMD, with the VALU queue counts (the
// shorter chain).  4: 2-4 envs per SIMD, with the scalar counts (profiles/r03w/ab_step_wave_fused.txt).
// Both take 118-120 VGPRs with no spill since the one-chunk observe is straight-line code (the
// chunk loop took 194 and spilled 64 under the 128 cap: profiles/r03o/).  Out of line, the observe
// phase's call frames went through 1 KB of scratch per lane (0.141 ms).
// MAXS = 8 (S = 5-8): the wave dynamics' S <= 8 form, then both chunks, one after the other, in a
// rolled loop whose inputs are opaque to the compiler (observe_env_wave), so that no chunk-invariant
// value is held across the two: 124 VGPRs, no scratch, hence OCC 4 too (hoisted, 170 and 184 B of
// spills per lane at the 128 cap).
template <int NG, int POLICY, bool TRACE, int OCC, int MAXS = kObsChunk>
__global__ void __launch_bounds__(64, OCC)
    step_wave_kernel(DevState st, SimParams p, const void* action, int action_dtype,
                     int32_t* assign_out, ObsOutputs out) {
  __shared__ union {
    WaveLds dyn;
    ObsScratch obs;
  } L;
  __shared__ float s_obs[MAXS * NF];
  __shared__ float s_act[MAXS];
  const int lane = (int)threadIdx.x;
  if (!dyn_wave_env<NG, kModeStep, POLICY, TRACE, OCC == 2>(st, p, action, action_dtype,
                                                            assign_out, nullptr, blockIdx.x, lane,
                                                            L.dyn))
    return;
  __syncthreads();  // state stores complete and visible to this workgroup; LDS reused below
  observe_env_wave<MAXS>(st, p, out, blockIdx.x, L.obs, s_obs, s_act, lane);
}

template <int NG, int POLICY, int OCC>
void launch_wo(const LaunchCtx& L, const void* action, int dtype, int32_t* assign,
               const ObsOutputs& o, hipStream_t s) {
  const dim3 block(64), grid((unsigned)L.B);
  if constexpr (NG == 4) {  // S = 5-8: both chunks
    if (L.prm.trace)
      LBSIM_LAUNCH((step_wave_kernel<4, POLICY, true, OCC, 8>), grid, block, 0, s, L.st, L.prm,
                   action, dtype, assign, o);
    else
      LBSIM_LAUNCH((step_wave_kernel<4, POLICY, false, OCC, 8>), grid, block, 0, s, L.st, L.prm,
                   action, dtype, assign, o);
  } else {
    if (L.prm.trace)
      LBSIM_LAUNCH((step_wave_kernel<NG, POLICY, true, OCC>), grid, block, 0, s, L.st, L.prm,
                   action, dtype, assign, o);
    else
      LBSIM_LAUNCH((step_wave_kernel<NG, POLICY, false, OCC>), grid, block, 0, s, L.st, L.prm,
                   action, dtype, assign, o);
  }
}

// OCC 2 up to 2 envs per SIMD, else 4; LBSIM_STEP_WAVE_OCC = 2 | 4 forces one form at every
// batch size (the parity tests run the OCC-4 kernel that serves 2-4 envs per SIMD -- BASELINE
// configs[1]'s 4096 x 4 -- on every small-batch case).
template <int NG, int POLICY>
void launch_w(const LaunchCtx& L, const void* action, int dtype, int32_t* assign,
              const ObsOutputs& o, hipStream_t s) {
  static const int forced = [] {
    const char* e = std::getenv("LBSIM_STEP_WAVE_OCC");
    return e ? std::atoi(e) : 0;
  }();
  const bool occ2 = forced == 2 || (forced != 4 && (int64_t)L.B <= 2 * (int64_t)L.simds);
  if (occ2) launch_wo<NG, POLICY, 2>(L, action, dtype, assign, o, s);
  else launch_wo<NG, POLICY, 4>(L, action, dtype, assign, o, s);
}

template <int NG>
void launch_wpol(const LaunchCtx& L, const void* action, int dtype, int32_t* assign,
                 const ObsOutputs& o, hipStream_t s) {
  switch (L.prm.policy) {
    case LBSIM_POLICY_SED: launch_w<NG, 0>(L, action, dtype, assign, o, s); break;
    case LBSIM_POLICY_SED2: launch_w<NG, 1>(L, action, dtype, assign, o, s); break;
    case LBSIM_POLICY_LSQ: launch_w<NG, 2>(L, action, dtype, assign, o, s); break;
    default: launch_w<NG, 3>(L, action, dtype, assign, o, s); break;
  }
}

template <int G, int POLICY>
void launch_g(const LaunchCtx& L, const void* action, int dtype, int32_t* assign,
              const ObsOutputs& o, hipStream_t s) {
  constexpr int MAXS = G < 4 ? 4 : G;
  const dim3 block(64), grid((unsigned)((L.B + 64 / G - 1) / (64 / G)));
  if (L.prm.trace)
    LBSIM_LAUNCH((fused_step_kernel<G, MAXS, POLICY, true>), grid, block, 0, s, L.st, L.prm,
                       action, dtype, assign, o);
  else
    LBSIM_LAUNCH((fused_step_kernel<G, MAXS, POLICY, false>), grid, block, 0, s, L.st,
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

void launch_step_wave(const LaunchCtx& L, const void* action, int dtype, int32_t* assign,
                      const ObsOutputs& o, hipStream_t s) {
  if (L.S <= 2) launch_wpol<1>(L, action, dtype, assign, o, s);
  else if (L.S <= 4) launch_wpol<2>(L, action, dtype, assign, o, s);
  else launch_wpol<4>(L, action, dtype, assign, o, s);
}

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
