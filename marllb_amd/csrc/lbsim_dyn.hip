// lbsim_dyn.hip — dynamics launchers, one object per mode: built with
// -DLBSIM_DYN_MODE=0 (kModeStep, launch_dynamics_step), =1 (kModeReset, launch_dynamics_reset)
// and =2 (kModeStepNR, launch_dynamics_step_nr: the step of a next-step auto-reset handle) so the
// thirds of the template instantiations compile in parallel.
#include "lbsim_internal.h"
#include "lbsim_dyn_group.h"
#include "lbsim_dyn_wave.h"

#ifndef LBSIM_DYN_MODE
#error "build with -DLBSIM_DYN_MODE=0 (step), 1 (reset) or 2 (step with next-step resets)"
#endif

namespace lbk {
namespace {

constexpr int MODE = LBSIM_DYN_MODE == 0 ? kModeStep : (LBSIM_DYN_MODE == 1 ? kModeReset : kModeStepNR);

template <int MAXS, int POLICY>
void launch_dyn(const LaunchCtx& L, const void* action, int dtype, int32_t* assign,
                const uint8_t* mask, hipStream_t stream) {
  constexpr unsigned epb = 64u * kDynWaves<MAXS>;  // envs per workgroup (one per CU, kDynWaves)
  const dim3 block(epb), grid((unsigned)((L.B + epb - 1) / epb));
  if (L.prm.trace)
    LBSIM_LAUNCH((dynamics_kernel<MAXS, MODE, POLICY, true>), grid, block, 0, stream, L.st,
                       L.prm, action, dtype, assign, mask);
  else
    LBSIM_LAUNCH((dynamics_kernel<MAXS, MODE, POLICY, false>), grid, block, 0, stream, L.st,
                       L.prm, action, dtype, assign, mask);
}

// server per lane: G lanes per env, 64 / G envs per wave
template <int G, int POLICY>
void launch_dyn_group(const LaunchCtx& L, const void* action, int dtype, int32_t* assign,
                      const uint8_t* mask, hipStream_t stream) {
  // envs per wave: 64 / G; LBSIM_DYN_EPW (1 .. 64 / G) runs fewer per wave, more waves
  static const int forced_epw = [] {
    const char* e = std::getenv("LBSIM_DYN_EPW");
    return e ? std::atoi(e) : 0;
  }();
  const int epw = (forced_epw >= 1 && forced_epw <= 64 / G) ? forced_epw : 64 / G;
  SimParams prm = L.prm;
  prm.dyn_epw = epw;
  const dim3 block(64), grid((unsigned)((L.B + epw - 1) / epw));
  // a full handle (n_flow_on_mode VPP, a duration plane, lost-FIN deferral, reservoir_mode VPP):
  // the kernel with every feature's code (group_event_loop FULL), its own register budget
  if (L.prm.leak || L.st.res_dur != nullptr || L.prm.res_vpp) {
    if (L.prm.trace)
      LBSIM_LAUNCH((dynamics_group_full_kernel<G, MODE, POLICY, true>), grid, block, 0, stream,
                   L.st, prm, action, dtype, assign, mask);
    else
      LBSIM_LAUNCH((dynamics_group_full_kernel<G, MODE, POLICY, false>), grid, block, 0, stream,
                   L.st, prm, action, dtype, assign, mask);
    return;
  }
  // the step of a next-step auto-reset handle inlines the event loop twice (the reset's warm-up
  // and the step): unconstrained it took 133-137 VGPRs, 3 waves per SIMD, and ran 190 us against
  // the plain step's 149 at 65536 x 4 (profiles/r06b/modes): held to the 4-wave budget
  if constexpr (MODE == kModeStepNR) {
    if (L.prm.trace)
      LBSIM_LAUNCH((dynamics_group_kernel<G, MODE, POLICY, true, 4>), grid, block, 0, stream,
                   L.st, prm, action, dtype, assign, mask);
    else
      LBSIM_LAUNCH((dynamics_group_kernel<G, MODE, POLICY, false, 4>), grid, block, 0, stream,
                   L.st, prm, action, dtype, assign, mask);
    return;
  }
  // a step grid of more than 4 waves per SIMD: the 5-wave register budget (SED, 4 / 8 lanes)
  if constexpr (MODE == kModeStep && POLICY == 0 && (G == 4 || G == 8)) {
    if ((int64_t)grid.x > 4 * (int64_t)L.simds) {
      if (L.prm.trace)
        LBSIM_LAUNCH((dynamics_group_kernel<G, MODE, POLICY, true, 5>), grid, block, 0,
                           stream, L.st, prm, action, dtype, assign, mask);
      else
        LBSIM_LAUNCH((dynamics_group_kernel<G, MODE, POLICY, false, 5>), grid, block, 0,
                           stream, L.st, prm, action, dtype, assign, mask);
      return;
    }
  }
  if (L.prm.trace)
    LBSIM_LAUNCH((dynamics_group_kernel<G, MODE, POLICY, true>), grid, block, 0, stream,
                       L.st, prm, action, dtype, assign, mask);
  else
    LBSIM_LAUNCH((dynamics_group_kernel<G, MODE, POLICY, false>), grid, block, 0, stream,
                       L.st, prm, action, dtype, assign, mask);
}

template <int MAXS>
void launch_dyn_policy(const LaunchCtx& L, bool, const void* action, int dtype, int32_t* assign,
                       const uint8_t* mask, hipStream_t s) {
  switch (L.prm.policy) {
    case LBSIM_POLICY_SED: launch_dyn<MAXS, 0>(L, action, dtype, assign, mask, s); break;
    case LBSIM_POLICY_SED2: launch_dyn<MAXS, 1>(L, action, dtype, assign, mask, s); break;
    case LBSIM_POLICY_LSQ: launch_dyn<MAXS, 2>(L, action, dtype, assign, mask, s); break;
    case LBSIM_POLICY_LSQ2: launch_dyn<MAXS, 3>(L, action, dtype, assign, mask, s); break;
    default: launch_dyn<MAXS, 4>(L, action, dtype, assign, mask, s); break;
  }
}

// G lanes per env (dyn_group_lanes): 2, 4, 8, 16, and 32 / 64 for S > 16 (server-per-lane only:
// the env-per-lane kernel keeps its per-server state in registers / LDS rows sized for <= 16).
template <int G>
void launch_dyn_group_policy(const LaunchCtx& L, const void* action, int dtype, int32_t* assign,
                             const uint8_t* mask, hipStream_t s) {
  switch (L.prm.policy) {
    case LBSIM_POLICY_SED: launch_dyn_group<G, 0>(L, action, dtype, assign, mask, s); break;
    case LBSIM_POLICY_SED2: launch_dyn_group<G, 1>(L, action, dtype, assign, mask, s); break;
    case LBSIM_POLICY_LSQ: launch_dyn_group<G, 2>(L, action, dtype, assign, mask, s); break;
    case LBSIM_POLICY_LSQ2: launch_dyn_group<G, 3>(L, action, dtype, assign, mask, s); break;
    default: launch_dyn_group<G, 4>(L, action, dtype, assign, mask, s); break;
  }
}

// one wave per env: NG ring registers, two servers of 32 positions each
template <int NR, int POLICY>
void launch_dyn_wave(const LaunchCtx& L, const void* action, int dtype, int32_t* assign,
                     const uint8_t* mask, hipStream_t stream) {
  const dim3 block(64), grid((unsigned)L.B);
  if (L.prm.trace)
    LBSIM_LAUNCH((dynamics_wave_kernel<NR, MODE, POLICY, true>), grid, block, 0, stream,
                       L.st, L.prm, action, dtype, assign, mask);
  else
    LBSIM_LAUNCH((dynamics_wave_kernel<NR, MODE, POLICY, false>), grid, block, 0, stream,
                       L.st, L.prm, action, dtype, assign, mask);
}

template <int NR>
void launch_dyn_wave_policy(const LaunchCtx& L, const void* action, int dtype, int32_t* assign,
                            const uint8_t* mask, hipStream_t s) {
  switch (L.prm.policy) {
    case LBSIM_POLICY_SED: launch_dyn_wave<NR, 0>(L, action, dtype, assign, mask, s); break;
    case LBSIM_POLICY_SED2: launch_dyn_wave<NR, 1>(L, action, dtype, assign, mask, s); break;
    case LBSIM_POLICY_LSQ: launch_dyn_wave<NR, 2>(L, action, dtype, assign, mask, s); break;
    default: launch_dyn_wave<NR, 3>(L, action, dtype, assign, mask, s); break;
  }
}

// Mapping choice (LBSIM_DYN_AUTO): one lane per server.  With arrivals drawn G at a
// time (lbsim_dyn_group.h) it is faster than one lane per env at every measured shape
// (profiles/r02_round2/mapping_sweep.jsonl): 65536 x 4 0.182 vs 0.214 ms, 131072 x 4 0.316 vs
// 0.402, 65536 x 8 0.267 vs 0.320, configs[2] trace replay 0.317 vs 0.381, 16384 x 4 0.117 vs
// 0.198.  The env-per-lane kernel stays selectable (LBSIM_DYN_ENV_PER_LANE).  Group widths:
// dyn_group_lanes (lbsim_internal.h).
void launch_dynamics_t(const LaunchCtx& L, const void* action, int dtype, int32_t* assign,
                       const uint8_t* mask, hipStream_t stream) {
  if (dyn_wave_ok(L)) {
    if (L.S <= 2) launch_dyn_wave_policy<1>(L, action, dtype, assign, mask, stream);
    else if (L.S <= 4) launch_dyn_wave_policy<2>(L, action, dtype, assign, mask, stream);
    else launch_dyn_wave_policy<4>(L, action, dtype, assign, mask, stream);
    return;
  }
  switch (dyn_group_lanes(L)) {
    case 0:  // one lane per env
      if (L.S <= 4) launch_dyn_policy<4>(L, false, action, dtype, assign, mask, stream);
      else if (L.S <= 8) launch_dyn_policy<8>(L, false, action, dtype, assign, mask, stream);
      else launch_dyn_policy<16>(L, false, action, dtype, assign, mask, stream);
      break;
    case 2: launch_dyn_group_policy<2>(L, action, dtype, assign, mask, stream); break;
    case 4: launch_dyn_group_policy<4>(L, action, dtype, assign, mask, stream); break;
    case 8: launch_dyn_group_policy<8>(L, action, dtype, assign, mask, stream); break;
    case 16: launch_dyn_group_policy<16>(L, action, dtype, assign, mask, stream); break;
    case 32: launch_dyn_group_policy<32>(L, action, dtype, assign, mask, stream); break;
    default: launch_dyn_group_policy<64>(L, action, dtype, assign, mask, stream); break;
  }
}

}  // namespace

#if LBSIM_DYN_MODE == 0
void launch_dynamics_step(const LaunchCtx& L, const void* action, int dtype, int32_t* assign,
                          const uint8_t* mask, hipStream_t s) {
  launch_dynamics_t(L, action, dtype, assign, mask, s);
}
#elif LBSIM_DYN_MODE == 2
void launch_dynamics_step_nr(const LaunchCtx& L, const void* action, int dtype, int32_t* assign,
                             const uint8_t* mask, hipStream_t s) {
  launch_dynamics_t(L, action, dtype, assign, mask, s);
}
#else
void launch_dynamics_reset(const LaunchCtx& L, const void* action, int dtype, int32_t* assign,
                           const uint8_t* mask, hipStream_t s) {
  launch_dynamics_t(L, action, dtype, assign, mask, s);
}
#endif

}  // namespace lbk
