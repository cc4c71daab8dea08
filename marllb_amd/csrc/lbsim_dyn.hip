// lbsim_dyn.hip — dynamics launchers, one object per mode: built with
// -DLBSIM_DYN_MODE=0 (kModeStep, launch_dynamics_step) and =1 (kModeReset, launch_dynamics_reset)
// so the two halves of the template instantiations compile in parallel.
#include "lbsim_internal.h"
#include "lbsim_dyn_group.h"

#ifndef LBSIM_DYN_MODE
#error "build with -DLBSIM_DYN_MODE=0 (step) or 1 (reset)"
#endif

namespace lbk {
namespace {

constexpr int MODE = LBSIM_DYN_MODE == 0 ? kModeStep : kModeReset;

template <int MAXS, int POLICY>
void launch_dyn(const LaunchCtx& L, const void* action, int dtype, int32_t* assign,
                const uint8_t* mask, hipStream_t stream) {
  constexpr unsigned epb = 64u * kDynWaves<MAXS>;  // envs per workgroup (one per CU, kDynWaves)
  const dim3 block(epb), grid((unsigned)((L.B + epb - 1) / epb));
  if (L.prm.trace)
    hipLaunchKernelGGL((dynamics_kernel<MAXS, MODE, POLICY, true>), grid, block, 0, stream, L.st,
                       L.prm, action, dtype, assign, mask);
  else
    hipLaunchKernelGGL((dynamics_kernel<MAXS, MODE, POLICY, false>), grid, block, 0, stream, L.st,
                       L.prm, action, dtype, assign, mask);
}

// server per lane: G lanes per env, 64 / G envs per wave
template <int G, int POLICY>
void launch_dyn_group(const LaunchCtx& L, const void* action, int dtype, int32_t* assign,
                      const uint8_t* mask, hipStream_t stream) {
  constexpr int epw = 64 / G;
  const dim3 block(64), grid((unsigned)((L.B + epw - 1) / epw));
  if (L.prm.trace)
    hipLaunchKernelGGL((dynamics_group_kernel<G, MODE, POLICY, true>), grid, block, 0, stream,
                       L.st, L.prm, action, dtype, assign, mask);
  else
    hipLaunchKernelGGL((dynamics_group_kernel<G, MODE, POLICY, false>), grid, block, 0, stream,
                       L.st, L.prm, action, dtype, assign, mask);
}

template <int MAXS>
void launch_dyn_policy(const LaunchCtx& L, bool group, const void* action, int dtype,
                       int32_t* assign, const uint8_t* mask, hipStream_t s) {
  switch (L.prm.policy) {
#define LBSIM_POL(P)                                                  \
  if (group) launch_dyn_group<MAXS, P>(L, action, dtype, assign, mask, s); \
  else launch_dyn<MAXS, P>(L, action, dtype, assign, mask, s);        \
  break;
    case LBSIM_POLICY_SED: LBSIM_POL(0)
    case LBSIM_POLICY_SED2: LBSIM_POL(1)
    case LBSIM_POLICY_LSQ: LBSIM_POL(2)
    case LBSIM_POLICY_LSQ2: LBSIM_POL(3)
    default: LBSIM_POL(4)
#undef LBSIM_POL
  }
}

// A group width chosen apart from MAXS: the small-batch 8-lane tier (S <= 4), a forced
// LBSIM_DYN_GROUP_LANES width, and S > 16 (32 or 64 lanes per env, server-per-lane only: the
// env-per-lane kernel keeps its per-server state in registers / LDS rows sized for <= 16 servers).
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

// Lanes per env of the server-per-lane mapping: LBSIM_DYN_GROUP_LANES = 4 | 8 | 16 | 32 | 64
// forces the group width (>= S; lanes past S hold no server and only draw arrivals ahead): tests
// use 4 to run the headline 4-lane kernel on small batches, experiments the wider forms.
int forced_group_lanes() {
  static const int g = [] {
    const char* s = std::getenv("LBSIM_DYN_GROUP_LANES");
    return s ? std::atoi(s) : 0;
  }();
  return g;
}

// Mapping choice (LBSIM_DYN_AUTO): one lane per server.  With arrivals drawn G at a
// time (lbsim_dyn_group.h) it is faster than one lane per env at every measured shape
// (profiles/r02_round2/mapping_sweep.jsonl): 65536 x 4 0.182 vs 0.214 ms, 131072 x 4 0.316 vs
// 0.402, 65536 x 8 0.267 vs 0.320, configs[2] trace replay 0.317 vs 0.381, 16384 x 4 0.117 vs
// 0.198.  The env-per-lane kernel stays selectable (LBSIM_DYN_ENV_PER_LANE).
void launch_dynamics_t(const LaunchCtx& L, const void* action, int dtype, int32_t* assign,
                       const uint8_t* mask, hipStream_t stream) {
  const bool g = L.dyn_mapping != LBSIM_DYN_ENV_PER_LANE;
  const int fg = g ? forced_group_lanes() : 0;
  if (fg >= L.S && (fg == 4 || fg == 8 || fg == 16 || fg == 32 || fg == 64)) {
    if (fg == 4) launch_dyn_group_policy<4>(L, action, dtype, assign, mask, stream);
    else if (fg == 8) launch_dyn_group_policy<8>(L, action, dtype, assign, mask, stream);
    else if (fg == 16) launch_dyn_group_policy<16>(L, action, dtype, assign, mask, stream);
    else if (fg == 32) launch_dyn_group_policy<32>(L, action, dtype, assign, mask, stream);
    else launch_dyn_group_policy<64>(L, action, dtype, assign, mask, stream);
  } else if (g && L.S <= 2) launch_dyn_group_policy<2>(L, action, dtype, assign, mask, stream);
  // small batches (configs[1]: 4096 x 4): 8 lanes per env when 4-lane groups would give at most
  // one wave per two SIMDs (B * 4 / 64 <= simds / 2: B <= 8192 on 256 CUs) -- twice the waves for
  // SIMDs that would sit idle, the draw-ahead spread over 8 lanes: 4096 x 4 0.0908 -> 0.0894 ms,
  // 8192 x 4 0.0962 -> 0.0947 (profiles/r02_round2b/ab_group_lanes_small.txt); slower from 16384
  else if (g && L.S <= 4 && (int64_t)L.B * 4 / 64 <= L.simds / 2)
    launch_dyn_group_policy<8>(L, action, dtype, assign, mask, stream);
  else if (L.S <= 4) launch_dyn_policy<4>(L, g, action, dtype, assign, mask, stream);
  else if (L.S <= 8) launch_dyn_policy<8>(L, g, action, dtype, assign, mask, stream);
  else if (L.S <= 16) launch_dyn_policy<16>(L, g, action, dtype, assign, mask, stream);
  else if (L.S <= 32) launch_dyn_group_policy<32>(L, action, dtype, assign, mask, stream);
  else launch_dyn_group_policy<64>(L, action, dtype, assign, mask, stream);
}

}  // namespace

#if LBSIM_DYN_MODE == 0
void launch_dynamics_step(const LaunchCtx& L, const void* action, int dtype, int32_t* assign,
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
