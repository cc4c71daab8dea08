// lbsim_internal.h — host-side glue between the extern "C" API (lbsim_api.hip) and the translation
// units that instantiate the templated kernels (compiled in parallel, linked into liblbsim.so):
//
//   lbsim_dyn.hip      dynamics_kernel / dynamics_group_kernel launchers; built twice
//                      (-DLBSIM_DYN_MODE=0: step, 1: reset)
//   lbsim_obs.hip      observe_kernel launchers
//   lbsim_pol.hip      one-kernel policy networks (lbsim_fused.h)
//
// Non-template kernels live only in lbsim_api.hip (a __global__ defined in two objects would be
// defined twice); templates are instantiated where they are launched.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdlib>

#include "../../include/lbsim.h"
#include "lbsim_kernels.h"

namespace lbk {

// Launch log: every kernel launch of the library goes through LBSIM_LAUNCH, which records the
// launched kernel's host stub for the API call in progress (lbsim_launch_names resolves the stubs
// to their names afterwards, off the step path).  bench.py keys its committed PMC counter files by
// these names, so counters of a kernel that did not run are never attached to a measurement.
void note_launch(const void* host_fn);
#define LBSIM_LAUNCH(KERNEL, GRID, BLOCK, LDS, STREAM, ...)                 \
  do {                                                                    \
    ::lbk::note_launch(reinterpret_cast<const void*>(&KERNEL));           \
    hipLaunchKernelGGL(KERNEL, GRID, BLOCK, LDS, STREAM, __VA_ARGS__);    \
  } while (0)

// What a launcher needs of a handle.
struct LaunchCtx {
  DevState st;
  SimParams prm;
  int B, S;
  int simds;        // SIMDs of the device (CUs x 4)
  int dyn_mapping;  // lbsim_dyn_mapping
};

// Lanes per env of the server-per-lane dynamics (0: one lane per env, dyn_mapping ENV_PER_LANE).
// LBSIM_DYN_GROUP_LANES = 4 | 8 | 16 | 32 | 64 forces the width (>= S; lanes past S hold no server
// and only draw arrivals ahead): tests use 4 to run the headline 4-lane kernel on small batches,
// experiments the wider forms.  Otherwise pow2 >= S, except small batches with S <= 4: 8 lanes
// when 4-lane groups would give at most one wave per two SIMDs (B * 4 / 64 <= simds / 2: B <= 8192
// on 256 CUs) -- twice the waves for SIMDs that would sit idle, the draw-ahead spread over 8
// lanes: 4096 x 4 0.0908 -> 0.0894 ms, 8192 x 4 0.0962 -> 0.0947
// (profiles/r02_round2b/ab_group_lanes_small.txt); slower from 16384 envs on.
inline int dyn_group_lanes(const LaunchCtx& L) {
  // (split lost-FIN handles and reservoir_mode VPP run the server-per-lane kernel only)
  if (L.dyn_mapping == LBSIM_DYN_ENV_PER_LANE && L.S <= 16 && !L.prm.split && !L.prm.res_vpp)
    return 0;
  static const int forced = [] {
    const char* e = std::getenv("LBSIM_DYN_GROUP_LANES");
    return e ? std::atoi(e) : 0;
  }();
  if (forced >= L.S && (forced == 4 || forced == 8 || forced == 16 || forced == 32 || forced == 64))
    return forced;
  if (L.S <= 2) return 2;
  if (L.S <= 4) return (int64_t)L.B * 4 / 64 <= L.simds / 2 ? 8 : 4;
  int g = 8;
  while (g < L.S) g <<= 1;
  return g;
}

// One wave per env (lbsim_dyn_wave.h): S <= 8, Q <= 32, SED / SED2 / LSQ / LSQ2, the default
// mapping, and a batch small enough that one env's event-loop chain, not issue throughput, sets
// the step time: at most 4 waves (envs) per SIMD for S <= 4 (B <= 4096 on 256 CUs), 2 for S <= 8.
// Measured dynamics, wave vs server-per-lane groups (profiles/r03w/wave_sweep*.txt): S = 4 1024
// envs 0.041 vs 0.084 ms, 4096 0.066 vs 0.090, 8192 0.108 vs 0.095 (8 waves per SIMD:
// issue-bound, the groups win); S = 8 2048 envs 0.058 vs 0.078, 4096 0.087 vs 0.083.
// LBSIM_DYN_WAVE_MAX_B overrides the limit; LBSIM_DYN_WAVE = 0 disables the kernel, 1 uses it at
// every batch size it applies to; a forced LBSIM_DYN_GROUP_LANES width wins over both.
inline int dyn_wave_mode() {
  static const int mode = [] {
    const char* e = std::getenv("LBSIM_DYN_WAVE");
    return e ? std::atoi(e) : -1;
  }();
  return mode;
}

// Whether the wave dynamics can serve this handle at all (batch size aside).
inline bool dyn_wave_fits(const LaunchCtx& L) {
  static const bool forced_lanes = std::getenv("LBSIM_DYN_GROUP_LANES") != nullptr;
  if (dyn_wave_mode() == 0 || forced_lanes || L.dyn_mapping == LBSIM_DYN_ENV_PER_LANE) return false;
  if (L.S > 8 || L.prm.Q > 32 || L.prm.policy == LBSIM_POLICY_ALIAS) return false;
  // server failures, n_flow_on_mode VPP's lost-flow counts: the group / env-lane kernels; lost-FIN
  // deferral (split reservoirs, pending guesses) and reservoir_mode VPP: the group kernel
  return L.prm.fail_thr == 0u && L.prm.leak == 0 && L.prm.split == 0 && L.prm.res_vpp == 0;
}

inline bool dyn_wave_ok(const LaunchCtx& L) {
  static const int64_t max_b = [] {
    const char* e = std::getenv("LBSIM_DYN_WAVE_MAX_B");
    return e ? (int64_t)std::atoll(e) : (int64_t)-1;
  }();
  if (!dyn_wave_fits(L)) return false;
  const int mode = dyn_wave_mode();
  const int64_t per_simd = L.S <= 4 ? 4 : 2;  // S = 8: 2048 envs 0.058 vs 0.078 ms, 4096 0.087 vs 0.083
  return mode == 1 || (int64_t)L.B <= (max_b >= 0 ? max_b : per_simd * (int64_t)L.simds);
}

// Dynamics of one step (mode kModeStep) or of a reset with warm-up (kModeReset).
void launch_dynamics_step(const LaunchCtx& L, const void* action, int dtype, int32_t* assign,
                          const uint8_t* mask, hipStream_t s);
void launch_dynamics_reset(const LaunchCtx& L, const void* action, int dtype, int32_t* assign,
                           const uint8_t* mask, hipStream_t s);
// The step of a next-step auto-reset handle (kModeStepNR): envs done last step reset instead.
void launch_dynamics_step_nr(const LaunchCtx& L, const void* action, int dtype, int32_t* assign,
                             const uint8_t* mask, hipStream_t s);

void launch_observe_step(const LaunchCtx& L, const ObsOutputs& o, const uint8_t* mask,
                         hipStream_t s);
void launch_observe_reset(const LaunchCtx& L, const ObsOutputs& o, const uint8_t* mask,
                          hipStream_t s);

struct SacActorArgs;
struct QmixArgs;
// The fused dynamics + observe step (lbsim_step.hip) for the group width of dyn_group_lanes;
// false when that width has no fused form (S > 16, one lane per env): use the two launches.
bool launch_fused_step(const LaunchCtx& L, int group_lanes, const void* action, int dtype,
                       int32_t* assign, const ObsOutputs& o, hipStream_t s);

// The one-launch small-batch step (lbsim_step.hip): dynamics_wave then observe per env; only for
// a handle with dyn_wave_ok.
void launch_step_wave(const LaunchCtx& L, const void* action, int dtype, int32_t* assign,
                      const ObsOutputs& o, hipStream_t s);

// the fused policy kernels (lbsim_pol.hip): LBSIM_OK / LBSIM_EDEVICE / LBSIM_ENOTSUP
int launch_sac_actor(SacActorArgs& a, int64_t B, int mt, size_t lds, hipStream_t s);
int launch_qmix_policy(QmixArgs& a, int64_t B, int form, int mt, size_t lds, hipStream_t s);

}  // namespace lbk
