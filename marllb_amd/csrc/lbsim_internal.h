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

#include "../../include/lbsim.h"
#include "lbsim_kernels.h"

namespace lbk {

// What a launcher needs of a handle.
struct LaunchCtx {
  DevState st;
  SimParams prm;
  int B, S;
  int simds;        // SIMDs of the device (CUs x 4)
  int dyn_mapping;  // lbsim_dyn_mapping
};

// Dynamics of one step (mode kModeStep) or of a reset with warm-up (kModeReset).
void launch_dynamics_step(const LaunchCtx& L, const void* action, int dtype, int32_t* assign,
                          const uint8_t* mask, hipStream_t s);
void launch_dynamics_reset(const LaunchCtx& L, const void* action, int dtype, int32_t* assign,
                           const uint8_t* mask, hipStream_t s);

void launch_observe_step(const LaunchCtx& L, const ObsOutputs& o, const uint8_t* mask,
                         hipStream_t s);
void launch_observe_reset(const LaunchCtx& L, const ObsOutputs& o, const uint8_t* mask,
                          hipStream_t s);

struct SacActorArgs;
struct QmixArgs;
// the fused policy kernels (lbsim_pol.hip): LBSIM_OK / LBSIM_EDEVICE / LBSIM_ENOTSUP
int launch_sac_actor(SacActorArgs& a, int64_t B, int mt, size_t lds, hipStream_t s);
int launch_qmix_policy(QmixArgs& a, int64_t B, int form, int mt, size_t lds, hipStream_t s);

}  // namespace lbk
