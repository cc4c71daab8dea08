// lbsim_obs.hip — observe launchers: one wave per 4-server chunk, the chunks of an
// env in one workgroup, each with its own ObsScratch in dynamic LDS.
#include "lbsim_internal.h"

namespace lbk {
namespace {

template <int MODE>
void launch_observe_t(const LaunchCtx& L, const ObsOutputs& o, const uint8_t* mask,
                      hipStream_t stream) {
  const int nw = (L.S + kObsChunk - 1) / kObsChunk;
  const dim3 grid((unsigned)L.B), block((unsigned)(64 * nw));
  const size_t lds = (size_t)nw * sizeof(ObsScratch);
  if (lds > 65536) {  // S > 32: 9-16 chunk waves
    static const bool ok = hipFuncSetAttribute(
        reinterpret_cast<const void*>(&observe_kernel<64, MODE>),
        hipFuncAttributeMaxDynamicSharedMemorySize, 16 * (int)sizeof(ObsScratch)) == hipSuccess;
    (void)ok;
  }
  if (L.S <= 4)
    hipLaunchKernelGGL((observe_kernel<4, MODE>), grid, block, lds, stream, L.st, L.prm, o, mask);
  else if (L.S <= 8)
    hipLaunchKernelGGL((observe_kernel<8, MODE>), grid, block, lds, stream, L.st, L.prm, o, mask);
  else if (L.S <= 16)
    hipLaunchKernelGGL((observe_kernel<16, MODE>), grid, block, lds, stream, L.st, L.prm, o, mask);
  else
    hipLaunchKernelGGL((observe_kernel<64, MODE>), grid, block, lds, stream, L.st, L.prm, o, mask);
}

}  // namespace

void launch_observe_step(const LaunchCtx& L, const ObsOutputs& o, const uint8_t* mask,
                         hipStream_t s) {
  launch_observe_t<kModeStep>(L, o, mask, s);
}

void launch_observe_reset(const LaunchCtx& L, const ObsOutputs& o, const uint8_t* mask,
                          hipStream_t s) {
  launch_observe_t<kModeReset>(L, o, mask, s);
}

}  // namespace lbk
