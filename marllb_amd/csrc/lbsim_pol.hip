// lbsim_pol.hip — launchers of the one-kernel policy networks (lbsim_fused.h).
#include "lbsim_internal.h"
#include "lbsim_fused.h"

namespace lbk {
namespace {

template <typename Args>
int launch_fused(void (*kern)(Args), int64_t B, int mt, size_t lds, hipStream_t s, Args a,
                 unsigned threads = 256) {
  const void* f = reinterpret_cast<const void*>(kern);
  if (lds > 65536 &&
      hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds) != hipSuccess)
    return LBSIM_EDEVICE;
  void* args[] = {&a};
  const dim3 grid((unsigned)((B + 16 * mt - 1) / (16 * mt))), block(threads);
  return hipLaunchKernel(f, grid, block, args, lds, s) == hipSuccess ? LBSIM_OK : LBSIM_EDEVICE;
}

}  // namespace

int launch_sac_actor(SacActorArgs& a, int64_t B, int mt, size_t lds, hipStream_t s) {
  if (mt == 4) return launch_fused(&sac_actor_kernel<4, 128, 256>, B, 4, lds, s, a);
  if (mt == 2) return launch_fused(&sac_actor_kernel<2, 128, 256>, B, 2, lds, s, a);
  return launch_fused(&sac_actor_kernel<1, 128, 256>, B, 1, lds, s, a);
}

// form: 0 = layer-split tile kernel (mt = 1 | 2 | 4), 1 = one wave per agent, 2 = two waves per
// agent (8-wave workgroups, A = 4)
int launch_qmix_policy(QmixArgs& a, int64_t B, int form, int mt, size_t lds, hipStream_t s) {
  if (form == 2) return launch_fused(&qmix_agent_pair_kernel<64, 128>, B, 1, lds, s, a, 512);
  if (form == 1) return launch_fused(&qmix_agent_wave_kernel<64, 128>, B, 1, lds, s, a);
  if (mt == 4) return launch_fused(&qmix_policy_kernel<4, 64, 128>, B, 4, lds, s, a);
  if (mt == 2) return launch_fused(&qmix_policy_kernel<2, 64, 128>, B, 2, lds, s, a);
  return launch_fused(&qmix_policy_kernel<1, 64, 128>, B, 1, lds, s, a);
}

}  // namespace lbk

#if LBSIM_EXP_PHASES
// timing diagnostic (lbsim_fused.h LB_PHASE): the last policy launch's phase clocks, 64 x 16 u64
extern "C" int lbsim_exp_phase_read(unsigned long long* out) {
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(lbk::lbsim_exp_ts), sizeof(lbk::lbsim_exp_ts)) ==
                 hipSuccess
             ? 0
             : -1;
}
#endif
