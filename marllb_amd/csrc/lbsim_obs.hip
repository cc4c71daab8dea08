// lbsim_obs.hip — observe launchers: one wave per 4-server chunk, the chunks of an
// env in one workgroup, each with its own ObsScratch in dynamic LDS.
#include <cstdlib>
#include <cstring>

#include "lbsim_internal.h"

namespace lbk {
namespace {

template <int MODE, bool FAC>
void launch_observe_t(const LaunchCtx& L, const ObsOutputs& o, const uint8_t* mask,
                      hipStream_t stream) {
  const int nw = (L.S + kObsChunk - 1) / kObsChunk;
  const dim3 grid((unsigned)L.B), block((unsigned)(64 * nw));
  const size_t lds = (size_t)nw * sizeof(ObsScratch);
  if (lds > 65536) {  // S > 32: 9-16 chunk waves
    static const bool ok = hipFuncSetAttribute(
        reinterpret_cast<const void*>(&observe_kernel<64, MODE, FAC>),
        hipFuncAttributeMaxDynamicSharedMemorySize, 16 * (int)sizeof(ObsScratch)) == hipSuccess;
    (void)ok;
  }
  if (L.S <= 4)
    LBSIM_LAUNCH((observe_kernel<4, MODE, FAC>), grid, block, lds, stream, L.st, L.prm, o,
                       mask);
  else if (L.S <= 8)
    LBSIM_LAUNCH((observe_kernel<8, MODE, FAC>), grid, block, lds, stream, L.st, L.prm, o,
                       mask);
  else if (L.S <= 16)
    LBSIM_LAUNCH((observe_kernel<16, MODE, FAC>), grid, block, lds, stream, L.st, L.prm, o,
                       mask);
  else
    LBSIM_LAUNCH((observe_kernel<64, MODE, FAC>), grid, block, lds, stream, L.st, L.prm, o,
                       mask);
}

// Envs of more than LBSIM_OBSERVE_SPLIT_S servers (default 16) observe in two launches
// (observe_chunks_kernel + observe_rows_kernel) instead of one workgroup of S / 4 waves per env.
int observe_split_s() {
  static const int v = [] {
    const char* e = std::getenv("LBSIM_OBSERVE_SPLIT_S");
    return e ? std::atoi(e) : 16;
  }();
  return v;
}

template <int MODE, bool FAC>
void launch_observe_split(const LaunchCtx& L, const ObsOutputs& o, const uint8_t* mask,
                          hipStream_t stream) {
  const int nchunks = (L.S + kObsChunk - 1) / kObsChunk;
  LBSIM_LAUNCH(observe_chunks_kernel<MODE>, dim3((unsigned)((int64_t)L.B * nchunks)), dim3(64), 0,
               stream, L.st, L.prm, o, mask, nchunks);
  const dim3 grid((unsigned)L.B), block(64);
  if (L.S <= 8)
    LBSIM_LAUNCH((observe_rows_kernel<8, MODE, FAC>), grid, block, 0, stream, L.st, L.prm, o, mask);
  else if (L.S <= 16)
    LBSIM_LAUNCH((observe_rows_kernel<16, MODE, FAC>), grid, block, 0, stream, L.st, L.prm, o, mask);
  else
    LBSIM_LAUNCH((observe_rows_kernel<64, MODE, FAC>), grid, block, 0, stream, L.st, L.prm, o, mask);
}

// The paired step observe (observe_pair_kernel): no duration plane (duration == fct by
// construction: duration_mode AGE, lost-FIN off) and S <= 8 (8 / S whole envs per wave), or S a
// multiple of 8 (S / 8 waves per env: observe_pair16_kernel, observe_pair_chunks_kernel).  LBSIM_OBSERVE_PAIRED=0
// turns it off (A/B; the same bits either way).
bool observe_paired(const LaunchCtx& L) {
  static const bool on = [] {
    const char* e = std::getenv("LBSIM_OBSERVE_PAIRED");
    return !(e != nullptr && std::strcmp(e, "0") == 0);
  }();
  return on && L.st.res_dur == nullptr && (L.S <= 8 || L.S % 8 == 0);
}

// the problem-05 facade rows (agent_obs / state) come from their own instantiation
template <int MODE>
void launch_observe_m(const LaunchCtx& L, const ObsOutputs& o, const uint8_t* mask,
                      hipStream_t stream) {
  const bool fac = o.agent_obs != nullptr || o.state != nullptr;
  if constexpr (MODE == kModeStep) {
  if (observe_paired(L) && L.S > 8) {  // 8 rows per wave, S / 8 per env
    if (L.S == 16) {
      const dim3 grid((unsigned)L.B), block(128);
      if (fac)
        LBSIM_LAUNCH((observe_pair16_kernel<MODE, true>), grid, block, 0, stream, L.st, L.prm, o);
      else
        LBSIM_LAUNCH((observe_pair16_kernel<MODE, false>), grid, block, 0, stream, L.st, L.prm, o);
      return;
    }
    const int ng = L.S / 8;
    LBSIM_LAUNCH(observe_pair_chunks_kernel<MODE>, dim3((unsigned)((int64_t)L.B * ng)), dim3(64), 0,
                 stream, L.st, L.prm, o, ng);
    const dim3 grid((unsigned)L.B), block(64);
    if (fac)
      LBSIM_LAUNCH((observe_rows_kernel<64, MODE, true>), grid, block, 0, stream, L.st, L.prm, o,
                   nullptr);
    else
      LBSIM_LAUNCH((observe_rows_kernel<64, MODE, false>), grid, block, 0, stream, L.st, L.prm, o,
                   nullptr);
    return;
  }
  }
  if (MODE == kModeStep && observe_paired(L)) {  // 8 rows per wave: 8 / S envs
    const int epw = 8 / L.S;
    const dim3 grid((unsigned)((L.B + epw - 1) / epw)), block(64);
    if (fac)
      LBSIM_LAUNCH((observe_pair_kernel<MODE, true>), grid, block, 0, stream, L.st, L.prm, o);
    else
      LBSIM_LAUNCH((observe_pair_kernel<MODE, false>), grid, block, 0, stream, L.st, L.prm, o);
    return;
  }
  if (L.S > kObsChunk && L.S > observe_split_s()) {
    if (fac) launch_observe_split<MODE, true>(L, o, mask, stream);
    else launch_observe_split<MODE, false>(L, o, mask, stream);
    return;
  }
  if (MODE == kModeReset && L.S <= kObsChunk) {  // kObsResetEnvs single-wave envs per workgroup
    const dim3 grid((unsigned)((L.B + kObsResetEnvs - 1) / kObsResetEnvs)),
        block(64 * kObsResetEnvs);
    const size_t lds = kObsResetEnvs * sizeof(ObsScratch);
    if (fac)
      LBSIM_LAUNCH(observe_reset_kernel<true>, grid, block, lds, stream, L.st, L.prm, o,
                         mask);
    else
      LBSIM_LAUNCH(observe_reset_kernel<false>, grid, block, lds, stream, L.st, L.prm, o,
                         mask);
    return;
  }
  if (fac)
    launch_observe_t<MODE, true>(L, o, mask, stream);
  else
    launch_observe_t<MODE, false>(L, o, mask, stream);
}

}  // namespace

void launch_observe_step(const LaunchCtx& L, const ObsOutputs& o, const uint8_t* mask,
                         hipStream_t s) {
  launch_observe_m<kModeStep>(L, o, mask, s);
}

void launch_observe_reset(const LaunchCtx& L, const ObsOutputs& o, const uint8_t* mask,
                          hipStream_t s) {
  launch_observe_m<kModeReset>(L, o, mask, s);
}

}  // namespace lbk
