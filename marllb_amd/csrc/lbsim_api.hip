// lbsim_api.hip — extern "C" boundary of liblbsim (include/lbsim.h) over the gfx950 kernels.
//
// The handle owns the device state (one hipMalloc per section, SoA); the caller
// owns every I/O buffer.  No allocation, no host synchronisation and no host<->device copy
// happens inside lbsim_reset / lbsim_step, so a caller may capture them into a hipGraph.
#include <hip/hip_runtime.h>

#include <cxxabi.h>

#include <algorithm>
#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/lbsim.h"
#include "lbsim_internal.h"
#include "lbsim_fused.h"
#include "lbsim_nets.h"
#include "lbsim_stateless.h"
#include "lbsim_vpp.h"

using namespace lbk;

// The launch log of LBSIM_LAUNCH (lbsim_internal.h): (profile class, host stub) of each kernel
// the API call in progress launched.  The calls that launch simulator kernels set the class
// before each launch; a scoped LaunchLog copies the log into the handle when the call returns.
namespace {
constexpr int kLogMax = 8;
thread_local const void* g_log_fn[kLogMax];
thread_local int g_log_cls[kLogMax];
thread_local int g_log_n = 0;
thread_local int g_log_lost = 0;  // launches past kLogMax (reported, not dropped silently)
thread_local int g_log_class = -1;
}  // namespace

void lbk::note_launch(const void* host_fn) {
  if (g_log_n < kLogMax) {
    g_log_fn[g_log_n] = host_fn;
    g_log_cls[g_log_n] = g_log_class;
    ++g_log_n;
  } else {
    ++g_log_lost;
  }
}

struct Profiler {
  bool on = false;
  std::vector<hipEvent_t> ev;  // at most 2 per timed launch
  std::vector<int> cls;        // kernel class per timed launch
  std::vector<int> beg, end;   // event indices bracketing each timed launch
  size_t used = 0;             // events recorded
  size_t cap = 0;              // events this profile may record (2 per requested launch)
  // lbsim_step: the event that ends the dynamics launch also starts the observe launch (one
  // event between the two kernels instead of two)
  bool chain = false;
  int chain_ev = -1;
};

struct lbsim {
  lbsim_config_t cfg;
  Profiler prof;
  int device;
  int simds;  // SIMDs of the device (CUs x 4): the env-per-lane mapping fills them at B >= 64·simds
  int B, S, Q;
  DevState st;
  SimParams prm;
  std::vector<void*> allocs;
  void* trace_buf = nullptr;  // gap_us[rows] then work[rows]
  unsigned long long* stats_buf = nullptr;  // lbsim_step_stats sums (2 x u64)
  bool initialised;  // a full reset has been issued
  std::string err;
  // (class, host stub) of the kernels the last lbsim_step_ex / lbsim_reset_ex launched
  std::vector<std::pair<int, const void*>> launched[2];
  int launched_lost[2] = {0, 0};  // launches of that call past the log's capacity
};

namespace {

thread_local std::string g_create_err;

int fail(lbsim_t* h, int code, const char* fmt, ...) {
  char buf[512];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof(buf), fmt, ap);
  va_end(ap);
  if (h) h->err = buf;
  else g_create_err = buf;
  return code;
}

// Scoped hipSetDevice that restores the caller's current device (torch keeps its own).
struct DeviceGuard {
  int prev = -1;
  bool ok = false;
  explicit DeviceGuard(int dev) {
    if (hipGetDevice(&prev) != hipSuccess) prev = -1;
    ok = hipSetDevice(dev) == hipSuccess;
  }
  ~DeviceGuard() {
    if (prev >= 0) (void)hipSetDevice(prev);
  }
};

int bad_msg(char* msg, size_t n, const char* fmt, ...) __attribute__((format(printf, 3, 4)));
int bad_msg(char* msg, size_t n, const char* fmt, ...) {
  if (msg && n) {
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(msg, n, fmt, ap);
    va_end(ap);
  }
  return LBSIM_EINVAL;
}

int validate(const lbsim_config_t* c, char* msg, size_t n) {
#define bad(...) bad_msg(msg, n, __VA_ARGS__)
  if (c == nullptr) return bad("config is NULL");
  if (c->num_envs < 1) return bad("num_envs must be >= 1 (got %d)", c->num_envs);
  if (c->num_servers < 1 || c->num_servers > LBSIM_MAX_SERVERS)
    return bad("num_servers must be in [1, %d] (got %d)", LBSIM_MAX_SERVERS, c->num_servers);
  if ((int64_t)c->env_id_offset < 0 ||
      (uint64_t)c->env_id_offset + (uint64_t)c->num_envs > 0xFFFFFFFFull)
    return bad("global env ids must fit in 32 bits");
  if (c->action_type != LBSIM_ACTION_DISCRETE && c->action_type != LBSIM_ACTION_CONTINUOUS)
    return bad("Unknown action_type: %d", c->action_type);
  if (c->action_type == LBSIM_ACTION_DISCRETE &&
      (c->num_discrete < 1 || c->num_discrete > LBSIM_MAX_DISCRETE))
    return bad("num_discrete must be in [1, %d]", LBSIM_MAX_DISCRETE);
  if (c->reward_metric < LBSIM_METRIC_JAIN || c->reward_metric > LBSIM_METRIC_GINI)
    return bad("Unsupported metric: %d", c->reward_metric);
  if (c->reward_field < -1 || c->reward_field >= LBSIM_NUM_FEATURES)
    return bad("reward_field must be -1 or a column in [0, 10]");
  if (!(c->step_interval > 0.0f) || c->step_interval > 100.0f)
    return bad("step_interval must be in (0, 100] seconds");
  if ((int64_t)std::llround((double)c->step_interval * 1e6) < 1)
    return bad("step_interval must be >= 1 us");
  if (c->max_steps < 1) return bad("max_steps must be >= 1");
  if (c->assign_policy < LBSIM_POLICY_SED || c->assign_policy > LBSIM_POLICY_ALIAS)
    return bad("unknown assign_policy %d", c->assign_policy);
  if (c->arrival_source != LBSIM_ARRIVAL_POISSON && c->arrival_source != LBSIM_ARRIVAL_TRACE)
    return bad("unknown arrival_source");
  if (!(c->arrival_rate >= 0.1f) || !(c->arrival_rate <= 1.0e6f))
    return bad("arrival_rate must be in [0.1, 1e6] flows/s");
  for (int s = 0; s < c->num_servers; ++s)
    if (!(c->server_rate[s] >= 1.0f) || !(c->server_rate[s] <= 1.0e7f))
      return bad("server_rate[%d] must be in [1, 1e7] flows/s", s);
  if (!(c->decay_factor > 0.0f) || !(c->decay_factor < 1.0f))
    return bad("decay_factor must be in (0, 1)");
  if (c->queue_capacity < 1 || c->queue_capacity > 64)
    return bad("queue_capacity must be in [1, 64]");
  if (c->warmup_steps < 0 || c->warmup_steps > 100000) return bad("warmup_steps out of range");
  if (c->dyn_mapping < LBSIM_DYN_AUTO || c->dyn_mapping > LBSIM_DYN_SERVER_PER_LANE)
    return bad("unknown dyn_mapping %d", c->dyn_mapping);
  if (c->step_kernel < LBSIM_STEP_AUTO || c->step_kernel > LBSIM_STEP_FUSED)
    return bad("unknown step_kernel %d", c->step_kernel);
  if (!(c->lost_fin_prob >= 0.0f) || !(c->lost_fin_prob <= 1.0f))
    return bad("lost_fin_prob must be in [0, 1]");
  if (c->lost_fin_prob > 0.0f) {
    if (!(c->flow_timeout_s >= 0.0f)) return bad("flow_timeout_s must be >= 0");
    if (c->flow_buckets < 1) return bad("flow_buckets must be >= 1");
    // the guess fct + (flow_timeout - 40 s) + wait and its wrap-up delay flow_timeout + wait are
    // signed int32 us: with the wait <= 16.7 x its mean flow_buckets / arrival_rate (24-bit
    // uniforms) and an fct of at most ~1,070 s (64 queued flows of <= 16.7 s service each at
    // >= 1 flow/s), flow_timeout + 16.7 x the mean wait <= 1040 s keeps both below 2^31 us
    // (lost_fct also saturates, for trace work beyond that bound)
    const double wmean = (double)c->flow_buckets / (double)c->arrival_rate;
    if ((double)c->flow_timeout_s + 16.7 * wmean > 1040.0) {
      if ((double)c->flow_timeout_s >= 1040.0)
        return bad("lost-FIN: flow_timeout_s must be < 1040 s (got %.1f)", c->flow_timeout_s);
      return bad("lost-FIN: flow_timeout_s + 16.7 * flow_buckets / arrival_rate must be <= 1040 s "
                 "(signed 32-bit us guesses): with flow_timeout_s = %.1f, flow_buckets / "
                 "arrival_rate must be <= %.3f s (got %.3f)",
                 c->flow_timeout_s, (1040.0 - (double)c->flow_timeout_s) / 16.7, wmean);
    }
    if (c->lost_fin_pending < 1 || c->lost_fin_pending > 4096)
      return bad("lost_fin_pending must be in [1, 4096]");
  }
  if (c->lost_fin_prob > 0.0f && std::llround((double)c->lost_fin_prob * 16777216.0) == 0)
    return bad("lost_fin_prob must be 0 or >= 2^-25 (a 24-bit threshold)");
  if (!(c->fail_prob >= 0.0f) || !(c->fail_prob <= 1.0f)) return bad("fail_prob must be in [0, 1]");
  if (c->fail_prob > 0.0f && std::llround((double)c->fail_prob * 16777216.0) == 0)
    return bad("fail_prob must be 0 or >= 2^-25 (a 24-bit threshold)");
  if (c->next_step_reset != 0 && c->next_step_reset != 1) return bad("next_step_reset must be 0 or 1");
  if (c->duration_mode != LBSIM_DURATION_AGE && c->duration_mode != LBSIM_DURATION_SERVICE)
    return bad("unknown duration_mode %d", c->duration_mode);
  if (c->n_flow_on_mode != LBSIM_NFLOW_QUEUE && c->n_flow_on_mode != LBSIM_NFLOW_VPP)
    return bad("unknown n_flow_on_mode %d", c->n_flow_on_mode);
  if (c->reservoir_mode != LBSIM_RESERVOIR_ALGR && c->reservoir_mode != LBSIM_RESERVOIR_VPP)
    return bad("unknown reservoir_mode %d", c->reservoir_mode);
  if (!(c->recover_prob >= 0.0f) || !(c->recover_prob <= 1.0f))
    return bad("recover_prob must be in [0, 1]");
  if (c->dyn_mapping == LBSIM_DYN_ENV_PER_LANE && c->num_servers > 16)
    return bad("the env-per-lane dynamics mapping takes at most 16 servers (got %d)",
               c->num_servers);
  return LBSIM_OK;
#undef bad
}

void derive_params(const lbsim_config_t& c, SimParams& p) {
  memset(&p, 0, sizeof(p));
  p.B = c.num_envs;
  p.S = c.num_servers;
  p.Q = c.queue_capacity;
  p.dt_us = (int32_t)std::llround((double)c.step_interval * 1e6);
  p.mean_gap_us = (float)(1e6 / (double)c.arrival_rate);
  for (int s = 0; s < MAX_S; ++s)
    p.svc_scale[s] = s < c.num_servers ? (float)(1e6 / (double)c.server_rate[s]) : 0.0f;
  p.key0 = (uint32_t)(c.seed & 0xFFFFFFFFull);
  p.key1 = (uint32_t)(c.seed >> 32);
  p.env_id_offset = (uint32_t)c.env_id_offset;
  p.policy = c.assign_policy;
  p.action_type = c.action_type;
  p.num_discrete = c.num_discrete;
  for (int i = 0; i < 8; ++i) p.dw[i] = c.discrete_weights[i];
  p.min_w = c.min_weight;
  p.max_w = c.max_weight;
  p.warmup_steps = c.warmup_steps;
  p.max_steps = c.max_steps;
  p.reward_metric = c.reward_metric;
  p.reward_field = c.reward_field;
  p.decay_c = (float)(std::log2((double)c.decay_factor) / 1000.0);
  p.normalize = c.normalize_obs ? 1 : 0;
  p.trace = c.arrival_source == LBSIM_ARRIVAL_TRACE ? 1 : 0;
  p.trace_rows = 0;
  p.lf_thr = (uint32_t)std::llround((double)c.lost_fin_prob * 16777216.0);
  p.lf_off_us = (int32_t)(std::llround((double)c.flow_timeout_s * 1e6) - 40000000LL);
  p.lf_wait_us = c.lost_fin_prob > 0.0f
                     ? (float)((double)c.flow_buckets * 1e6 / (double)c.arrival_rate) : 0.0f;
  p.fail_thr = (uint32_t)std::llround((double)c.fail_prob * 16777216.0);
  p.rec_thr = (uint32_t)std::llround((double)c.recover_prob * 16777216.0);
  p.big_in_step = (p.dt_us >= (int32_t)kPackLimit || p.lf_thr != 0u) ? 1 : 0;
  p.next_reset = c.next_step_reset ? 1 : 0;
  p.dur_service = c.duration_mode == LBSIM_DURATION_SERVICE ? 1 : 0;
  p.leak = (c.n_flow_on_mode == LBSIM_NFLOW_VPP && p.lf_thr != 0u) ? 1 : 0;
  p.split = p.lf_thr != 0u ? 1 : 0;
  p.pend_P = p.split ? c.lost_fin_pending : 0;
  p.res_vpp = c.reservoir_mode == LBSIM_RESERVOIR_VPP ? 1 : 0;
}

// Whether a handle keeps a duration plane (DevState::res_dur): duration_mode SERVICE (the service
// time differs from the age) or lost-FIN guesses (their fct differs from the duration).  Otherwise
// every duration sample equals its fct sample, and the duration reservoir is the fct reservoir.
bool dur_plane(const SimParams& p) { return p.dur_service != 0 || p.lf_thr != 0u; }

// State sections in snapshot order.
struct Section {
  void** ptr;
  size_t bytes;
};

std::vector<Section> sections(lbsim_t* h) {
  const size_t B = h->B, BS = (size_t)h->B * h->S, BSQ = BS * h->Q, BSK = BS * K;
  DevState& s = h->st;
  std::vector<Section> v = {
      {(void**)&s.next_arr, B * 4},   {(void**)&s.next_work, B * 4}, {(void**)&s.next_u2, B * 4},
      {(void**)&s.next_u3, B * 4},    {(void**)&s.arr_idx, B * 4},   {(void**)&s.episode, B * 4},
      {(void**)&s.clock, B * 4},      {(void**)&s.ep_step, B * 4},   {(void**)&s.dropped, B * 4},
      {(void**)&s.norm_count, B * 4}, {(void**)&s.ep_return, B * 8}, {(void**)&s.hc, BS * 4},
      {(void**)&s.last_tc, BS * 4},   {(void**)&s.res_count, BS * 4}, {(void**)&s.ring, BSQ * 8},
      {(void**)&s.res, BSK * 8},      {(void**)&s.chg, BS * 16},      {(void**)&s.fcache, BS * 40},
  };
  if (h->cfg.normalize_obs) {
    v.push_back({(void**)&s.norm_mean, BS * NF * 8});
    v.push_back({(void**)&s.norm_std, BS * NF * 8});
  }
  if (h->cfg.fail_prob > 0.0f) v.push_back({(void**)&s.down, BS * 4});
  if (h->prm.leak) v.push_back({(void**)&s.lost_on, BS * 4});
  // the duration plane: only when a flow's duration sample can differ from its fct; split
  // handles (lost-FIN): {us, ts} records, the duration count, the pending guesses, lf_over
  if (dur_plane(h->prm)) v.push_back({(void**)&s.res_dur, BSK * (h->prm.split ? 8 : 4)});
  if (h->prm.split) {
    v.push_back({(void**)&s.res_count_dur, BS * 4});
    v.push_back({(void**)&s.pend_hc, BS * 4});
    v.push_back({(void**)&s.pend, BS * (size_t)h->prm.pend_P * 8});
    v.push_back({(void**)&s.lf_over, B * 4});
  }
  return v;
}

__global__ void init_norm_std(double* p, size_t n) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) p[i] = 1.0;  // env.py:153 obs_std = ones
}

// lbsim_step_stats: popcount of the written-slot masks and the sum of the queue counts, one
// device-wide sum each (wave shuffles, then one vector atomic per wave).
__global__ void __launch_bounds__(256)
    step_stats_kernel(const uint32_t* chg, const uint32_t* hc, int64_t n_srv,
                      unsigned long long* out) {
  unsigned long long slots = 0, flows = 0;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n_srv;
       i += (int64_t)gridDim.x * 256) {
    const uint4 m = reinterpret_cast<const uint4*>(chg)[i];
    slots += __popc(m.x) + __popc(m.y) + __popc(m.z) + __popc(m.w);
    flows += hc[i] >> 16;
  }
  for (int d = 32; d > 0; d >>= 1) {
    slots += __shfl_xor(slots, d, 64);
    flows += __shfl_xor(flows, d, 64);
  }
  if ((threadIdx.x & 63) == 0) {
    atomicAdd(out, slots);
    atomicAdd(out + 1, flows);
  }
}

__global__ void copy_episode_stats(const int32_t* steps, const double* ret, int32_t* lo,
                                   double* ro, int B) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= B) return;
  if (lo) lo[i] = steps[i];
  if (ro) ro[i] = ret[i];
}

int launch_check(lbsim_t* h, const char* what) {
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess) return fail(h, LBSIM_EDEVICE, "%s: %s", what, hipGetErrorString(e));
  return LBSIM_OK;
}

// Brackets one launch with profiler events when profiling is on (class: see lbsim.h).
struct ProfScope {
  lbsim_t* h;
  hipStream_t s;
  bool rec = false;
  ProfScope(lbsim_t* h_, hipStream_t s_, int cls) : h(h_), s(s_) {
    g_log_class = cls;  // the launch log's class of the kernel launched in this scope
    Profiler& p = h->prof;
    if (!p.on) return;
    if (p.chain_ev >= 0 && p.used + 1 <= p.cap) {
      p.beg.push_back(p.chain_ev);  // the previous launch's end event, on the same stream
      rec = true;
    } else if (p.used + 2 <= p.cap && hipEventRecord(p.ev[p.used], s) == hipSuccess) {
      p.beg.push_back((int)p.used++);
      rec = true;
    }
    p.chain_ev = -1;
    if (rec) p.cls.push_back(cls);
  }
  ~ProfScope() {
    g_log_class = -1;  // a launch outside any scope is logged with class -1, not a stale one
    if (!rec) return;
    Profiler& p = h->prof;
    (void)hipEventRecord(p.ev[p.used], s);
    p.end.push_back((int)p.used);
    p.chain_ev = p.chain ? (int)p.used : -1;
    ++p.used;
  }
};

// Scope of one lbsim_step_ex (which = 0) / lbsim_reset_ex (1): the launch log starts empty and
// is kept in the handle when the call returns (lbsim_launch_names).
struct LaunchLog {
  lbsim_t* h;
  int which;
  LaunchLog(lbsim_t* h_, int w) : h(h_), which(w) {
    g_log_n = 0;
    g_log_lost = 0;
  }
  ~LaunchLog() {
    auto& v = h->launched[which];
    v.clear();
    for (int i = 0; i < g_log_n; ++i) v.emplace_back(g_log_cls[i], g_log_fn[i]);
    h->launched_lost[which] = g_log_lost;
    g_log_n = 0;
    g_log_lost = 0;
    g_log_class = -1;
  }
};

// "void lbk::observe_kernel<4, 0, false>(lbk::DevState, ...)" -> "observe_kernel<4, 0, false>":
// the form tools/pmc_traffic.py and tools/pmc_valu.py key their counter files by.
std::string short_kernel_name(const char* raw) {
  std::string s = raw ? raw : "?";
  int st = 0;
  if (char* d = abi::__cxa_demangle(s.c_str(), nullptr, nullptr, &st)) {
    if (st == 0) s = d;
    free(d);
  }
  int depth = 0;  // cut the parameter list: the first '(' outside template brackets
  for (size_t i = 0; i < s.size(); ++i) {
    if (s[i] == '<') ++depth;
    else if (s[i] == '>') --depth;
    else if (s[i] == '(' && depth == 0 && s.compare(i, 21, "(anonymous namespace)") != 0) {
      s.resize(i);
      break;
    }
  }
  for (const char* pre : {"void ", "lbk::", "(anonymous namespace)::"}) {
    for (size_t at; (at = s.find(pre)) != std::string::npos;) s.erase(at, strlen(pre));
  }
  return s;
}

LaunchCtx ctx(const lbsim_t* h) {
  return LaunchCtx{h->st, h->prm, h->B, h->S, h->simds, h->cfg.dyn_mapping};
}

int launch_dynamics(lbsim_t* h, const void* action, int dtype, int32_t* assign,
                    const uint8_t* mask, int mode, hipStream_t stream) {
  ProfScope ps(h, stream, mode == kModeStep ? 0 : 2);
  if (mode == kModeStep && h->prm.next_reset)  // next-step auto-reset: done envs reset instead
    launch_dynamics_step_nr(ctx(h), action, dtype, assign, mask, stream);
  else if (mode == kModeStep)
    launch_dynamics_step(ctx(h), action, dtype, assign, mask, stream);
  else
    launch_dynamics_reset(ctx(h), action, dtype, assign, mask, stream);
  return launch_check(h, "dynamics_kernel");
}

bool facade_bad(const lbsim_t* h, const lbsim_step_outputs_t* out) {
  if (out->agent_obs == nullptr && out->state == nullptr) return false;
  return out->num_agents < 1 || out->servers_per_agent < 1 ||
         (int64_t)out->num_agents * out->servers_per_agent != h->S;
}

ObsOutputs obs_outputs(const lbsim_step_outputs_t* out, bool reset) {
  ObsOutputs o{};
  o.obs = out->obs;
  o.raw_obs = out->raw_obs;
  if (!reset) {
    o.reward = out->reward;
    o.done = out->done;
    o.ep_len = out->episode_length;
    o.ep_ret = out->episode_return;
    o.done_word = out->done_word;
    o.done_value = out->done_value;
  }
  o.agent_obs = out->agent_obs;
  o.state = out->state;
  o.num_agents = out->num_agents;
  o.servers_per_agent = out->servers_per_agent;
  return o;
}

// The step kernel a handle asks for: its config, else LBSIM_STEP_KERNEL=split|fused, else AUTO.
int step_kernel_of(const lbsim_t* h) {
  static const int env = [] {
    const char* e = std::getenv("LBSIM_STEP_KERNEL");
    if (e != nullptr && std::strcmp(e, "split") == 0) return LBSIM_STEP_SPLIT;
    if (e != nullptr && std::strcmp(e, "fused") == 0) return LBSIM_STEP_FUSED;
    return LBSIM_STEP_AUTO;
  }();
  return h->cfg.step_kernel != LBSIM_STEP_AUTO ? h->cfg.step_kernel : env;
}

// The one-launch wave step (step_wave_kernel): one wave per env and S <= 8, FUSED asked for, or
// AUTO on batches of at most 4 envs per SIMD (LBSIM_STEP_WAVE_MAX_B overrides), where one launch
// instead of two pays: 2048 x 4 0.0711 -> 0.0620 ms per step, 4096 x 4 +2.5 %
// (profiles/r03w/ab_step_wave_fused.txt).  S = 5-8 between 2 and 4 envs per SIMD: the wave
// dynamics alone lose to the server-per-lane groups there (dyn_wave_ok), the one launch with both
// chunks observed in it wins (profiles/r04s/).
bool use_step_wave(const lbsim_t* h) {
  static const int64_t max_b = [] {
    const char* e = std::getenv("LBSIM_STEP_WAVE_MAX_B");
    return e ? (int64_t)std::atoll(e) : (int64_t)-1;
  }();
  const LaunchCtx L = ctx(h);
  // next-step auto-reset handles step in two launches (the dynamics' kModeStepNR instantiation)
  if (!dyn_wave_fits(L) || h->prm.next_reset) return false;
  const int k = step_kernel_of(h);
  if (k == LBSIM_STEP_FUSED) return dyn_wave_ok(L);
  return k == LBSIM_STEP_AUTO && (int64_t)L.B <= (max_b >= 0 ? max_b : 4 * (int64_t)L.simds);
}

// The fused step for this handle: its config (LBSIM_STEP_KERNEL=split|fused overrides AUTO) and
// a group width that has a fused form.
bool use_fused_step(const lbsim_t* h) {
  // AUTO = SPLIT: the fused kernel measured slower at every shape tried
  if (step_kernel_of(h) != LBSIM_STEP_FUSED || h->prm.next_reset) return false;
  // full handles (dynamics_group_full_kernel: leak, a duration plane, lost-FIN deferral,
  // reservoir_mode VPP) step in the two launches
  if (h->prm.leak || dur_plane(h->prm) || h->prm.res_vpp) return false;
  const int g = dyn_group_lanes(ctx(h));
  return g >= 2 && g <= 16;
}

int launch_observe(lbsim_t* h, const ObsOutputs& o, const uint8_t* mask, int mode,
                   hipStream_t stream) {
  ProfScope ps(h, stream, mode == kModeStep ? 1 : 3);
  if (mode == kModeStep) launch_observe_step(ctx(h), o, mask, stream);
  else launch_observe_reset(ctx(h), o, mask, stream);
  return launch_check(h, "observe_kernel");
}

// ---- one-kernel policy inference (lbsim_fused.h)

// LDS row stride of the fused kernels: >= need floats and = 4 (mod 64), so the 16 rows one
// ds_read_b128 touches fall in distinct banks.
int fused_ld(int need) { return ((need - 4 + 63) / 64) * 64 + 4; }
int round16(int x) { return (x + 15) / 16 * 16; }
constexpr size_t kFusedLdsMax = 160 * 1024;

// Envs per workgroup = 16 MT.  QMIX's tile kernel: MT = 1 (8192 x 16 0.121 / 0.157 / 0.251 ms at
// MT = 1 / 2 / 4, profiles/r01s3a).  The SAC actor: MT = 2 since round 6 -- with its staging one
// HBM round trip (r06n), a 32-env tile halves the weight stream per env, and the weight stream is
// what the staging waited behind: 187-188 -> 179.3-179.7 us at 65536 x 8, 0.53 -> 0.556 of the
// f32 MFMA peak (profiles/r06q/; round 1, with the staging serialised, MT = 2 was the slower:
// 0.231 vs 0.267 ms).  LBSIM_FUSED_MT = 1 | 2 | 4 forces it for both.
int fused_mt(int64_t, int dflt = 1) {
  static const int forced = [] {
    const char* s = std::getenv("LBSIM_FUSED_MT");
    return s ? std::atoi(s) : 0;
  }();
  return (forced == 1 || forced == 2 || forced == 4) ? forced : dflt;
}

}  // namespace

extern "C" {

const char* lbsim_version(void) { return "lbsim 0.1.0 (gfx950, HIP)"; }
int lbsim_abi_version(void) { return LBSIM_ABI_VERSION; }

int lbsim_config_default(lbsim_config_t* c) {
  if (c == nullptr) return LBSIM_EINVAL;
  memset(c, 0, sizeof(*c));
  c->num_envs = 1;
  c->num_servers = 4;
  c->env_id_offset = 0;
  c->seed = 0;
  c->action_type = LBSIM_ACTION_DISCRETE;
  c->num_discrete = 3;
  c->discrete_weights[0] = 1.0f;
  c->discrete_weights[1] = 1.5f;
  c->discrete_weights[2] = 2.0f;
  c->min_weight = 0.1f;
  c->max_weight = 10.0f;
  c->reward_metric = LBSIM_METRIC_JAIN;
  c->reward_field = 10;
  c->step_interval = 0.25f;
  c->max_steps = 10000;
  c->normalize_obs = 0;
  c->assign_policy = LBSIM_POLICY_SED;
  c->arrival_source = LBSIM_ARRIVAL_POISSON;
  c->arrival_rate = 400.0f;
  for (int s = 0; s < LBSIM_MAX_SERVERS; ++s) c->server_rate[s] = 125.0f;
  c->decay_factor = 0.9f;
  c->queue_capacity = 32;
  c->warmup_steps = 8;
  c->lost_fin_prob = 0.0f;
  c->flow_timeout_s = 40.0f;  // LB_DEFAULT_FLOW_TIMEOUT (lb.c:1437)
  c->flow_buckets = 1024;     // LB_DEFAULT_PER_CPU_STICKY_BUCKETS (lb.h:46)
  c->fail_prob = 0.0f;
  c->recover_prob = 0.1f;
  c->duration_mode = LBSIM_DURATION_AGE;  // lbhash.h:129-136: the flow's age
  c->lost_fin_pending = 256;
  c->reservoir_mode = LBSIM_RESERVOIR_ALGR;
  return LBSIM_OK;
}

int lbsim_config_validate(const lbsim_config_t* cfg, char* msg, size_t msg_len) {
  return validate(cfg, msg, msg_len);
}

int lbsim_create(const lbsim_config_t* cfg, int device, lbsim_t** out) {
  if (out == nullptr) return fail(nullptr, LBSIM_EINVAL, "out is NULL");
  *out = nullptr;
  char msg[256] = {0};
  if (validate(cfg, msg, sizeof(msg)) != LBSIM_OK) return fail(nullptr, LBSIM_EINVAL, "%s", msg);
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0)
    return fail(nullptr, LBSIM_EDEVICE, "no HIP device available");
  if (device < 0 || device >= ndev)
    return fail(nullptr, LBSIM_EINVAL, "device %d out of range [0, %d)", device, ndev);
  DeviceGuard g(device);
  if (!g.ok) return fail(nullptr, LBSIM_EDEVICE, "hipSetDevice(%d) failed", device);

  lbsim_t* h = new lbsim_t();
  h->cfg = *cfg;
  h->device = device;
  int cus = 0;
  if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device) != hipSuccess ||
      cus < 1)
    cus = 256;
  h->simds = 4 * cus;
  h->B = cfg->num_envs;
  h->S = cfg->num_servers;
  h->Q = cfg->queue_capacity;
  h->initialised = false;
  memset(&h->st, 0, sizeof(h->st));
  derive_params(*cfg, h->prm);
  for (Section& sec : sections(h)) {
    void* p = nullptr;
    if (hipMalloc(&p, sec.bytes) != hipSuccess) {
      lbsim_destroy(h);
      return fail(nullptr, LBSIM_ENOMEM, "hipMalloc(%zu) failed", sec.bytes);
    }
    h->allocs.push_back(p);
    *sec.ptr = p;
    if (hipMemset(p, 0, sec.bytes) != hipSuccess) {
      lbsim_destroy(h);
      return fail(nullptr, LBSIM_EDEVICE, "hipMemset failed");
    }
  }
  if (cfg->normalize_obs) {
    const size_t n = (size_t)h->B * h->S * NF;
    hipLaunchKernelGGL(init_norm_std, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, nullptr,
                       h->st.norm_std, n);
  }
  if (hipDeviceSynchronize() != hipSuccess) {
    lbsim_destroy(h);
    return fail(nullptr, LBSIM_EDEVICE, "device init failed");
  }
  *out = h;
  return LBSIM_OK;
}

int lbsim_destroy(lbsim_t* h) {
  if (h == nullptr) return LBSIM_OK;
  {
    DeviceGuard g(h->device);
    for (void* p : h->allocs) (void)hipFree(p);
    if (h->trace_buf) (void)hipFree(h->trace_buf);
    if (h->stats_buf) (void)hipFree(h->stats_buf);
    for (hipEvent_t e : h->prof.ev) (void)hipEventDestroy(e);
  }
  delete h;
  return LBSIM_OK;
}

const char* lbsim_last_error(const lbsim_t* h) {
  return h ? h->err.c_str() : g_create_err.c_str();
}

int lbsim_dynamics_kernel(const lbsim_t* h) {
  if (h == nullptr) return -1;
  const LaunchCtx L = ctx(h);
  if (dyn_wave_ok(L)) return LBSIM_DYN_KERNEL_WAVE;
  return dyn_group_lanes(L) == 0 ? LBSIM_DYN_KERNEL_ENV_LANE : LBSIM_DYN_KERNEL_GROUP;
}

int lbsim_seed(lbsim_t* h, uint64_t seed) {
  if (h == nullptr) return LBSIM_EINVAL;
  DeviceGuard g(h->device);
  h->cfg.seed = seed;
  h->prm.key0 = (uint32_t)(seed & 0xFFFFFFFFull);
  h->prm.key1 = (uint32_t)(seed >> 32);
  if (hipMemset(h->st.episode, 0, (size_t)h->B * 4) != hipSuccess)
    return fail(h, LBSIM_EDEVICE, "hipMemset failed");
  return LBSIM_OK;
}

int lbsim_reset(lbsim_t* h, const uint8_t* env_mask, float* obs_out, void* stream) {
  lbsim_step_outputs_t o;
  memset(&o, 0, sizeof(o));
  o.obs = obs_out;
  return lbsim_reset_ex(h, env_mask, &o, stream);
}

int lbsim_reset_ex(lbsim_t* h, const uint8_t* env_mask, const lbsim_step_outputs_t* out,
                   void* stream) {
  if (h == nullptr) return LBSIM_EINVAL;
  if (out == nullptr || out->obs == nullptr) return fail(h, LBSIM_EINVAL, "obs_out is NULL");
  if (facade_bad(h, out)) return fail(h, LBSIM_EINVAL, "agent_obs / state need num_agents * "
                                                       "servers_per_agent == num_servers");
  if (h->prm.trace && h->prm.trace_rows == 0)
    return fail(h, LBSIM_EINVAL, "arrival_source TRACE: call lbsim_set_trace before lbsim_reset");
  DeviceGuard g(h->device);
  LaunchLog log(h, 1);
  const hipStream_t s = (hipStream_t)stream;
  int rc = launch_dynamics(h, nullptr, 0, nullptr, env_mask, kModeReset, s);
  if (rc != LBSIM_OK) return rc;
  const ObsOutputs o = obs_outputs(out, true);
  rc = launch_observe(h, o, env_mask, kModeReset, s);
  if (rc != LBSIM_OK) return rc;
  if (env_mask == nullptr) h->initialised = true;
  return LBSIM_OK;
}

int lbsim_step(lbsim_t* h, const void* action, int action_dtype, float* obs_out,
               float* reward_out, uint8_t* done_out, int32_t* assign_count_out, void* stream) {
  lbsim_step_outputs_t o;
  memset(&o, 0, sizeof(o));
  o.obs = obs_out;
  o.reward = reward_out;
  o.done = done_out;
  o.assign_count = assign_count_out;
  return lbsim_step_ex(h, action, action_dtype, &o, stream);
}

size_t lbsim_config_size(void) { return sizeof(lbsim_config_t); }
size_t lbsim_step_outputs_size(void) { return sizeof(lbsim_step_outputs_t); }

int lbsim_step_ex(lbsim_t* h, const void* action, int action_dtype,
                  const lbsim_step_outputs_t* out, void* stream) {
  if (h == nullptr) return LBSIM_EINVAL;
  if (!h->initialised) return fail(h, LBSIM_EINVAL, "call lbsim_reset before lbsim_step");
  if (out == nullptr || action == nullptr || out->obs == nullptr || out->reward == nullptr ||
      out->done == nullptr)
    return fail(h, LBSIM_EINVAL, "action/obs/reward/done buffers must be non-NULL");
  if (h->cfg.action_type == LBSIM_ACTION_DISCRETE) {
    if (action_dtype != LBSIM_DTYPE_I32 && action_dtype != LBSIM_DTYPE_I64)
      return fail(h, LBSIM_EINVAL, "discrete actions must be int32 or int64");
  } else if (action_dtype != LBSIM_DTYPE_F32) {
    return fail(h, LBSIM_EINVAL, "continuous actions must be float32");
  }
  if (facade_bad(h, out)) return fail(h, LBSIM_EINVAL, "agent_obs / state need num_agents * "
                                                       "servers_per_agent == num_servers");
  if (out->done_word != nullptr && h->B != 1)
    return fail(h, LBSIM_EINVAL, "done_word needs a one-env handle (num_envs = 1)");
  DeviceGuard g(h->device);
  LaunchLog log(h, 0);
  const hipStream_t s = (hipStream_t)stream;
  const ObsOutputs o = obs_outputs(out, false);
  if (use_step_wave(h)) {
    ProfScope ps(h, s, 4);
    launch_step_wave(ctx(h), action, action_dtype, out->assign_count, o, s);
    return launch_check(h, "step_wave_kernel");
  }
  if (use_fused_step(h)) {
    ProfScope ps(h, s, 4);
    const LaunchCtx L = ctx(h);
    if (!launch_fused_step(L, dyn_group_lanes(L), action, action_dtype, out->assign_count, o, s))
      return fail(h, LBSIM_EINVAL, "no fused step for this group width");
    return launch_check(h, "fused_step_kernel");
  }
  h->prof.chain = true;  // dynamics then observe back to back on s: one event between them
  int rc = launch_dynamics(h, action, action_dtype, out->assign_count, nullptr, kModeStep, s);
  h->prof.chain = false;
  if (rc != LBSIM_OK) {
    h->prof.chain_ev = -1;
    return rc;
  }
  return launch_observe(h, o, nullptr, kModeStep, s);
}

int lbsim_step_stats(lbsim_t* h, int64_t* stats_out) {
  if (h == nullptr || stats_out == nullptr) return LBSIM_EINVAL;
  DeviceGuard g(h->device);
  if (h->stats_buf == nullptr && hipMalloc(&h->stats_buf, 16) != hipSuccess) {
    h->stats_buf = nullptr;
    return fail(h, LBSIM_ENOMEM, "hipMalloc(16) failed");
  }
  const int64_t n = (int64_t)h->B * h->S;
  unsigned long long host[2] = {0, 0};
  if (hipDeviceSynchronize() != hipSuccess || hipMemset(h->stats_buf, 0, 16) != hipSuccess)
    return fail(h, LBSIM_EDEVICE, "sync / memset failed");
  const int64_t blocks = std::min<int64_t>((n + 255) / 256, 4096);
  hipLaunchKernelGGL(step_stats_kernel, dim3((unsigned)blocks), dim3(256), 0, nullptr, h->st.chg,
                     h->st.hc, n, h->stats_buf);
  if (hipMemcpy(host, h->stats_buf, 16, hipMemcpyDeviceToHost) != hipSuccess)
    return fail(h, LBSIM_EDEVICE, "step_stats_kernel failed");
  stats_out[0] = (int64_t)host[0];
  stats_out[1] = (int64_t)host[1];
  return LBSIM_OK;
}

int lbsim_episode_stats(lbsim_t* h, int32_t* length_out, double* return_out, void* stream) {
  if (h == nullptr) return LBSIM_EINVAL;
  DeviceGuard g(h->device);
  hipLaunchKernelGGL(copy_episode_stats, dim3((unsigned)((h->B + 255) / 256)), dim3(256), 0,
                     (hipStream_t)stream, h->st.ep_step, h->st.ep_return, length_out, return_out,
                     h->B);
  return launch_check(h, "copy_episode_stats");
}

int lbsim_reward(const lbsim_config_t* cfg, const float* obs, int64_t n, float* reward_out,
                 void* stream) {
  if (cfg == nullptr || obs == nullptr || reward_out == nullptr || n < 0) return LBSIM_EINVAL;
  if (cfg->num_servers < 1 || cfg->num_servers > LBSIM_MAX_SERVERS) return LBSIM_EINVAL;
  if (cfg->reward_metric < 0 || cfg->reward_metric > 8) return LBSIM_EINVAL;
  if (n == 0) return LBSIM_OK;
  hipLaunchKernelGGL(reward_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0,
                     (hipStream_t)stream, obs, n, cfg->num_servers, cfg->reward_metric,
                     cfg->reward_field, reward_out);
  return hipGetLastError() == hipSuccess ? LBSIM_OK : LBSIM_EDEVICE;
}

int lbsim_set_trace(lbsim_t* h, const uint32_t* gap_us, const float* work, int64_t rows,
                    void* stream) {
  if (h == nullptr) return LBSIM_EINVAL;
  if (!h->prm.trace) return fail(h, LBSIM_EINVAL, "lbsim_set_trace needs arrival_source TRACE");
  if (gap_us == nullptr || work == nullptr || rows < 1 || rows > (int64_t)0x7FFFFFFF)
    return fail(h, LBSIM_EINVAL, "trace: need device gap_us/work and 1 <= rows < 2^31");
  DeviceGuard g(h->device);
  const hipStream_t s = (hipStream_t)stream;
  if (hipStreamSynchronize(s) != hipSuccess) return fail(h, LBSIM_EDEVICE, "stream sync failed");
  if (h->trace_buf) {
    (void)hipFree(h->trace_buf);
    h->trace_buf = nullptr;
    h->prm.trace_rows = 0;
  }
  const size_t n = (size_t)rows;
  if (hipMalloc(&h->trace_buf, n * 8) != hipSuccess) {
    h->trace_buf = nullptr;
    return fail(h, LBSIM_ENOMEM, "hipMalloc(%zu) failed", n * 8);
  }
  uint32_t* g_dev = (uint32_t*)h->trace_buf;
  float* w_dev = (float*)(g_dev + n);
  if (hipMemcpyAsync(g_dev, gap_us, n * 4, hipMemcpyDeviceToDevice, s) != hipSuccess ||
      hipMemcpyAsync(w_dev, work, n * 4, hipMemcpyDeviceToDevice, s) != hipSuccess ||
      hipStreamSynchronize(s) != hipSuccess)
    return fail(h, LBSIM_EDEVICE, "trace copy failed");
  h->st.trace_gap = g_dev;
  h->st.trace_work = w_dev;
  h->prm.trace_rows = (uint32_t)rows;
  return LBSIM_OK;
}

int lbsim_agent_obs(const float* obs, int64_t n, int S, int num_agents, int servers_per_agent,
                    float* out, void* stream) {
  if (n < 0 || S < 1 || S > LBSIM_MAX_SERVERS || num_agents < 1 || servers_per_agent < 1 ||
      num_agents * servers_per_agent != S)
    return LBSIM_EINVAL;
  if (n == 0) return LBSIM_OK;
  if (!obs || !out) return LBSIM_EINVAL;
  const int64_t total = n * num_agents * (4 * servers_per_agent + 7 * S);
  hipLaunchKernelGGL(agent_obs_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0,
                     (hipStream_t)stream, obs, n, S, num_agents, servers_per_agent, out);
  return hipGetLastError() == hipSuccess ? LBSIM_OK : LBSIM_EDEVICE;
}

int lbsim_gru_gates(const float* gi, const float* gh, const float* h, float* h_out, int64_t B,
                    int H, void* stream) {
  if (B < 0 || H < 1 || (B > 0 && (!gi || !gh || !h || !h_out))) return LBSIM_EINVAL;
  if (B == 0) return LBSIM_OK;
  const int64_t n = B * H;
  hipLaunchKernelGGL(gru_gates_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0,
                     (hipStream_t)stream, gi, gh, h, h_out, B, H);
  return hipGetLastError() == hipSuccess ? LBSIM_OK : LBSIM_EDEVICE;
}

int lbsim_sac_head(const float* y, int64_t B, int A, float log_std_min, float log_std_max,
                   float action_scale, float action_bias, int deterministic, uint64_t seed,
                   uint32_t step, float* action_out, float* log_std_out, void* stream) {
  if (B < 0 || A < 1 || (B > 0 && (!y || !action_out))) return LBSIM_EINVAL;
  if (B == 0) return LBSIM_OK;
  const int64_t n = B * A;
  hipLaunchKernelGGL(sac_head_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0,
                     (hipStream_t)stream, y, B, A, log_std_min, log_std_max, action_scale,
                     action_bias, deterministic, (uint32_t)(seed & 0xFFFFFFFFull),
                     (uint32_t)(seed >> 32), step, action_out, log_std_out);
  return hipGetLastError() == hipSuccess ? LBSIM_OK : LBSIM_EDEVICE;
}

int lbsim_qmix_tail(const float* q, const float* w1, int64_t w1_ld, const float* b1,
                    int64_t b1_ld, const float* w2, int64_t w2_ld, const float* b2, int64_t b2_ld,
                    int64_t B, int A, int E, float* q_tot, void* stream) {
  if (B < 0 || A < 1 || E < 1) return LBSIM_EINVAL;
  if (B == 0) return LBSIM_OK;
  if (!q || !w1 || !b1 || !w2 || !b2 || !q_tot) return LBSIM_EINVAL;
  hipLaunchKernelGGL(qmix_tail_kernel, dim3((unsigned)((B + 255) / 256)), dim3(256), 0,
                     (hipStream_t)stream, q, w1, w1_ld, b1, b1_ld, w2, w2_ld, b2, b2_ld, B, A, E,
                     q_tot);
  return hipGetLastError() == hipSuccess ? LBSIM_OK : LBSIM_EDEVICE;
}

size_t lbsim_sac_actor_size(void) { return sizeof(lbsim_sac_actor_t); }
size_t lbsim_qmix_policy_size(void) { return sizeof(lbsim_qmix_policy_t); }

int lbsim_sac_actor_step(const lbsim_sac_actor_t* n, const float* state, float* hidden,
                         const uint8_t* reset_mask, int64_t B, int deterministic, uint64_t seed,
                         uint32_t step, float* action_out, float* log_std_out, void* stream) {
  if (n == nullptr || B < 0 || n->state_dim < 1 || n->state_dim > 512 || n->action_dim < 1 ||
      n->action_dim > 16)
    return LBSIM_EINVAL;
  if (n->gru_dim != 128 || n->hidden_dim != 256) return LBSIM_ENOTSUP;
  if (B == 0) return LBSIM_OK;
  if (!state || !hidden || !action_out || !n->w_ih || !n->w_hh || !n->b_ih || !n->b_hh ||
      !n->w1 || !n->b1 || !n->wh || !n->bh)
    return LBSIM_EINVAL;
  SacActorArgs a{};
  a.state = state;
  a.hidden = hidden;
  a.reset = reset_mask;
  a.w_ih = n->w_ih;
  a.w_hh = n->w_hh;
  a.b_ih = n->b_ih;
  a.b_hh = n->b_hh;
  a.w1 = n->w1;
  a.b1 = n->b1;
  a.wh = n->wh;
  a.bh = n->bh;
  a.action = action_out;
  a.log_std = log_std_out;
  a.B = B;
  a.I = n->state_dim;
  a.kxp = round16(n->state_dim);
  a.ld = fused_ld(std::max(a.kxp + 128, 256));
  a.A = n->action_dim;
  a.lo = n->log_std_min;
  a.hi = n->log_std_max;
  a.scale = n->action_scale;
  a.bias = n->action_bias;
  a.deterministic = deterministic;
  a.key0 = (uint32_t)(seed & 0xFFFFFFFFull);
  a.key1 = (uint32_t)(seed >> 32);
  a.step = step;
  a.step_dev = n->step_dev;
  int mt = fused_mt(B, 2);
  // the [R][ld] tile + split-K scratch of the heads ([4][nt][R][16], nt = ceil(2A / 16)): at A = 8
  // 20.6 KB per 16-env tile, 7 tiles per CU
  const int nt_heads = (2 * a.A + 15) / 16;
  // (the 32-env tile's heads keep two partials per row, not four: LBSIM_SAC_SPLIT_M, lbsim_fused.h)
  auto lds_of = [&](int m) {
    return (size_t)16 * m * (a.ld + (m == 2 && LBSIM_SAC_SPLIT_M ? 32 : 64) * nt_heads) * 4;
  };
  while (mt > 1 && lds_of(mt) > kFusedLdsMax) mt >>= 1;
  const size_t lds = lds_of(mt);
  const hipStream_t s = (hipStream_t)stream;
  return launch_sac_actor(a, B, mt, lds, s);
}

int lbsim_qmix_policy_step(const lbsim_qmix_policy_t* n, const float* obs, float* hidden,
                           const uint8_t* reset_mask, const float* state, int64_t B,
                           uint64_t seed, uint32_t step, int64_t* actions_out,
                           int32_t* server_actions_out, float* q_out, float* q_chosen_out,
                           float* q_tot_out, void* stream) {
  if (n == nullptr || B < 0) return LBSIM_EINVAL;
  const int A = n->num_agents, E = n->mixing_embed_dim, he = n->hypernet_embed_dim;
  if (A < 1 || A > 16 || n->obs_dim < 1 || n->obs_dim > 512 || n->state_dim < 1 ||
      n->state_dim > 512 || n->n_actions < 1 || n->n_actions > 16 || n->servers_per_agent < 1 ||
      !(n->epsilon >= 0.0f && n->epsilon <= 1.0f))
    return LBSIM_EINVAL;
  // layer widths the kernel is built for; the mixer's second-layer outputs [0, A E + E + 16)
  // must not reach hyper_b1's columns [3 he, 3 he + E) of the same LDS rows
  if (n->gru_dim != 64 || n->hidden_dim != 128 || E < 16 || E % 16 != 0 || he < 16 ||
      he % 16 != 0 || 3 * he + E > 256 || A * E / 16 + E / 16 + 1 > 16 || A * E + E + 16 > 3 * he)
    return LBSIM_ENOTSUP;
  if (B == 0) return LBSIM_OK;
  if (!obs || !hidden || !state || !actions_out || !q_tot_out || !n->w_ih || !n->w_hh ||
      !n->b_ih || !n->b_hh || !n->w1 || !n->b1 || !n->w2 || !n->b2 || !n->w3 || !n->b3 ||
      !n->m0 || !n->mb0 || !n->mw1 || !n->mbw1 || !n->mw2 || !n->mbw2 || !n->mb2 || !n->mbb2)
    return LBSIM_EINVAL;
  QmixArgs a{};
  a.obs = obs;
  a.hidden = hidden;
  a.reset = reset_mask;
  a.state = state;
  a.w_ih = n->w_ih;
  a.w_hh = n->w_hh;
  a.b_ih = n->b_ih;
  a.b_hh = n->b_hh;
  a.w1 = n->w1;
  a.b1 = n->b1;
  a.w2 = n->w2;
  a.b2 = n->b2;
  a.w3 = n->w3;
  a.b3 = n->b3;
  a.m0 = n->m0;
  a.mb0 = n->mb0;
  a.mw1 = n->mw1;
  a.mbw1 = n->mbw1;
  a.mw2 = n->mw2;
  a.mbw2 = n->mbw2;
  a.mb2 = n->mb2;
  a.mbb2 = n->mbb2;
  a.actions = actions_out;
  a.server_actions = server_actions_out;
  a.q_out = q_out;
  a.q_chosen = q_chosen_out;
  a.q_tot = q_tot_out;
  a.B = B;
  a.A = A;
  a.I = n->obs_dim;
  a.kxp = round16(n->obs_dim);
  a.Ds = n->state_dim;
  a.ksp = round16(n->state_dim);
  a.ld = fused_ld(std::max({a.kxp + 64, 128, a.ksp, 3 * he + E}));
  a.n_act = n->n_actions;
  a.k = n->servers_per_agent;
  a.he = he;
  a.E = E;
  a.epsilon = n->epsilon;
  a.key0 = (uint32_t)(seed & 0xFFFFFFFFull);
  a.key1 = (uint32_t)(seed >> 32);
  a.step = step;
  a.step_dev = n->step_dev;
  auto lds_of = [&](int mt) {
    const size_t R = 16 * (size_t)mt;
    return (R * a.ld + (size_t)A * R * 16 + R * A + 64 * R) * 4;  // + split-K scratch
  };
  int mt = fused_mt(B);
  while (mt > 1 && lds_of(mt) > kFusedLdsMax) mt >>= 1;
  const hipStream_t s = (hipStream_t)stream;
  // LBSIM_QMIX_KERNEL = tile | wave | pair (default: pair when A = 4, else wave)
  static const int form = [] {
    const char* e = std::getenv("LBSIM_QMIX_KERNEL");
    if (e != nullptr && std::strcmp(e, "tile") == 0) return 0;
    if (e != nullptr && std::strcmp(e, "wave") == 0) return 1;
    return 2;
  }();
  if (mt == 1 && form != 0) {  // one or two waves per agent, 16 envs per workgroup
    a.lda = fused_ld(std::max(a.kxp + 64, 128));
    if (form == 2 && A == 4) {  // two waves per agent: 8-wave workgroups
      // + the mixer's state rows, staged at the start when they fit (a.sld = 0: staged by the
      // mixer, as the other forms)
      const size_t base = ((size_t)4 * 16 * a.lda + 2 * (size_t)A * 16 * 16 + 16 * (size_t)A) * 4;
      a.sld = fused_ld(a.ksp);
      if (base + (size_t)16 * a.sld * 4 > kFusedLdsMax) a.sld = 0;
      const size_t lds = base + (size_t)16 * a.sld * 4;
      if (a.ld > 4 * a.lda || lds > kFusedLdsMax) return LBSIM_ENOTSUP;
      return launch_qmix_policy(a, B, 2, 1, lds, s);
    }
    const size_t lds = ((size_t)4 * 16 * a.lda + (size_t)A * 16 * 16 + 16 * (size_t)A) * 4;
    if (a.ld > 4 * a.lda || lds > kFusedLdsMax) return LBSIM_ENOTSUP;
    return launch_qmix_policy(a, B, 1, 1, lds, s);
  }
  return launch_qmix_policy(a, B, 0, mt, lds_of(mt), s);
}

int lbsim_alias_tables(const float* weights, int64_t n, int S, float* odd_out, int32_t* alias_out,
                       int32_t* active_out, void* stream) {
  if (n < 0 || S < 1 || S > LBSIM_MAX_SERVERS) return LBSIM_EINVAL;
  if (n == 0) return LBSIM_OK;
  if (!weights || !odd_out || !alias_out || !active_out) return LBSIM_EINVAL;
  hipLaunchKernelGGL(alias_tables_kernel, dim3((unsigned)((n + 63) / 64)), dim3(64), 0,
                     (hipStream_t)stream, weights, n, S, odd_out, alias_out, active_out);
  return hipGetLastError() == hipSuccess ? LBSIM_OK : LBSIM_EDEVICE;
}

int lbsim_vose_tables(const float* weights, int64_t n, int S, float* prob_out,
                      uint32_t* alias_out, void* stream) {
  if (n < 0 || S < 1 || S > LBSIM_MAX_SERVERS) return LBSIM_EINVAL;
  if (n == 0) return LBSIM_OK;
  if (!weights || !prob_out || !alias_out) return LBSIM_EINVAL;
  hipLaunchKernelGGL(vose_tables_kernel, dim3((unsigned)((n + 63) / 64)), dim3(64), 0,
                     (hipStream_t)stream, weights, n, S, prob_out, alias_out);
  return hipGetLastError() == hipSuccess ? LBSIM_OK : LBSIM_EDEVICE;
}

int lbsim_vose_sample(const float* prob, const uint32_t* alias, int64_t n, int S,
                      uint32_t* state_io, int64_t k, int32_t* idx_out, uint64_t* hist_out,
                      void* stream) {
  if (n < 0 || S < 1 || S > LBSIM_MAX_SERVERS || k < 0 || k > INT32_MAX) return LBSIM_EINVAL;
  if (n == 0) return LBSIM_OK;
  if (!prob || !alias || !state_io) return LBSIM_EINVAL;
  hipLaunchKernelGGL(vose_sample_kernel, dim3((unsigned)((n + 63) / 64)), dim3(64), 0,
                     (hipStream_t)stream, prob, alias, n, S, state_io, k, idx_out, hist_out);
  return hipGetLastError() == hipSuccess ? LBSIM_OK : LBSIM_EDEVICE;
}

int lbsim_reservoir_features(const float* values, const uint32_t* ts_ms, const uint32_t* counts,
                             int64_t n, float decay_factor, float* feats_out, void* stream) {
  if (values == nullptr || ts_ms == nullptr || counts == nullptr || feats_out == nullptr || n < 0)
    return LBSIM_EINVAL;
  if (!(decay_factor > 0.0f) || !(decay_factor < 1.0f)) return LBSIM_EINVAL;
  if (n == 0) return LBSIM_OK;
  const float c = (float)(std::log2((double)decay_factor) / 1000.0);
  hipLaunchKernelGGL(features_kernel, dim3((unsigned)((n + 3) / 4)), dim3(64), 0,
                     (hipStream_t)stream, values, ts_ms, counts, n, c, feats_out);
  return hipGetLastError() == hipSuccess ? LBSIM_OK : LBSIM_EDEVICE;
}

int lbsim_vpp_export(lbsim_t* h, int64_t env_begin, int64_t n_envs, float* tv_out,
                     int32_t* n_flow_on_out, float* ts_out, void* stream) {
  if (h == nullptr) return LBSIM_EINVAL;
  if (env_begin < 0 || n_envs < 0 || env_begin + n_envs > h->B)
    return fail(h, LBSIM_EINVAL, "envs [%lld, %lld) outside [0, %d)", (long long)env_begin,
                (long long)(env_begin + n_envs), h->B);
  if (!h->initialised) return fail(h, LBSIM_EINVAL, "call lbsim_reset before lbsim_vpp_export");
  if (n_envs == 0) return LBSIM_OK;
  if (tv_out == nullptr) return fail(h, LBSIM_EINVAL, "tv_out is NULL");
  DeviceGuard g(h->device);
  hipLaunchKernelGGL(vpp_export_kernel, dim3((unsigned)(n_envs * h->S)), dim3(64), 0,
                     (hipStream_t)stream, h->st, h->prm, env_begin, n_envs,
                     reinterpret_cast<float2*>(tv_out), n_flow_on_out, ts_out);
  return launch_check(h, "vpp_export_kernel");
}

int lbsim_vpp_features(const float* tv, const float* ts, int64_t res_per_ts, int64_t n,
                       double decay, double* feats_out, void* stream) {
  if (n < 0 || res_per_ts < 1 || !(decay > 0.0) || !(decay < 1.0)) return LBSIM_EINVAL;
  if (n == 0) return LBSIM_OK;
  if (!tv || !ts || !feats_out || n > 0x7FFFFFFF) return LBSIM_EINVAL;
  hipLaunchKernelGGL(vpp_features_kernel, dim3((unsigned)n), dim3(64), 0, (hipStream_t)stream,
                     reinterpret_cast<const float2*>(tv), ts, res_per_ts, n, decay, feats_out);
  return hipGetLastError() == hipSuccess ? LBSIM_OK : LBSIM_EDEVICE;
}

int lbsim_profile_begin(lbsim_t* h, int max_launches) {
  if (h == nullptr || max_launches < 1) return LBSIM_EINVAL;
  DeviceGuard g(h->device);
  Profiler& p = h->prof;
  const size_t need = 2 * (size_t)max_launches;
  // Timing-only events: no system-scope fence when they are recorded.  A default event's record
  // writes back and invalidates the caches between the launches it brackets, which costs the
  // timed step itself (the caller synchronises the device before reading the times, so nothing
  // needs the fence).  LBSIM_PROFILE_FENCE=1 keeps the default events (A/B).
  static const unsigned flags = [] {
    const char* e = std::getenv("LBSIM_PROFILE_FENCE");
    return (e != nullptr && std::strcmp(e, "1") == 0) ? (unsigned)hipEventDefault
                                                       : (unsigned)hipEventDisableSystemFence;
  }();
  while (p.ev.size() < need) {
    hipEvent_t e;
    if (hipEventCreateWithFlags(&e, flags) != hipSuccess)
      return fail(h, LBSIM_EDEVICE, "hipEventCreateWithFlags failed");
    p.ev.push_back(e);
  }
  p.used = 0;
  p.cap = need;
  p.cls.clear();
  p.beg.clear();
  p.end.clear();
  p.chain = false;
  p.chain_ev = -1;
  p.on = true;
  return LBSIM_OK;
}

int lbsim_profile_end(lbsim_t* h, double* ms_out, int64_t* count_out) {
  return lbsim_profile_end_ex(h, ms_out, count_out, 4);
}

int lbsim_profile_end_ex(lbsim_t* h, double* ms_out, int64_t* count_out, int n_classes) {
  if (h == nullptr || n_classes < 0 || n_classes > LBSIM_PROFILE_CLASSES) return LBSIM_EINVAL;
  DeviceGuard g(h->device);
  Profiler& p = h->prof;
  double ms[LBSIM_PROFILE_CLASSES] = {0, 0, 0, 0, 0};
  int64_t cnt[LBSIM_PROFILE_CLASSES] = {0, 0, 0, 0, 0};
  if (p.used > 0 && hipEventSynchronize(p.ev[p.used - 1]) != hipSuccess)
    return fail(h, LBSIM_EDEVICE, "hipEventSynchronize failed");
  for (size_t i = 0; i < p.cls.size(); ++i) {
    float t = 0.0f;
    if (hipEventElapsedTime(&t, p.ev[p.beg[i]], p.ev[p.end[i]]) != hipSuccess)
      return fail(h, LBSIM_EDEVICE, "hipEventElapsedTime failed");
    ms[p.cls[i]] += t;
    cnt[p.cls[i]] += 1;
  }
  p.on = false;
  p.used = 0;
  p.cls.clear();
  p.beg.clear();
  p.end.clear();
  p.chain_ev = -1;
  for (int i = 0; i < n_classes; ++i) {
    if (ms_out) ms_out[i] = ms[i];
    if (count_out) count_out[i] = cnt[i];
  }
  return LBSIM_OK;
}

int lbsim_launch_names(lbsim_t* h, int which, char* buf, size_t buf_len) {
  if (h == nullptr || which < 0 || which > 1 || buf == nullptr || buf_len == 0)
    return LBSIM_EINVAL;
  DeviceGuard g(h->device);
  std::string txt;
  for (const auto& [cls, fn] : h->launched[which]) {
    const char* raw = hipKernelNameRefByPtr(fn, nullptr);
    if (!txt.empty()) txt += ';';
    txt += std::to_string(cls) + "=" + short_kernel_name(raw);
  }
  // more launches than the log holds: a marker no counter file is keyed by
  if (h->launched_lost[which] > 0)
    txt += (txt.empty() ? "" : ";") + std::string("-1=truncated(") +
           std::to_string(h->launched_lost[which]) + " more)";
  if (txt.size() + 1 > buf_len)
    return fail(h, LBSIM_ESHAPE, "launch names need %zu bytes", txt.size() + 1);
  memcpy(buf, txt.c_str(), txt.size() + 1);
  return LBSIM_OK;
}

int lbsim_state_size(const lbsim_t* h, size_t* bytes_out) {
  if (h == nullptr || bytes_out == nullptr) return LBSIM_EINVAL;
  size_t t = 0;
  for (const Section& s : sections(const_cast<lbsim_t*>(h))) t += s.bytes;
  *bytes_out = t;
  return LBSIM_OK;
}

int lbsim_get_state(lbsim_t* h, void* host_buf, size_t bytes) {
  if (h == nullptr || host_buf == nullptr) return LBSIM_EINVAL;
  size_t need = 0;
  lbsim_state_size(h, &need);
  if (bytes != need) return fail(h, LBSIM_ESHAPE, "state buffer is %zu bytes, need %zu", bytes, need);
  DeviceGuard g(h->device);
  if (hipDeviceSynchronize() != hipSuccess) return fail(h, LBSIM_EDEVICE, "sync failed");
  char* dst = (char*)host_buf;
  for (const Section& s : sections(h)) {
    if (hipMemcpy(dst, *s.ptr, s.bytes, hipMemcpyDeviceToHost) != hipSuccess)
      return fail(h, LBSIM_EDEVICE, "hipMemcpy D2H failed");
    dst += s.bytes;
  }
  return LBSIM_OK;
}

int lbsim_set_state(lbsim_t* h, const void* host_buf, size_t bytes) {
  if (h == nullptr || host_buf == nullptr) return LBSIM_EINVAL;
  size_t need = 0;
  lbsim_state_size(h, &need);
  if (bytes != need) return fail(h, LBSIM_ESHAPE, "state buffer is %zu bytes, need %zu", bytes, need);
  DeviceGuard g(h->device);
  if (hipDeviceSynchronize() != hipSuccess) return fail(h, LBSIM_EDEVICE, "sync failed");
  const char* src = (const char*)host_buf;
  for (const Section& s : sections(h)) {
    if (hipMemcpy(*s.ptr, src, s.bytes, hipMemcpyHostToDevice) != hipSuccess)
      return fail(h, LBSIM_EDEVICE, "hipMemcpy H2D failed");
    src += s.bytes;
  }
  h->initialised = true;
  return LBSIM_OK;
}

}  // extern "C"
