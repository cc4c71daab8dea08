/*
 * lbsim.h — C ABI of the MI355X-native vectorised load-balancing environment.
 *
 * One handle = B independent LB environments (a shard of the global env range) resident in the
 * HBM of one GPU.  Every entry point is extern "C", takes plain pointers and sizes, never throws,
 * and returns an int status (LBSIM_OK or a negative LBSIM_E* code; message via lbsim_last_error).
 *
 * Buffers passed to reset/step/reward/features are DEVICE pointers owned by the caller (e.g. a
 * torch tensor's data_ptr()); nothing is allocated inside lbsim_reset/lbsim_step, so both can be
 * captured into a hipGraph.  `stream` is a hipStream_t (NULL = default stream).  Calls on one
 * handle are stream-ordered and NOT thread-safe across host threads.
 *
 * Reference interfaces replaced (paths relative to the MARLLB reference tree):
 *   LoadBalanceEnv.__init__ / _setup_spaces   simulation-mode/problem-03-rl-environment/src/env.py:71-184
 *   LoadBalanceEnv.reset                      env.py:186-213
 *   LoadBalanceEnv.step                       env.py:215-286
 *   LoadBalanceEnv.seed / close               env.py:321-330
 *   RewardFunction.compute + active rule      src/rewards.py:290-381, env.py:391-423
 *   ReservoirSampler.add / get_features       problem-01-reservoir-sampling/src/reservoir.py:50-196
 *   C twin reservoir_add / compute_stats      problem-01-reservoir-sampling/src/reservoir.h:118-268
 *   server assignment SED/SED2/LSQ/LSQ2       src/vpp/lb/node.c:388-441
 *   flow-completion samples (fct, duration)   src/vpp/lb/lbhash.h:87-172 (duration: :129-136)
 * Full semantics: DESIGN.md §3 (the simulator spec the GPU kernels and oracle/ both implement).
 */
#ifndef LBSIM_H
#define LBSIM_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define LBSIM_ABI_VERSION 10 /* 10: lbsim_step_outputs_t ends with done_word / done_value (the */
                             /* one-env completion word); 9: lost-FIN guesses deferred to their */
                             /* wrap-up time, reservoir_mode VPP                                 */
#define LBSIM_MAX_SERVERS 64   /* S <= 64: BASELINE configs[4] read literally is 4 agents x 16 */
                               /* servers = 64 (S > 16: server-per-lane dynamics only)       */
#define LBSIM_RESERVOIR_K 128  /* reservoir.py:31 capacity=128, reservoir.h:24               */
#define LBSIM_NUM_FEATURES 11  /* env.py:46-48 (S, 11) observation                           */
#define LBSIM_MAX_DISCRETE 8

/* ---- status codes (never thrown across the ABI) ---- */
#define LBSIM_OK 0
#define LBSIM_EINVAL (-1)  /* bad argument / config (Python facade re-raises ValueError)      */
#define LBSIM_ENOMEM (-2)  /* device allocation failed                                        */
#define LBSIM_EDEVICE (-3) /* HIP runtime error (no GPU, launch failure, ...)                 */
#define LBSIM_ESHAPE (-4)  /* buffer size does not match the handle's B/S                     */
#define LBSIM_ENOTSUP (-5) /* option not built in this version                                */

/* ---- enums ---- */
enum lbsim_action_type { LBSIM_ACTION_DISCRETE = 0, LBSIM_ACTION_CONTINUOUS = 1 };
enum lbsim_dtype { LBSIM_DTYPE_I32 = 0, LBSIM_DTYPE_I64 = 1, LBSIM_DTYPE_F32 = 2 };

/* rewards.py:297-307 SUPPORTED_METRICS, same order */
enum lbsim_reward_metric {
  LBSIM_METRIC_JAIN = 0,
  LBSIM_METRIC_VARIANCE = 1,
  LBSIM_METRIC_STD = 2,
  LBSIM_METRIC_CV = 3,
  LBSIM_METRIC_MAX = 4,
  LBSIM_METRIC_MIN = 5,
  LBSIM_METRIC_PRODUCT = 6,
  LBSIM_METRIC_RANGE = 7,
  LBSIM_METRIC_GINI = 8
};

/* node.c:393-441: LB_SED, LB_SED2 (power of two), LB_LSQ, LB_LSQ2; node.c:442-460 LB_ALIAS with
 * the table of gen_alias (src/lb/shm_proxy.py:127-146) over the action weights */
enum lbsim_assign_policy {
  LBSIM_POLICY_SED = 0,
  LBSIM_POLICY_SED2 = 1,
  LBSIM_POLICY_LSQ = 2,
  LBSIM_POLICY_LSQ2 = 3,
  LBSIM_POLICY_ALIAS = 4
};

/* POISSON: exponential gaps of mean 1/arrival_rate, Exp(1) work.  TRACE: replay of an arrival
 * trace set with lbsim_set_trace (data/trace/poisson_for_loop/rate_N.csv). */
enum lbsim_arrival_source { LBSIM_ARRIVAL_POISSON = 0, LBSIM_ARRIVAL_TRACE = 1 };

/* The flow-duration sample of a completed flow (the reservoir behind obs columns 6-10 and the
 * default reward field).  AGE (default): the flow's age at its last data packet, tc - t_arrival --
 * VPP records time_now - t_init on every plain ACK after the first (src/vpp/lb/lbhash.h:129-136),
 * the last one at the flow's completion, so the backlog wait is included (problem-01 README:
 * "from first packet to last packet").  SERVICE: tc - max(t_arrival, predecessor's tc), the
 * service time alone (the ABI-6 sample; independent of the queue, so a duration-based reward
 * does not see the policy). */
enum lbsim_duration_mode { LBSIM_DURATION_AGE = 0, LBSIM_DURATION_SERVICE = 1 };

/* Observation column 0 (n_flow_on).  QUEUE (default): the flows in flight at the server.  VPP:
 * the data plane's as_stat_t n_flow_on, +1 at a flow's first ACK and -1 at its RSTACK
 * (src/vpp/lb/lbhash.h:116-120,138-142,167): a lost-FIN flow is never decremented (the decrement
 * is commented out, lbhash.h:193,214), so the column is the flows in flight plus the server's
 * lost-FIN flows completed since the episode start (or its last failure).  Only differs from
 * QUEUE with lost_fin_prob > 0. */
enum lbsim_n_flow_on_mode { LBSIM_NFLOW_QUEUE = 0, LBSIM_NFLOW_VPP = 1 };

/* Reservoir replacement rule.  ALGR (default): problem-01's Algorithm R (reservoir.py:64-85) --
 * slot `count` while count < 128, else slot j = randint(0, count + 1) if j < 128; observe takes
 * the features over the first min(count, 128) slots.  VPP: the live data plane's rule
 * (src/vpp/lb/lbhash.h:108,179 `res_id = rand() % RESERVOIR_N_BIN`, register_reservoir_as): every
 * sample overwrites slot rand() % 128 unconditionally, and the bins start zeroed at reset (VPP's
 * zeroed shm), so the upstream agent's process_reservoir over ALL 128 bins (shm_proxy.py:518-543,
 * lbsim_vpp_export / feature_mode "upstream") sees a sparse, recency-biased reservoir until every
 * bin was hit.  The counts still count samples. */
enum lbsim_reservoir_mode { LBSIM_RESERVOIR_ALGR = 0, LBSIM_RESERVOIR_VPP = 1 };

/* Dynamics-kernel mapping; every choice produces the same bits.  AUTO = SERVER_PER_LANE (faster
 * than one lane per env at every measured shape). */
enum lbsim_dyn_mapping {
  LBSIM_DYN_AUTO = 0,
  LBSIM_DYN_ENV_PER_LANE = 1,    /* one lane = one env                                        */
  LBSIM_DYN_SERVER_PER_LANE = 2  /* a group of G lanes = one env, one lane per server: G =     */
                                 /* pow2 >= S, except S <= 4 on small batches (B*4/64 <= half */
                                 /* the device's SIMDs), which get G = 8 (twice the waves);    */
                                 /* S <= 8 batches of at most 4 (S <= 4) or 2 envs per SIMD   */
                                 /* (Q <= 32, no ALIAS) run one WAVE per env    */
};

/* The dynamics kernel a handle's launches use (lbsim_dynamics_kernel). */
enum lbsim_dyn_kernel {
  LBSIM_DYN_KERNEL_ENV_LANE = 0,  /* dynamics_kernel: one lane per env                        */
  LBSIM_DYN_KERNEL_GROUP = 1,     /* dynamics_group_kernel: one lane per server, G-lane groups */
  LBSIM_DYN_KERNEL_WAVE = 2       /* dynamics_wave_kernel: one wave per env                    */
};

/* How lbsim_step runs; every choice produces the same bits.  FUSED: one launch per step whose
 * workgroups simulate their envs and then observe them: step_wave_kernel for
 * one-wave-per-env handles, fused_step_kernel for server-per-lane groups of <= 16 lanes (else
 * SPLIT); SPLIT: a dynamics launch and an observe launch.  AUTO: the one-launch step_wave_kernel
 * for one-wave-per-env handles with S <= 8 and at most 4 envs per SIMD (the single-env facade
 * and BASELINE configs[1]'s 4096 x 4 on 256 CUs; LBSIM_STEP_WAVE_MAX_B overrides the limit),
 * else SPLIT (the server-per-lane fused form measured slower).  The environment
 * variable LBSIM_STEP_KERNEL=split|fused overrides AUTO. */
enum lbsim_step_kernel { LBSIM_STEP_AUTO = 0, LBSIM_STEP_SPLIT = 1, LBSIM_STEP_FUSED = 2 };

/*
 * POD configuration.  Mirrors the LoadBalanceEnv kwargs (env.py:71-87) plus the simulator knobs
 * the reference leaves implicit.  Fill with lbsim_config_default() and override.
 */
typedef struct lbsim_config {
  int32_t num_envs;          /* B: envs in this handle (this GPU's shard)                    */
  int32_t num_servers;       /* S: 1..LBSIM_MAX_SERVERS                         env.py:73   */
  int64_t env_id_offset;     /* global id of local env 0 (RNG key; sharding-invariant)       */
  uint64_t seed;             /* Philox4x32-10 key                               env.py:86   */
  int32_t action_type;       /* lbsim_action_type                               env.py:74   */
  int32_t num_discrete;      /* len(discrete_weights)                           env.py:75   */
  float discrete_weights[LBSIM_MAX_DISCRETE]; /* default [1.0, 1.5, 2.0]         env.py:69   */
  float min_weight;          /* continuous clip lower bound, default 0.1        env.py:77   */
  float max_weight;          /* continuous clip upper bound, default 10.0       env.py:76   */
  int32_t reward_metric;     /* lbsim_reward_metric, default JAIN               env.py:78   */
  int32_t reward_field;      /* obs column 0..10 (default 10 =                               */
                             /* 'flow_duration_avg_decay', env.py:79,377-381);               */
                             /* -1 = field name unknown -> reward 0.0 (rewards.py:375-376)  */
  float step_interval;       /* simulated seconds per step, default 0.25        env.py:80   */
  int32_t max_steps;         /* done when episode step >= max_steps (10000)     env.py:81   */
  int32_t normalize_obs;     /* running mean/std normalisation    env.py:85,450-470   */
  int32_t assign_policy;     /* lbsim_assign_policy, default SED                             */
  int32_t arrival_source;    /* lbsim_arrival_source, default POISSON                        */
  float arrival_rate;        /* lambda, flows/s per env, default 400 (poisson_for_loop);     */
                             /* TRACE: informational (the trace sets the rate)               */
  float server_rate[LBSIM_MAX_SERVERS]; /* mu_s, flows/s each server can serve (Exp work)   */
  float decay_factor;        /* reservoir decay, default 0.9          reservoir.py:106       */
  int32_t queue_capacity;    /* Q: max flows in flight per server (1..64), default 32       */
  int32_t warmup_steps;      /* simulated steps run inside reset() with weights 1.0         */
  int32_t dyn_mapping;       /* lbsim_dyn_mapping: how envs map onto lanes (results identical) */
  int32_t step_kernel;       /* lbsim_step_kernel: one fused launch or two (results identical) */
  /* Lost-FIN flows (VPP's timed-out flow sample, src/vpp/lb/lbhash.h:175-217, stats.h:27): a
   * flow's FIN/RST is missed with probability lost_fin_prob; its flow-table entry expires
   * flow_timeout_s after its last packet and the next flow hashed into its bucket (an exponential
   * wait of mean flow_buckets / arrival_rate) wraps it up with fct = now - t_init - 40 s.  That
   * signed-us sample enters the server's fct reservoir at the wrap-up time (completion +
   * flow_timeout + wait), stamped with it, in time order with the server's other samples: each
   * server holds its pending guesses in a ring of lost_fin_pending entries sorted by due time (a
   * guess arriving at a full ring is dropped and counted).  The flow's duration sample is
   * recorded at its completion, so under lost-FIN the fct and duration reservoirs are separate
   * (own counts, own timestamps).  0 = off. */
  float lost_fin_prob;       /* [0, 1], default 0                                            */
  float flow_timeout_s;      /* the lb plugin's flow timeout, default 40 (lb.c:1437)        */
  int32_t flow_buckets;      /* sticky buckets per core, default 1024 (lb.h:46)             */
  /* Server failure / recovery (THEORY.md §6.4 "server_failure ~ Bernoulli(p_fail)"): at the
   * start of each step an up server fails with probability fail_prob (its queued flows are lost
   * and counted as dropped, its reservoirs emptied: an all-zero observation row, inactive in the
   * reward, env.py:410-413) and a down server recovers with probability recover_prob.  A down
   * server takes no flows (as a full one).  fail_prob 0 = off (no state is allocated). */
  float fail_prob;           /* [0, 1], default 0                                            */
  float recover_prob;        /* [0, 1], default 0.1                                          */
  /* Next-step auto-reset (gymnasium's NEXT_STEP autoreset mode): lbsim_step resets, in place of
   * stepping, every env whose previous step returned done (episode step >= max_steps), ignoring
   * its action; that env's outputs are its reset observation, reward 0, done 0, episode length
   * and return 0, assignment counts 0.  Inside the step launches: no extra kernel, so a captured
   * step needs no masked-reset launch; such a handle steps in two launches
   * (dynamics, observe), not the one-launch forms.  0 = off (the caller resets).             */
  int32_t next_step_reset;
  int32_t duration_mode;     /* lbsim_duration_mode, default AGE            */
  int32_t n_flow_on_mode;    /* lbsim_n_flow_on_mode, default QUEUE         */
  int32_t lost_fin_pending;  /* pending lost-FIN guesses held per server, 1..4096, default 256 */
  int32_t reservoir_mode;    /* lbsim_reservoir_mode, default ALGR           */
} lbsim_config_t;

typedef struct lbsim lbsim_t; /* opaque handle */

/* Library identity; never fails, no GPU needed. */
const char* lbsim_version(void);
int lbsim_abi_version(void);

/* Fill *cfg with the reference defaults (env.py:71-87) and the simulator defaults. */
int lbsim_config_default(lbsim_config_t* cfg);

/* Validate a config without touching the GPU (ValueError paths of env.py:184, rewards.py:321). */
int lbsim_config_validate(const lbsim_config_t* cfg, char* msg, size_t msg_len);

/* Allocate device state for cfg->num_envs envs on `device`.  Replaces LoadBalanceEnv.__init__. */
int lbsim_create(const lbsim_config_t* cfg, int device, lbsim_t** out);

/* Free device state.  Replaces LoadBalanceEnv.close (env.py:321-325). */
int lbsim_destroy(lbsim_t* h);

/* Thread-local message of the last failure on this handle (or of the last create if h==NULL). */
const char* lbsim_last_error(const lbsim_t* h);

/* Re-key the RNG and rewind every env's episode counter (env.py:327-330 seed()). */
int lbsim_seed(lbsim_t* h, uint64_t seed);

/* Which dynamics kernel (lbsim_dyn_kernel) this handle's step and reset launches use, for the
 * handle's shape, config and the LBSIM_DYN_* environment overrides; -1 on a NULL handle.  No
 * GPU work (measurement labels; the reference has no counterpart). */
int lbsim_dynamics_kernel(const lbsim_t* h);

/*
 * Reset the envs whose env_mask[b] != 0 (env_mask == NULL: all envs) and write their first
 * observation into obs_out[b, S, 11] (f32); rows of unmasked envs are left untouched.
 * Replaces LoadBalanceEnv.reset (env.py:186-213).
 */
int lbsim_reset(lbsim_t* h, const uint8_t* env_mask, float* obs_out, void* stream);

/*
 * Advance every env by one step of step_interval simulated seconds.
 *   action        [B, S]: discrete indices (I32 or I64) or continuous weights (F32)
 *   obs_out       [B, S, 11] f32   reward_out [B] f32   done_out [B] u8
 *   assign_count_out [B, S] i32 (optional, NULL = skip): flows assigned per server this step
 * Replaces LoadBalanceEnv.step (env.py:215-286).
 */
int lbsim_step(lbsim_t* h, const void* action, int action_dtype, float* obs_out,
               float* reward_out, uint8_t* done_out, int32_t* assign_count_out, void* stream);

/*
 * Optional outputs of one step, all device pointers, NULL = not wanted.  Written by the same
 * launch as obs/reward/done (no extra kernel, no host sync).
 */
typedef struct lbsim_step_outputs {
  float* obs;              /* [B, S, 11] f32 observation (normalised if normalize_obs)        */
  float* reward;           /* [B] f32                                                         */
  uint8_t* done;           /* [B] u8                                                          */
  int32_t* assign_count;   /* [B, S] i32 flows assigned per server this step                  */
  float* raw_obs;          /* [B, S, 11] f32 un-normalised obs (reward/active_servers basis)  */
  int32_t* episode_length; /* [B] i32 step count of the episode after this step (info['step'])*/
  double* episode_return;  /* [B] f64 return of the episode after this step                   */
  /* problem-05 MultiAgentLoadBalanceEnv facade (multi_agent_env.py:152-188, 240-258), written by
   * the same launch; num_agents * servers_per_agent must equal S when either is requested */
  float* agent_obs;        /* [B, A, 4k + 7S] f32: agent a = flat[4ak, 4(a+1)k) ++ flat[4S:] of */
                           /* the returned (S, 11) rows                                        */
  float* state;            /* [B, 4S + 10] f32 get_state(): zeros, episode step / max_steps, A */
  int32_t num_agents;      /* A                                                               */
  int32_t servers_per_agent; /* k                                                             */
  /* Completion word (one-env handles, B = 1, lbsim_step_ex only; NULL = none): the step launch
   * stores done_value to *done_word (device-accessible host memory) after every other output of
   * the step, with a system-scope release, so a host polling the word sees the outputs complete
   * without a stream synchronisation (the single-env facade's step, problem-04 Trainer path). */
  uint32_t* done_word;
  uint32_t done_value;
} lbsim_step_outputs_t;

/* lbsim_step with every output optional except obs, reward and done. */
int lbsim_step_ex(lbsim_t* h, const void* action, int action_dtype,
                  const lbsim_step_outputs_t* out, void* stream);

/* lbsim_reset with the step outputs that make sense after a reset: out->obs (required),
 * out->raw_obs, out->agent_obs and out->state (rows of reset envs only). */
int lbsim_reset_ex(lbsim_t* h, const uint8_t* env_mask, const lbsim_step_outputs_t* out,
                   void* stream);

/* sizeof(lbsim_config_t) / sizeof(lbsim_step_outputs_t) for binding-side layout checks. */
size_t lbsim_config_size(void);
size_t lbsim_step_outputs_size(void);

/* Per-env episode length (i32 [B]) and return (f64 [B]) into device buffers (info['episode']). */
int lbsim_episode_stats(lbsim_t* h, int32_t* length_out, double* return_out, void* stream);

/* Accounting of the last step (bench.py's algorithmic bytes; synchronises the device): HOST
 * stats_out[0] = reservoir slots the last dynamics launch wrote (popcount of the written-slot
 * masks: each an 8-B record store, + 4 B with a duration plane), stats_out[1] = flows in flight after it (sum of the queue
 * counts: ring entries carried into the next step). */
int lbsim_step_stats(lbsim_t* h, int64_t* stats_out);

/* Stateless reward of given raw observations obs[n, S, 11] -> reward_out[n] (f32), using
 * cfg->reward_metric / reward_field and the active rule any(obs[s] > 0) (env.py:410-417,
 * rewards.py:329-381). */
int lbsim_reward(const lbsim_config_t* cfg, const float* obs, int64_t n, float* reward_out,
                 void* stream);

/* Stateless reservoir features: for r in [0, n): values[r, K] f32, ts_ms[r, K] u32 sample
 * timestamps (integer ms), counts[r] u32 (samples seen; min(count, K) valid slots) ->
 * feats_out[r, 5] = {mean, p90, std, mean_decay, p90_decay} (reservoir.py:105-196). */
int lbsim_reservoir_features(const float* values, const uint32_t* ts_ms, const uint32_t* counts,
                             int64_t n, float decay_factor, float* feats_out, void* stream);

/* Stateless: n alias tables of S weights each (weights[n, S] f32, device pointers): gen_alias
 * (src/lb/shm_proxy.py:127-146) over the weights > 0 of each row, as the ALIAS policy builds it
 * every step -> odd_out[n, S] (float32, as packed into shm.h alias_t), alias_out[n, S] (position
 * in the row's active list), active_out[n, S] (server of each active position; -1 past the end).
 * Entries past a row's active count are (1, 0, -1). */
/* Stateless: problem-05 per-agent observations (multi_agent_env.py:152-188) of n flattened
 * (S, 11) observations (device pointers), num_agents * servers_per_agent == S.  Agent a gets the
 * 4-value slices of the flattened obs for its servers -- flat[4 a k : 4 (a+1) k], the wrapper's
 * `server_features_per_server = 4` -- then flat[4 S :]: out[n, A, 4 k + 7 S] (128 at 4 x 4). */
int lbsim_agent_obs(const float* obs, int64_t n, int S, int num_agents, int servers_per_agent,
                    float* out, void* stream);

/* Policy-network epilogues (device pointers, row-major), used between hipBLASLt GEMMs by
 * marllb_amd/policies.py for problem-04 PolicyNetwork (networks.py:82-146) and problem-05
 * AgentQNetwork (agent_network.py:63-87):
 *  lbsim_gru_gates: torch.nn.GRU cell from gi = x W_ih^T + b_ih, gh = h W_hh^T + b_hh ([B, 3H],
 *    gates r, z, n): h_out = (1 - z) n + z h, r = sig(gi_r + gh_r), z = sig(gi_z + gh_z),
 *    n = tanh(gi_n + r gh_n).
 *  lbsim_sac_head: y = [B, 2A] = [mean | log_std]: log_std clamped to [min, max]; action =
 *    tanh(mean) (deterministic) or tanh(mean + exp(log_std) eps), eps ~ N(0,1) from Philox
 *    (key = seed, counter = (row, step, a, 3 << 24)); times scale plus bias.  log_std_out optional. */
int lbsim_gru_gates(const float* gi, const float* gh, const float* h, float* h_out, int64_t B,
                    int H, void* stream);
int lbsim_sac_head(const float* y, int64_t B, int A, float log_std_min, float log_std_max,
                   float action_scale, float action_bias, int deterministic, uint64_t seed,
                   uint32_t step, float* action_out, float* log_std_out, void* stream);
/* QMIX mixing tail (mixing_network.py:96-116) after the hypernetwork GEMMs, per env b:
 *  hidden_e = elu(b1[b,e] + sum_a q[b,a] |w1[b, a E + e]|), q_tot[b] = sum_e hidden_e |w2[b,e]| + b2[b]
 * (row strides *_ld in floats, so the outputs of one concatenated GEMM can be passed directly). */
int lbsim_qmix_tail(const float* q, const float* w1, int64_t w1_ld, const float* b1,
                    int64_t b1_ld, const float* w2, int64_t w2_ld, const float* b2, int64_t b2_ld,
                    int64_t B, int A, int E, float* q_tot, void* stream);

/* ---- one-kernel policy inference (marllb_amd/csrc/lbsim_fused.h) ----
 * The whole network of a tile of envs per workgroup on v_mfma_f32_16x16x4_f32, activations in LDS,
 * one launch per step.  Weights are device pointers packed once by marllb_amd/policies.py
 * `pack_linear`: a Linear weight W [N, K] zero-padded to [16 ceil(N/16), 16 ceil(K/16)] and stored
 * in MFMA-fragment order P[nt][kb][lane 0..63][4] = W[16 nt + (lane & 15)][16 kb + 4 (lane >> 4)
 * + s]; biases zero-padded to the padded N.  Layer widths other than the reference defaults return
 * LBSIM_ENOTSUP (callers then use the GEMM + epilogue entry points above). */
typedef struct lbsim_sac_actor { /* problem-04 PolicyNetwork (networks.py:19-146)             */
  int32_t state_dim;             /* S * 11, <= 512                                            */
  int32_t gru_dim;               /* 128 (networks.py default)                                 */
  int32_t hidden_dim;            /* 256                                                       */
  int32_t action_dim;            /* A <= 16                                                   */
  const float* w_ih;             /* gru.weight_ih_l0 [3 gru, state_dim] packed (gates r, z, n) */
  const float* w_hh;             /* gru.weight_hh_l0 [3 gru, gru] packed                      */
  const float* b_ih;             /* [3 gru]                                                   */
  const float* b_hh;             /* [3 gru]                                                   */
  const float* w1;               /* fc1 [hidden, gru] packed                                  */
  const float* b1;               /* [hidden]                                                  */
  const float* wh;               /* [fc_mean; fc_logstd] [2 A, hidden] packed                 */
  const float* bh;               /* [2 A], zero-padded to a multiple of 16                    */
  float log_std_min, log_std_max; /* clamp (networks.py:93)                                   */
  float action_scale, action_bias;
  const uint32_t* step_dev;      /* NULL, or a device u32 read as the Philox `step` counter      */
                                 /* instead of the argument (hipGraph replays: the caller        */
                                 /* advances it in the graph)                                     */
} lbsim_sac_actor_t;
size_t lbsim_sac_actor_size(void);

/* PolicyNetwork.sample (networks.py:113-146) of B envs in one launch: state [B, state_dim];
 * hidden [B, gru] updated IN PLACE, rows whose reset_mask byte is set starting from zeros
 * (init_hidden at an episode start; reset_mask may be NULL); action_out [B, A] = tanh(x) * scale +
 * bias, x = mean (deterministic) or mean + exp(clamped log_std) eps with eps ~ N(0,1) drawn from
 * Philox exactly as lbsim_sac_head; log_std_out [B, A] optional. */
int lbsim_sac_actor_step(const lbsim_sac_actor_t* net, const float* state, float* hidden,
                         const uint8_t* reset_mask, int64_t B, int deterministic, uint64_t seed,
                         uint32_t step, float* action_out, float* log_std_out, void* stream);

typedef struct lbsim_qmix_policy { /* problem-05 QMIXAgent agents + QMixingNetwork            */
  int32_t num_agents;            /* A <= 16                                                   */
  int32_t obs_dim;               /* per-agent observation (128 at 4 x 4), <= 512              */
  int32_t gru_dim;               /* 64 (agent_network.py default)                             */
  int32_t hidden_dim;            /* 128                                                       */
  int32_t n_actions;             /* <= 16                                                     */
  int32_t state_dim;             /* global state (74 at 4 x 4), <= 512                        */
  int32_t mixing_embed_dim;      /* E = 32 (mixing_network.py default)                        */
  int32_t hypernet_embed_dim;    /* 64                                                        */
  int32_t servers_per_agent;     /* k: server_actions_out repeats each agent's action k times */
  float epsilon;                 /* exploration rate (qmix_agent.py:153)                      */
  /* agent networks, A copies stacked agent-major (packed / padded as above) */
  const float *w_ih, *w_hh, *b_ih, *b_hh; /* GRU [3 gru, obs_dim], [3 gru, gru]; [3 gru]      */
  const float *w1, *b1, *w2, *b2;         /* fc1 [hidden, gru], fc2 [hidden, hidden]           */
  const float *w3, *b3;                   /* fc3 [n_actions padded to 16, hidden]; [16]        */
  /* mixer: m0 = the first layers stacked [hyper_w1[0]; hyper_w2[0]; hyper_b2[0]; hyper_b1[0]]
   * [3 he + E, state_dim]; then hyper_w1[2] [A E, he], hyper_w2[2] [E, he], hyper_b2[2] [1, he]
   * (rows padded to 16) with their biases */
  const float *m0, *mb0, *mw1, *mbw1, *mw2, *mbw2, *mb2, *mbb2;
  const uint32_t* step_dev;      /* as lbsim_sac_actor_t.step_dev                              */
} lbsim_qmix_policy_t;
size_t lbsim_qmix_policy_size(void);

/* QMIXAgent.select_actions (qmix_agent.py:138-178) for every agent + QMixingNetwork.forward
 * (mixing_network.py:78-117) of B envs in one launch: obs [B, A, obs_dim]; hidden [B, A, gru]
 * updated in place (reset_mask as above); state [B, state_dim]; per agent the greedy action
 * (first maximum, as torch.argmax) or, with probability epsilon, a uniform one, drawn from Philox
 * (key = seed, counter = (env, step, agent, 4 << 24)); actions_out [B, A] int64,
 * server_actions_out [B, A k] int32 or NULL, q_out [B, A, n_actions] or NULL, q_chosen_out
 * [B, A] or NULL, q_tot_out [B] = the mixer on the chosen Q-values. */
int lbsim_qmix_policy_step(const lbsim_qmix_policy_t* net, const float* obs, float* hidden,
                           const uint8_t* reset_mask, const float* state, int64_t B,
                           uint64_t seed, uint32_t step, int64_t* actions_out,
                           int32_t* server_actions_out, float* q_out, float* q_chosen_out,
                           float* q_tot_out, void* stream);

/* Arrival trace for arrival_source == TRACE (the TRACE counterpart of the Poisson draw in
 * env.py's simulation; rows of replay_fork_io.py:95-121's `time<TAB>query` CSV): gap_us[rows]
 * (us since the previous row; row 0: the wrap-around gap) and work[rows] (service demand in mean-1
 * units, row N / mean N), device pointers, copied into the handle.  Env gid in episode e replays
 * rows (gid * 7919 + (e - 1) * 1000003 + k) mod rows for its k-th arrival.  Must precede the
 * first lbsim_reset of a TRACE handle; setting it again takes effect at the next reset. */
int lbsim_set_trace(lbsim_t* h, const uint32_t* gap_us, const float* work, int64_t rows,
                    void* stream);

int lbsim_alias_tables(const float* weights, int64_t n, int S, float* odd_out, int32_t* alias_out,
                       int32_t* active_out, void* stream);

/* Stateless: n Vose alias tables of S weights each (device pointers), the O(n) build of
 * problem-07's realtime VPP plugin (realtime-mode/problem-07-realtime-deployment/vpp-plugin/
 * alias_table.h:82-158, alias_table_build, rebuilt by lb_rl_node.c:92-111 from the weights the
 * controller writes): weights[n, S] f32 -> prob_out[n, S] f32, alias_out[n, S] u32, in the
 * float32 arithmetic of the C (a row summing to <= 0 gets the identity table). */
int lbsim_vose_tables(const float* weights, int64_t n, int S, float* prob_out,
                      uint32_t* alias_out, void* stream);

/* Stateless: k draws of alias_table_sample (alias_table.h:195-209, the per-packet pick of
 * lb_rl_node.c:246-288) from each of n tables (prob[n, S], alias[n, S] as lbsim_vose_tables
 * writes them) with the table's xorshift32 state (alias_table.h:163-172; state_io[n] u32, the
 * C's random_state, advanced in place).  idx_out[n, k] i32 (may be NULL) gets the picks;
 * hist_out[n, S] u64 (may be NULL) the per-server counts of this call
 * (alias_table_test_distribution, :221-237).  k <= INT32_MAX. */
int lbsim_vose_sample(const float* prob, const uint32_t* alias, int64_t n, int S,
                      uint32_t* state_io, int64_t k, int32_t* idx_out, uint64_t* hist_out,
                      void* stream);

/* ---- the VPP LB plugin's shared-memory view (src/vpp/lb/shm.h:14-91, marllb_amd/vpp_shm.py) ----
 * lbsim_vpp_export: envs [env_begin, env_begin + n_envs) of the handle as the data plane's raw
 * per-AS reservoirs (reservoir_as_t, shm.h:35-37; written by lbhash.h:116-135):
 *   tv_out [n_envs, S, 2, 128, 2] f32 = per server {fct[128], flow_duration[128]} of (t, v)
 *   pairs, t = the sample's completion time and v = the sample, both in seconds (slots past
 *   min(count, 128) are (0, 0), VPP's zeroed shm); n_flow_on_out [n_envs, S] i32 (as_stat_t
 *   n_flow_on, may be NULL); ts_out [n_envs] f32 frame time = simulated seconds since reset
 *   (msg_out_t ts, may be NULL).
 * lbsim_vpp_features: Shm_Manager.process_reservoir (src/lb/shm_proxy.py:518-543) of n raw
 *   reservoirs tv[n, 128, 2] (t, v) f32, reservoir r at frame time ts[r / res_per_ts] ->
 *   feats_out[n, 5] f64 {avg, 90, std, avg_decay, 90_decay} over all 128 bins, the decayed value
 *   v * decay^(ts - t) (numpy order; everything but the f64 pow bit-identical). */
int lbsim_vpp_export(lbsim_t* h, int64_t env_begin, int64_t n_envs, float* tv_out,
                     int32_t* n_flow_on_out, float* ts_out, void* stream);
int lbsim_vpp_features(const float* tv, const float* ts, int64_t res_per_ts, int64_t n,
                       double decay, double* feats_out, void* stream);

/*
 * Kernel timing: between lbsim_profile_begin and lbsim_profile_end every kernel launch of this
 * handle is bracketed by hipEvents recorded on the launch stream (at most max_launches launches
 * are timed; inside lbsim_step the event that closes the dynamics launch also opens the observe
 * launch, so a step records three events, not four).  lbsim_profile_end synchronises, and returns per kernel class
 * {0: dynamics step, 1: observe step, 2: dynamics reset, 3: observe reset} the summed event time
 * in ms (ms_out[4]) and the number of timed launches (count_out[4]).  lbsim_profile_end_ex
 * returns the first n_classes (<= LBSIM_PROFILE_CLASSES) classes, class 4 being the fused step
 * kernel.  Used by bench.py.  The events are created with hipEventDisableSystemFence (no cache
 * writeback / invalidate between the bracketed launches; LBSIM_PROFILE_FENCE=1 restores default
 * events): read the times only after synchronising the device, as lbsim_profile_end's callers do.
 */
#define LBSIM_PROFILE_CLASSES 5
/* (lbsim_profile_end reports the first 4 classes only: a handle whose steps are one launch --
 * step_wave_kernel under AUTO, or FUSED -- times them in class 4, so its callers need
 * lbsim_profile_end_ex(..., 5).) */
int lbsim_profile_begin(lbsim_t* h, int max_launches);
int lbsim_profile_end(lbsim_t* h, double* ms_out, int64_t* count_out);
int lbsim_profile_end_ex(lbsim_t* h, double* ms_out, int64_t* count_out, int n_classes);

/* The kernels the last lbsim_step_ex (which = 0) or lbsim_reset_ex (which = 1) of this handle
 * launched, in launch order, as "class=name;class=name" (class as in the profiler above; name the
 * kernel's template signature as rocprofv3 reports it, e.g. "0=dynamics_group_kernel<4, 0, 0,
 * false, 1>;1=observe_kernel<4, 0, false>").  bench.py keys its committed PMC counter files by
 * these names.  LBSIM_ESHAPE if buf_len is too short.  Measurement labels; no reference
 * counterpart. */
int lbsim_launch_names(lbsim_t* h, int which, char* buf, size_t buf_len);

/* Snapshot: total bytes of the device state, and copies to/from a HOST buffer of that size.
 * Layout: DESIGN.md §4 (used by the parity tests to compare every state word with oracle/).  A
 * handle whose duration samples can differ from its fct samples (duration_mode SERVICE, or
 * lost_fin_prob > 0) keeps a duration plane and has a larger snapshot: lbsim_set_state rejects a
 * snapshot of the other record format by its size (LBSIM_ESHAPE). */
int lbsim_state_size(const lbsim_t* h, size_t* bytes_out);
int lbsim_get_state(lbsim_t* h, void* host_buf, size_t bytes);
int lbsim_set_state(lbsim_t* h, const void* host_buf, size_t bytes);

#ifdef __cplusplus
}
#endif
#endif /* LBSIM_H */
