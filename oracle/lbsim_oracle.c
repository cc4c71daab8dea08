/*
 * lbsim_oracle.c — CPU ORACLE for the lbsim GPU path.  TEST INFRASTRUCTURE ONLY.
 *
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load this library, and
 * only as the checker / the timed CPU baseline.  The product path (marllb_amd/, liblbsim.so)
 * never links, loads or calls it.
 *
 * What it restates (one env at a time, scalar C99, no wave-level tricks):
 *   - ReservoirSampler.add (Algorithm R)              reservoir.py:50-85, reservoir.h:118-143
 *   - ReservoirSampler.get_features (numpy 2 f32)     reservoir.py:105-196
 *   - MultiMetricReservoir shared replacement stream  reservoir.py:236-265
 *   - PerServerFeatures.get_state_vector (S, 11)      features.py:256-286
 *   - RewardFunction.compute + 9 metrics (float64)    rewards.py:21-381
 *   - active-server rule any(obs[s] > 0)              env.py:410-413
 *   - _action_to_weights                              env.py:334-353
 *   - _normalize_observation (float64)                env.py:450-470
 *   - step/reset bookkeeping (done, return)           env.py:186-286
 *   - SED/SED2/LSQ/LSQ2 server choice                 src/vpp/lb/node.c:388-441
 *   - completion samples fct / duration               src/vpp/lb/lbhash.h:116-135 (duration
 *     = the flow's age at its last data packet, :129-136)
 *   - lost-FIN flows' timed-out fct guess             src/vpp/lb/lbhash.h:175-217, stats.h:27
 *   - server failure / recovery (Bernoulli per step)  problem-03 THEORY.md §6.4 (:687-693)
 * plus the flow dynamics the reference does not have (Poisson arrivals, per-server
 * FIFO service, Philox4x32-10 counter RNG).  Those are "parity unpinned" against the reference:
 * this file is their executable specification.
 *
 * Pinning: tests/test_oracle_golden.py checks the features, rewards and plumbing against golden
 * vectors produced by the reference Python itself (tests/golden/gen_golden.py), and Philox against
 * the Random123 known-answer vectors.
 *
 * Build: oracle/Makefile (gcc -O2 -ffp-contract=off -fopenmp).  -ffp-contract=off is required:
 * the GPU kernels are compiled the same way and integer state must match bit for bit.
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

#include "../include/lbsim.h"

#define K LBSIM_RESERVOIR_K
#define NF LBSIM_NUM_FEATURES
#define LAST_NONE (-(1 << 30))

/* ------------------------------------------------------------------ Philox4x32-10 */
void oracle_philox(const uint32_t ctr[4], const uint32_t key[2], uint32_t out[4]) {
  uint32_t c0 = ctr[0], c1 = ctr[1], c2 = ctr[2], c3 = ctr[3];
  uint32_t k0 = key[0], k1 = key[1];
  for (int r = 0; r < 10; ++r) {
    const uint64_t p0 = (uint64_t)0xD2511F53u * c0;
    const uint64_t p1 = (uint64_t)0xCD9E8D57u * c2;
    const uint32_t n0 = (uint32_t)(p1 >> 32) ^ c1 ^ k0;
    const uint32_t n1 = (uint32_t)p1;
    const uint32_t n2 = (uint32_t)(p0 >> 32) ^ c3 ^ k1;
    const uint32_t n3 = (uint32_t)p0;
    c0 = n0; c1 = n1; c2 = n2; c3 = n3;
    k0 += 0x9E3779B9u;
    k1 += 0xBB67AE85u;
  }
  out[0] = c0; out[1] = c1; out[2] = c2; out[3] = c3;
}

static float bits_f(uint32_t u) { float f; memcpy(&f, &u, 4); return f; }
static uint32_t f_bits(float f) { uint32_t u; memcpy(&u, &f, 4); return u; }

static float u01(uint32_t r) { return (float)((r >> 8) + 1u) * 5.9604644775390625e-8f; }

/* ln x for x in [2^-24, 1] — DESIGN.md §3.2 (same operation sequence as the GPU: Cephes logf
 * polynomial for log1p(m - 1), fmaf Horner, no division). */
float oracle_logf(float x) {
  const uint32_t b = f_bits(x);
  int e = (int)(b >> 23) - 127;
  float m = bits_f((b & 0x007fffffu) | 0x3f800000u);
  if (m > 1.41421354f) { m = m * 0.5f; e = e + 1; }
  const float f = m - 1.0f;  /* exact */
  const float z = f * f;
  float p = 7.0376836292e-2f;
  p = fmaf(p, f, -1.1514610310e-1f);
  p = fmaf(p, f, 1.1676998740e-1f);
  p = fmaf(p, f, -1.2420140846e-1f);
  p = fmaf(p, f, 1.4249322787e-1f);
  p = fmaf(p, f, -1.6668057665e-1f);
  p = fmaf(p, f, 2.0000714765e-1f);
  p = fmaf(p, f, -2.4999993993e-1f);
  p = fmaf(p, f, 3.3333331174e-1f);
  float y = (p * f) * z;
  y = fmaf(-0.5f, z, y);
  const float fe = (float)e;  /* ln 2 = 0.693359375 - 2.12194440e-4 (Cephes split) */
  float r = fmaf(fe, -2.12194440e-4f, y);
  r = r + f;
  return fmaf(fe, 0.693359375f, r);
}

/* 2^x for x <= 0 — DESIGN.md §3.4. */
float oracle_exp2f(float x) {
  if (x < -60.0f) return 0.0f;
  const float fl = floorf(x + 0.5f);  /* exact for |x| <= 60 */
  const int n = (int)fl;
  const float f = x - fl;             /* exact, in [-0.5, 0.5) */
  float p = 1.52527336e-5f;
  p = fmaf(p, f, 1.54035297e-4f);
  p = fmaf(p, f, 1.33335581e-3f);
  p = fmaf(p, f, 9.61812911e-3f);
  p = fmaf(p, f, 5.55041086e-2f);
  p = fmaf(p, f, 0.240226507f);
  p = fmaf(p, f, 0.693147182f);
  p = fmaf(p, f, 1.0f);
  return p * bits_f((uint32_t)(n + 127) << 23);
}

/* ------------------------------------------------------------------ numpy pairwise sums */
/* numpy/_core/src/umath/loops_utils.h.src pairwise_sum, n <= 128 (PW_BLOCKSIZE). */
static float pw32(const float* a, int n) {
  if (n < 8) {
    float r = 0.0f;
    for (int i = 0; i < n; ++i) r += a[i];
    return r;
  }
  float r[8];
  for (int j = 0; j < 8; ++j) r[j] = a[j];
  const int m8 = n - (n % 8);
  for (int i = 8; i < m8; i += 8)
    for (int j = 0; j < 8; ++j) r[j] += a[i + j];
  float res = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]));
  for (int i = m8; i < n; ++i) res += a[i];
  return res;
}

static double pw64(const double* a, int n) {
  if (n < 8) {
    double r = 0.0;
    for (int i = 0; i < n; ++i) r += a[i];
    return r;
  }
  double r[8];
  for (int j = 0; j < 8; ++j) r[j] = a[j];
  const int m8 = n - (n % 8);
  for (int i = 8; i < m8; i += 8)
    for (int j = 0; j < 8; ++j) r[j] += a[i + j];
  double res = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]));
  for (int i = m8; i < n; ++i) res += a[i];
  return res;
}

/* ------------------------------------------------------------------ reservoir features */
typedef struct { float v; int slot; } vs_t;
static int cmp_vs(const void* a, const void* b) {
  const vs_t* x = (const vs_t*)a;
  const vs_t* y = (const vs_t*)b;
  if (x->v < y->v) return -1;
  if (x->v > y->v) return 1;
  return (x->slot > y->slot) - (x->slot < y->slot);
}

/* get_features(decay, now) of one reservoir; w[]/wq[] are the slot weights (see below). */
static void features_one(const float* vals, const float* w, const uint64_t* wq, int n,
                         float out[5]) {
  if (n == 0) { for (int f = 0; f < 5; ++f) out[f] = 0.0f; return; }
  /* mean, std: numpy float32 pairwise (np.mean / np.std ddof 0) */
  const float fn = (float)n;
  const float mean = pw32(vals, n) / fn;
  float d2[K];
  for (int i = 0; i < n; ++i) { const float d = vals[i] - mean; d2[i] = d * d; }
  const float sd = sqrtf(pw32(d2, n) / fn);
  /* mean_decay = np.average(values, weights=w) in float64 */
  double vw[K], ww[K];
  for (int i = 0; i < n; ++i) { ww[i] = (double)w[i]; vw[i] = (double)vals[i] * (double)w[i]; }
  const float md = (float)(pw64(vw, n) / pw64(ww, n));
  /* sorted order by (value, slot) */
  vs_t srt[K];
  for (int i = 0; i < n; ++i) { srt[i].v = vals[i]; srt[i].slot = i; }
  qsort(srt, (size_t)n, sizeof(vs_t), cmp_vs);
  /* p90: numpy 2 'linear' with float32 q = 90 / float32(100) (virtual index (n-1)*q) */
  const float q = 0.9f;
  const float h = (float)(n - 1) * q;
  const float fl = floorf(h);
  const int lo = (int)fl;
  const float g = h - fl;
  const float a = srt[lo].v;
  const float b = srt[lo + 1 < n ? lo + 1 : lo].v;
  const float diff = b - a;
  const float p90 = (g >= 0.5f) ? (b - diff * (1.0f - g)) : (a + diff * g);
  /* p90_decay: first sorted index with cumsum >= 0.9 * total (searchsorted 'left'), with the
   * weights in exact 2^-48 fixed point so the comparison does not depend on summation order. */
  uint64_t total = 0;
  for (int i = 0; i < n; ++i) total += wq[i];
  uint64_t cum = 0;
  int idx = n - 1;
  for (int i = 0; i < n; ++i) {
    cum += wq[srt[i].slot];
    if (cum * 10u >= total * 9u) { idx = i; break; }
  }
  out[0] = mean; out[1] = p90; out[2] = sd; out[3] = md; out[4] = srt[idx].v;
}

/* Decay weights relative to the newest sample: w = 2^(log2(decay)/1000 * age_ms). */
static void slot_weights(const uint32_t* ts, int n, float decay_c, float* w, uint64_t* wq) {
  uint32_t newest = 0;
  for (int i = 0; i < n; ++i) newest = ts[i] > newest ? ts[i] : newest;
  for (int i = 0; i < n; ++i) {
    w[i] = oracle_exp2f((float)(newest - ts[i]) * decay_c);
    wq[i] = (uint64_t)(w[i] * 281474976710656.0f);
  }
}

float oracle_decay_c(float decay_factor) {
  return (float)(log2((double)decay_factor) / 1000.0);
}

void oracle_reservoir_features(const float* values, const uint32_t* ts_ms, uint32_t count,
                               float decay_factor, float out[5]) {
  const int n = count < (uint32_t)K ? (int)count : K;
  float w[K];
  uint64_t wq[K];
  slot_weights(ts_ms, n, oracle_decay_c(decay_factor), w, wq);
  features_one(values, w, wq, n, out);
}

/* ------------------------------------------------------------------ reward (float64) */
static double np_var(const double* x, int n) {
  const double mean = pw64(x, n) / (double)n;
  double d[LBSIM_MAX_SERVERS];
  for (int i = 0; i < n; ++i) { const double t = x[i] - mean; d[i] = t * t; }
  return pw64(d, n) / (double)n;
}

double oracle_reward(const float* obs, int S, int metric, int field) {
  if (field < 0 || field >= NF) return 0.0;
  double x[LBSIM_MAX_SERVERS];
  int n = 0;
  for (int s = 0; s < S; ++s) {
    int active = 0;
    for (int f = 0; f < NF; ++f) active |= obs[s * NF + f] > 0.0f;
    if (active) x[n++] = (double)obs[s * NF + field];
  }
  if (n == 0) return 0.0;
  const double eps = 1e-10;
  switch (metric) {
    case LBSIM_METRIC_JAIN: {
      const double sv = pw64(x, n);
      if (sv < eps) return 1.0;
      double x2[LBSIM_MAX_SERVERS];
      for (int i = 0; i < n; ++i) x2[i] = x[i] * x[i];
      const double sq = pw64(x2, n);
      if (sq < eps) return 1.0;
      const double j = (sv * sv) / ((double)n * sq);
      const double lo = 1.0 / (double)n;
      return j < lo ? lo : (j > 1.0 ? 1.0 : j);
    }
    case LBSIM_METRIC_VARIANCE: return -np_var(x, n);
    case LBSIM_METRIC_STD: return -sqrt(np_var(x, n));
    case LBSIM_METRIC_CV: {
      const double mean = pw64(x, n) / (double)n;
      if (mean < eps) return 0.0;
      return -(sqrt(np_var(x, n)) / (mean + eps));
    }
    case LBSIM_METRIC_MAX: {
      double m = x[0];
      for (int i = 1; i < n; ++i) m = x[i] > m ? x[i] : m;
      return -m;
    }
    case LBSIM_METRIC_MIN: {
      double m = x[0];
      for (int i = 1; i < n; ++i) m = x[i] < m ? x[i] : m;
      return m;
    }
    case LBSIM_METRIC_PRODUCT: {
      double l[LBSIM_MAX_SERVERS];
      for (int i = 0; i < n; ++i) l[i] = log(x[i] + eps);
      return pw64(l, n);
    }
    case LBSIM_METRIC_RANGE: {
      double mx = x[0], mn = x[0];
      for (int i = 1; i < n; ++i) { if (x[i] > mx) mx = x[i]; if (x[i] < mn) mn = x[i]; }
      return -(mx - mn);
    }
    case LBSIM_METRIC_GINI: {
      const double mean = pw64(x, n) / (double)n;
      if (mean == 0.0) return 0.0;
      double ds = 0.0;
      for (int i = 0; i < n; ++i)
        for (int k = 0; k < n; ++k) ds += fabs(x[i] - x[k]);
      return -(ds / ((double)(2 * n * n) * mean));
    }
    default: return 0.0;
  }
}

/* ------------------------------------------------------------------ simulator state */
typedef struct oracle {
  lbsim_config_t cfg;
  int B, S, Q;
  int32_t dt_us;
  float mean_gap_us, svc_scale[LBSIM_MAX_SERVERS], decay_c;
  /* lost-FIN flows: 24-bit probability threshold (0 = off), flow_timeout - 40 s in us, the mean
   * bucket wait in us; server failures: 24-bit thresholds (fail 0 = off, no `down` section) */
  uint32_t lf_thr;
  int32_t lf_off_us;
  float lf_wait_us;
  uint32_t fail_thr, rec_thr;
  int big_in_step; /* an in-step record can hold a sample >= PACK_LIMIT (dt >= it, or lost-FIN) */
  uint32_t key[2];
  int threads;
  int initialised;
  char* buf;
  size_t bytes;
  /* sections, snapshot order == liblbsim */
  int32_t* next_arr; float* next_work; uint32_t* next_u2; uint32_t* next_u3; uint32_t* arr_idx;
  uint32_t* episode; uint32_t* clock; int32_t* ep_step; uint32_t* dropped; int32_t* norm_count;
  double* ep_return;
  uint32_t* hc; int32_t* last_tc; uint32_t* res_count;
  int32_t* ring; /* [B*S*Q][2] = {t_complete, t_arrival} */
  /* reservoir slot records [B*S*K][2] = {fct us, timestamp ms}; the feature value of a sample is
   * (float)us * 1e-6f.  dur [B*S*K]: the duration us of each slot, only when a duration sample can
   * differ from its fct (duration_mode SERVICE, lost-FIN guesses): else NULL, and the duration
   * reservoir IS the fct reservoir */
  uint32_t* res;
  uint32_t* dur;
  /* unchanged-reservoir skip of observe: slots written by the last dynamics
   * launch (a 128-bit mask per server) and the server's 10 reservoir features at the last
   * observe */
  uint32_t* chg; float* fcache;
  double* norm_mean; double* norm_std;
  /* server failures (only if fail_prob > 0): 1 = the server is down, per (env, server) */
  uint32_t* down;
  /* n_flow_on_mode VPP with lost-FIN (leak): lost-FIN flows completed per (env, server) since the
   * episode start / the server's last failure, never decremented (lbhash.h:193,214) */
  int leak;
  uint32_t* lost_on;
  int dur_plane; /* the `dur` section exists */
  /* lost-FIN deferral (split: lf_thr != 0): the fct and duration reservoirs are
   * separate -- dur is then [B*S*K][2] {duration us, timestamp ms} with its own count
   * res_count_dur -- and each server holds its pending timed-out fct guesses in a ring of P
   * entries {due us mod 2^32 (absolute: clock * dt + t), guess us} sorted by due time, pend_hc =
   * head | count << 16; lf_over counts the guesses dropped at a full ring (per env, this episode) */
  int split, P;
  uint32_t* res_count_dur;
  uint32_t* pend_hc;
  uint32_t* pend;
  uint32_t* lf_over;
  /* reservoir_mode VPP: every sample overwrites slot rand() % 128 (lbhash.h:108,179), bins zeroed
   * at reset / failure */
  int res_vpp;
  /* TRACE arrivals (lbsim_set_trace semantics): us gap before each row, mean-1 work */
  uint32_t* trace_gap; float* trace_work; uint32_t trace_rows;
  /* not state: the Algorithm R draw word of each queued flow that arrived in the current step,
   * [B*S*Q] by ring position (written at the push, read at the pop in the same step) */
  uint32_t* flow_r;
} oracle_t;

static void derive(oracle_t* o) {
  const lbsim_config_t* c = &o->cfg;
  o->B = c->num_envs; o->S = c->num_servers; o->Q = c->queue_capacity;
  o->dt_us = (int32_t)llround((double)c->step_interval * 1e6);
  o->mean_gap_us = (float)(1e6 / (double)c->arrival_rate);
  for (int s = 0; s < LBSIM_MAX_SERVERS; ++s)
    o->svc_scale[s] = s < c->num_servers ? (float)(1e6 / (double)c->server_rate[s]) : 0.0f;
  o->decay_c = oracle_decay_c(c->decay_factor);
  o->lf_thr = (uint32_t)llround((double)c->lost_fin_prob * 16777216.0);
  o->lf_off_us = (int32_t)(llround((double)c->flow_timeout_s * 1e6) - 40000000LL);
  o->lf_wait_us = c->lost_fin_prob > 0.0f
                      ? (float)((double)c->flow_buckets * 1e6 / (double)c->arrival_rate) : 0.0f;
  o->fail_thr = (uint32_t)llround((double)c->fail_prob * 16777216.0);
  o->rec_thr = (uint32_t)llround((double)c->recover_prob * 16777216.0);
  o->big_in_step = (o->dt_us >= (int32_t)((1u << 25) - 1u)) || o->lf_thr != 0u;
  o->leak = c->n_flow_on_mode == LBSIM_NFLOW_VPP && o->lf_thr != 0u;
  o->dur_plane = c->duration_mode == LBSIM_DURATION_SERVICE || o->lf_thr != 0u;
  o->split = o->lf_thr != 0u;
  o->P = o->split ? c->lost_fin_pending : 0;
  o->res_vpp = c->reservoir_mode == LBSIM_RESERVOIR_VPP;
  o->key[0] = (uint32_t)(c->seed & 0xFFFFFFFFull);
  o->key[1] = (uint32_t)(c->seed >> 32);
}

oracle_t* oracle_create(const lbsim_config_t* cfg) {
  oracle_t* o = (oracle_t*)calloc(1, sizeof(oracle_t));
  if (!o) return NULL;
  o->cfg = *cfg;
  derive(o);
  o->threads = 1;
  const size_t B = o->B, BS = (size_t)o->B * o->S, BSQ = BS * o->Q, BSK = BS * K;
  const size_t sz[] = {B * 4, B * 4, B * 4, B * 4, B * 4, B * 4, B * 4, B * 4, B * 4, B * 4,
                       B * 8, BS * 4, BS * 4, BS * 4, BSQ * 8, BSK * 8, BS * 16, BS * 40,
                       cfg->normalize_obs ? BS * NF * 8 : 0, cfg->normalize_obs ? BS * NF * 8 : 0,
                       cfg->fail_prob > 0.0f ? BS * 4 : 0, o->leak ? BS * 4 : 0,
                       o->dur_plane ? BSK * (o->split ? 8 : 4) : 0, o->split ? BS * 4 : 0,
                       o->split ? BS * 4 : 0, o->split ? BS * (size_t)o->P * 8 : 0,
                       o->split ? B * 4 : 0};
  size_t total = 0;
  for (size_t i = 0; i < sizeof(sz) / sizeof(sz[0]); ++i) total += sz[i];
  o->bytes = total;
  o->buf = (char*)calloc(1, total ? total : 1);
  if (!o->buf) { free(o); return NULL; }
  char* p = o->buf;
  void** ptrs[] = {(void**)&o->next_arr, (void**)&o->next_work, (void**)&o->next_u2,
                   (void**)&o->next_u3, (void**)&o->arr_idx, (void**)&o->episode,
                   (void**)&o->clock, (void**)&o->ep_step, (void**)&o->dropped,
                   (void**)&o->norm_count, (void**)&o->ep_return, (void**)&o->hc,
                   (void**)&o->last_tc, (void**)&o->res_count, (void**)&o->ring,
                   (void**)&o->res, (void**)&o->chg, (void**)&o->fcache, (void**)&o->norm_mean,
                   (void**)&o->norm_std, (void**)&o->down, (void**)&o->lost_on, (void**)&o->dur,
                   (void**)&o->res_count_dur, (void**)&o->pend_hc, (void**)&o->pend,
                   (void**)&o->lf_over};
  for (size_t i = 0; i < sizeof(sz) / sizeof(sz[0]); ++i) {
    *ptrs[i] = sz[i] ? (void*)p : NULL;
    p += sz[i];
  }
  if (cfg->normalize_obs)
    for (size_t i = 0; i < BS * NF; ++i) o->norm_std[i] = 1.0; /* env.py:153 */
  o->flow_r = (uint32_t*)calloc(BSQ ? BSQ : 1, 4);
  if (!o->flow_r) { free(o->buf); free(o); return NULL; }
  return o;
}

void oracle_destroy(oracle_t* o) {
  if (!o) return;
  free(o->trace_gap);
  free(o->trace_work);
  free(o->flow_r);
  free(o->buf);
  free(o);
}

/* The trace replayed when cfg.arrival_source == TRACE (host copies). */
int oracle_set_trace(oracle_t* o, const uint32_t* gap_us, const float* work, long rows) {
  if (rows < 1) return -1;
  free(o->trace_gap);
  free(o->trace_work);
  o->trace_gap = (uint32_t*)malloc((size_t)rows * 4);
  o->trace_work = (float*)malloc((size_t)rows * 4);
  memcpy(o->trace_gap, gap_us, (size_t)rows * 4);
  memcpy(o->trace_work, work, (size_t)rows * 4);
  o->trace_rows = (uint32_t)rows;
  return 0;
}

void oracle_set_threads(oracle_t* o, int n) { o->threads = n < 1 ? 1 : n; }
size_t oracle_state_size(const oracle_t* o) { return o->bytes; }
void oracle_get_state(const oracle_t* o, void* dst) { memcpy(dst, o->buf, o->bytes); }
void oracle_set_state(oracle_t* o, const void* src) { memcpy(o->buf, src, o->bytes); o->initialised = 1; }

void oracle_seed(oracle_t* o, uint64_t seed) {
  o->cfg.seed = seed;
  o->key[0] = (uint32_t)(seed & 0xFFFFFFFFull);
  o->key[1] = (uint32_t)(seed >> 32);
  memset(o->episode, 0, (size_t)o->B * 4);
}

/* ------------------------------------------------------------------ one env, scalar */
typedef struct {
  oracle_t* o;
  size_t b;
  uint32_t gid;
  int assigned[LBSIM_MAX_SERVERS];
} env_ctx;

static float score_of(int policy, int32_t cnt, double den) {
  if (policy == LBSIM_POLICY_LSQ || policy == LBSIM_POLICY_LSQ2) return (float)cnt;
  return (float)((double)(cnt + 1) / den);
}

/* gen_alias (src/lb/shm_proxy.py:127-146) on n weights, in float64 as the reference's Python:
 * avg = sum(w) / (n + 1e-6) (sequential sum), p_i = w_i / (avg + 1e-6); the "small" (w < avg)
 * and "big" (w >= avg) generators walk the weights in index order; a big reduced below 1 becomes
 * the next small.  Unassigned entries keep (1, 0).  odd_out in float64 (the value the reference
 * packs into shm.h alias_t as float32). */
void oracle_gen_alias(const float* w, int n, double* odd_out, int32_t* alias_out) {
  double sum = 0.0;
  for (int i = 0; i < n; ++i) sum += (double)w[i];
  const double avg = sum / ((double)n + 1e-6);
  for (int i = 0; i < n; ++i) { odd_out[i] = 1.0; alias_out[i] = 0; }
  int si = 0, bi = 0, sk = -1, bk = -1;
  double sp = 0.0, bp = 0.0;
#define NEXT_SMALL()                                                    \
  do {                                                                  \
    while (si < n && !((double)w[si] < avg)) ++si;                      \
    if (si < n) { sk = si; sp = (double)w[si] / (avg + 1e-6); ++si; }   \
    else sk = -1;                                                       \
  } while (0)
#define NEXT_BIG()                                                      \
  do {                                                                  \
    while (bi < n && !((double)w[bi] >= avg)) ++bi;                     \
    if (bi < n) { bk = bi; bp = (double)w[bi] / (avg + 1e-6); ++bi; }   \
    else bk = -1;                                                       \
  } while (0)
  NEXT_SMALL();
  NEXT_BIG();
  while (bk >= 0 && sk >= 0) {
    odd_out[sk] = sp;
    alias_out[sk] = bk;
    bp = bp - (1.0 - sp);
    if (bp < 1.0) { sk = bk; sp = bp; NEXT_BIG(); }
    else NEXT_SMALL();
  }
#undef NEXT_SMALL
#undef NEXT_BIG
}

/* Vose alias table of problem-07's VPP plugin
 * (realtime-mode/problem-07-realtime-deployment/vpp-plugin/alias_table.h:82-158), in float32 as
 * the C: sequential f32 sum (:90-93); sum <= 0 (NaN is not) -> the identity table (:95-102);
 * prob_scaled[i] = (f32)n * w[i] / sum (:106-108); small (< 1) / large stacks filled in index
 * order (:116-122) and popped from the top (:125-139); the large's remainder
 * (prob_l + prob_s) - 1.0 is an f32 sum, a double subtraction and a store to f32 (:132) -- the
 * correctly rounded f32 subtraction, since double carries more than 2 x 24 + 2 bits; leftovers
 * get (1, self) (:142-152).  n <= LBSIM_MAX_SERVERS. */
void oracle_vose_build(const float* w, int n, float* prob, uint32_t* alias) {
  float sum = 0.0f;
  for (int i = 0; i < n; ++i) sum += w[i];
  if (sum <= 0.0f) {
    for (int i = 0; i < n; ++i) { prob[i] = 1.0f; alias[i] = (uint32_t)i; }
    return;
  }
  float ps[LBSIM_MAX_SERVERS];
  uint32_t small[LBSIM_MAX_SERVERS], large[LBSIM_MAX_SERVERS];
  int ns = 0, nl = 0;
  for (int i = 0; i < n; ++i) ps[i] = (float)(uint32_t)n * w[i] / sum;
  for (int i = 0; i < n; ++i) {
    if (ps[i] < 1.0f) small[ns++] = (uint32_t)i;
    else large[nl++] = (uint32_t)i;
  }
  while (ns > 0 && nl > 0) {
    const uint32_t s = small[--ns], l = large[--nl];
    prob[s] = ps[s];
    alias[s] = l;
    ps[l] = (float)((double)(ps[l] + ps[s]) - 1.0);
    if (ps[l] < 1.0f) small[ns++] = l;
    else large[nl++] = l;
  }
  while (ns > 0) { const uint32_t s = small[--ns]; prob[s] = 1.0f; alias[s] = s; }
  while (nl > 0) { const uint32_t l = large[--nl]; prob[l] = 1.0f; alias[l] = l; }
}

/* alias_table_sample (alias_table.h:195-209) k times from the table's xorshift32 state
 * (:163-172: x ^= x << 13; x ^= x >> 17; x ^= x << 5): i = x1 % n, r = (f32)x2 / (f32)0xFFFFFFFF
 * (:178-182), the pick is i if r < prob[i] else alias[i].  idx_out[k] (may be NULL) and the
 * histogram hist[n] += picks (alias_table_test_distribution, :221-237; not zeroed here).
 * Returns the final state. */
uint32_t oracle_vose_sample(const float* prob, const uint32_t* alias, int n, uint32_t state,
                            int64_t k, int32_t* idx_out, uint64_t* hist) {
  for (int64_t j = 0; j < k; ++j) {
    uint32_t x = state;
    x ^= x << 13; x ^= x >> 17; x ^= x << 5;
    const uint32_t i = x % (uint32_t)n;
    x ^= x << 13; x ^= x >> 17; x ^= x << 5;
    state = x;
    const float r = (float)x / (float)0xFFFFFFFFu;
    const uint32_t pick = r < prob[i] ? i : alias[i];
    if (idx_out) idx_out[j] = (int32_t)pick;
    if (hist) hist[pick] += 1;
  }
  return state;
}

/* hc = ring head | HC_BIG | count << 16.  HC_BIG (sticky): a record holding a sample >= 2^25 - 1
 * us as an unsigned word (negative lost-FIN guesses included) was stored in the server's
 * reservoirs since they were last emptied (reset, failure) -- the GPU observe's test for its
 * one-pass key sort; part of the state, so restated here. */
#define HC_BIG 0x8000u
#define PACK_LIMIT ((1u << 25) - 1u)
static int ring_head(const oracle_t* o, size_t sb) { return (int)(o->hc[sb] & (HC_BIG - 1u)); }
static int ring_count(const oracle_t* o, size_t sb) { return (int)(o->hc[sb] >> 16); }
static void ring_set(oracle_t* o, size_t sb, int head, int cnt) {
  o->hc[sb] = (o->hc[sb] & HC_BIG) | (uint32_t)head | ((uint32_t)cnt << 16);
}

/* A reservoir sample in seconds from its integer-microsecond form (env.py reports seconds). */
static float us_to_seconds(uint32_t us) { return (float)(int32_t)us * 1.0e-6f; }

/* murmur3's 32-bit finaliser (fmix32): the lost-FIN hash. */
static uint32_t lf_mix(uint32_t h) {
  h ^= h >> 16; h *= 0x85EBCA6Bu; h ^= h >> 13; h *= 0xC2B2AE35u; h ^= h >> 16;
  return h;
}

/* The fct sample of a completed flow (lbhash.h:116-124 RSTACK: now - t_init) or, for a flow whose
 * FIN/RST the data plane missed, VPP's timed-out guess (lbhash.h:175-217): its entry expires
 * flow_timeout after the last packet (the completion tc), the next flow hashed into the bucket
 * takes it after an exponential wait of mean flow_buckets / arrival_rate, and the plugin records
 * now - t_init - LB_DEFAULT_FLOW_TIMEOUT (40 s, stats.h:27) = fct + flow_timeout - 40 s + wait.
 * Lost or not, and the wait, are a hash of (seed, global env id, episode, the flow's absolute
 * arrival us mod 2^32): a pure function of the flow, whichever step records it.  Signed us, in
 * uint32 arithmetic. */
/* Lost or not (the 24-bit test), and the bucket wait in us, of the flow that arrived at abs_ta. */
static int lf_test(uint32_t abs_ta, uint32_t gid, uint32_t episode, uint32_t key0, uint32_t key1,
                   uint32_t thr, float wait_us, int32_t* wait_out) {
  if (thr == 0u) return 0;
  const uint32_t salt = lf_mix(lf_mix(key0 ^ (episode * 0x9E3779B9u)) ^ gid ^ (key1 * 0x85EBCA6Bu));
  const uint32_t h = lf_mix(abs_ta ^ salt);
  if ((h >> 8) >= thr) return 0;
  const uint32_t h2 = lf_mix(h ^ 0x6A09E667u);
  *wait_out = (int32_t)(-oracle_logf(u01(h2)) * wait_us);
  return 1;
}

/* The guess fct + off_us + wait as a signed int32 us sample, saturated (the config bound keeps
 * Poisson work in range). */
static uint32_t lf_guess(uint32_t fct, int32_t off_us, int32_t wait) {
  int64_t g = (int64_t)(int32_t)fct + (int64_t)off_us + (int64_t)wait;
  g = g > (int64_t)INT32_MAX ? (int64_t)INT32_MAX : (g < (int64_t)INT32_MIN ? (int64_t)INT32_MIN : g);
  return (uint32_t)(int32_t)g;
}

uint32_t oracle_lost_fin_fct(uint32_t fct, uint32_t abs_ta, uint32_t gid, uint32_t episode,
                             uint32_t key0, uint32_t key1, uint32_t thr, int32_t off_us,
                             float wait_us) {
  int32_t wait = 0;
  if (!lf_test(abs_ta, gid, episode, key0, key1, thr, wait_us, &wait)) return fct;
  return lf_guess(fct, off_us, wait);
}

/* Algorithm R slot for a flow that arrived in the step it completes in: the draw
 * is its arrival's word r (word 3 of the arrival's Philox block), j = floor(r (c + 1) / 2^32)
 * (reservoir.py:76 randint(0, count + 1), Lemire multiply-shift). */
long oracle_algr_slot_r32(uint32_t count, uint32_t r) {
  if (count < (uint32_t)K) return (long)count;
  const uint64_t j = ((uint64_t)r * ((uint64_t)count + 1u)) >> 32;
  return j < (uint64_t)K ? (long)j : -1;
}

/* The slot one sample takes in a reservoir holding c samples (-1: not kept).  ALGR (reservoir.py:
 * 64-85): c < K -> c, else j = randint(0, c + 1) if j < K; VPP (lbhash.h:108,179): rand() % 128,
 * always.  The draw: a flow that arrived in this step (has_r) uses its arrival's word r (the top 7
 * bits for VPP); otherwise the reservoir stream's block (c >> 1), half (c & 1), at counter word w
 * (2 << 24) | sub | s -- sub = 1 << 16 for the fct reservoir of a split handle. */
static long res_slot(env_ctx* e, int s, uint32_t c, int has_r, uint32_t r, uint32_t sub) {
  oracle_t* o = e->o;
  if (!o->res_vpp && c < (uint32_t)K) return (long)c;
  if (has_r) return o->res_vpp ? (long)(r >> 25) : oracle_algr_slot_r32(c, r);
  const uint32_t ctr[4] = {c >> 1, e->gid, o->episode[e->b], (2u << 24) | sub | (uint32_t)s};
  uint32_t d[4];
  oracle_philox(ctr, o->key, d);
  const uint32_t hi = (c & 1u) ? d[3] : d[1];
  const uint32_t lo = (c & 1u) ? d[2] : d[0];
  if (o->res_vpp) return (long)(hi >> 25);
  /* j = floor(r64 * (c + 1) / 2^64): randint(0, count + 1) (reservoir.py:76) */
  const unsigned __int128 prod = (unsigned __int128)(((uint64_t)hi << 32) | lo) * ((uint64_t)c + 1u);
  const uint64_t j = (uint64_t)(prod >> 64);
  return j < (uint64_t)K ? (long)j : -1;
}

/* Algorithm R insert of one completion into both reservoirs of server s (shared decision, paired
 * handles).  A flow that arrived in this step (has_r) uses its arrival's draw word r; a flow
 * carried in from an earlier step uses the reservoir stream's block (count >> 1), half
 * (count & 1). */
static void reservoir_add(env_ctx* e, int s, uint32_t fct, uint32_t dur, uint32_t ts_ms, int has_r,
                          uint32_t r) {
  oracle_t* o = e->o;
  const size_t sb = e->b * (size_t)o->S + (size_t)s;
  const uint32_t c = o->res_count[sb];
  const long slot = res_slot(e, s, c, has_r, r, 0u);
  if (slot >= 0) {
    const size_t r = sb * K + (size_t)slot;
    /* HC_BIG at the store for a flow carried in from an earlier step; in-step records by the
     * end-of-launch scan (big_scan) */
    if (!has_r && (fct > dur ? fct : dur) >= PACK_LIMIT) o->hc[sb] |= HC_BIG;
    o->res[2 * r + 0] = fct;
    o->res[2 * r + 1] = ts_ms;
    if (o->dur) o->dur[r] = dur;
    o->chg[sb * 4 + (size_t)(slot >> 5)] |= 1u << (slot & 31);
  }
  if (c != 0xFFFFFFFFu) o->res_count[sb] = c + 1u;
}

/* Split handles (lost-FIN): one sample into the fct reservoir (res, res_count) or the duration
 * reservoir (dur {us, ts}, res_count_dur) of server s, each with its own decision. */
static void split_add(env_ctx* e, int s, int is_dur, uint32_t v, uint32_t ts_ms, int has_r,
                      uint32_t r) {
  oracle_t* o = e->o;
  const size_t sb = e->b * (size_t)o->S + (size_t)s;
  uint32_t* cnt = is_dur ? o->res_count_dur : o->res_count;
  const uint32_t c = cnt[sb];
  /* the duration reservoir draws as the paired reservoirs of a run without losses (its samples
   * are the same: every completion's), the fct reservoir's carried / deferred draws at 1 << 16 */
  const long slot = res_slot(e, s, c, has_r, r, is_dur ? 0u : 1u << 16);
  if (slot >= 0) {
    const size_t i = sb * K + (size_t)slot;
    if (!has_r && v >= PACK_LIMIT) o->hc[sb] |= HC_BIG;
    uint32_t* rec = is_dur ? o->dur : o->res;
    rec[2 * i + 0] = v;
    rec[2 * i + 1] = ts_ms;
    o->chg[sb * 4 + (size_t)(slot >> 5)] |= 1u << (slot & 31);
  }
  if (c != 0xFFFFFFFFu) cnt[sb] = c + 1u;
}

/* A timed-out flow's guess, due (absolute us mod 2^32) at its wrap-up, into server s's pending
 * ring, sorted by due time (wrap-aware; an equal due goes after the entries already there), by an
 * insertion from the tail.  A full ring drops it (lf_over). */
static void pend_push(env_ctx* e, int s, uint32_t due, uint32_t val) {
  oracle_t* o = e->o;
  const size_t sb = e->b * (size_t)o->S + (size_t)s;
  const int P = o->P;
  const int head = (int)(o->pend_hc[sb] & 0xFFFFu), cnt = (int)(o->pend_hc[sb] >> 16);
  if (cnt == P) { o->lf_over[e->b] += 1u; return; }
  uint32_t* ring = o->pend + sb * (size_t)P * 2;
  int i = cnt;
  while (i > 0) {
    int pos = head + i - 1;
    if (pos >= P) pos -= P;
    if ((int32_t)(ring[2 * pos] - due) <= 0) break;
    int to = pos + 1 == P ? 0 : pos + 1;
    ring[2 * to] = ring[2 * pos];
    ring[2 * to + 1] = ring[2 * pos + 1];
    --i;
  }
  int pos = head + i;
  if (pos >= P) pos -= P;
  ring[2 * pos] = due;
  ring[2 * pos + 1] = val;
  o->pend_hc[sb] = (uint32_t)head | ((uint32_t)(cnt + 1) << 16);
}

/* Server s's pending guesses due by step time t (relative us) into its fct reservoir, in due
 * order, each stamped with its due time (the wrap-up of lbhash.h:182-217: the next flow of the
 * bucket records now - t_init - 40 s at its own arrival). */
static void pend_flush(env_ctx* e, int s, int32_t t, uint64_t base_us) {
  oracle_t* o = e->o;
  const size_t sb = e->b * (size_t)o->S + (size_t)s;
  const int P = o->P;
  int head = (int)(o->pend_hc[sb] & 0xFFFFu), cnt = (int)(o->pend_hc[sb] >> 16);
  const uint32_t* ring = o->pend + sb * (size_t)P * 2;
  while (cnt > 0) {
    const int32_t rel = (int32_t)(ring[2 * head] - (uint32_t)base_us);
    if (rel > t) break;
    const uint32_t ts_ms = (uint32_t)((uint64_t)((int64_t)base_us + (int64_t)rel) / 1000u);
    split_add(e, s, 0, ring[2 * head + 1], ts_ms, 0, 0u);
    head = head + 1 == P ? 0 : head + 1;
    cnt -= 1;
  }
  o->pend_hc[sb] = (uint32_t)head | ((uint32_t)cnt << 16);
}

/* End of a dynamics launch (a step, or a reset with its warm-up): when an in-step record can be
 * big, HC_BIG |= any slot the launch wrote (below the count) holding one -- the GPU's big_written. */
static void big_scan(oracle_t* o, size_t b) {
  if (!o->big_in_step) return;
  for (int s = 0; s < o->S; ++s) {
    const size_t sb = b * (size_t)o->S + (size_t)s;
    const uint32_t c = o->res_count[sb];
    const uint32_t n = c < (uint32_t)K ? c : (uint32_t)K;
    /* split handles: the duration reservoir's own count and {us, ts} records */
    const uint32_t cd = o->split ? o->res_count_dur[sb] : c;
    const uint32_t nd = cd < (uint32_t)K ? cd : (uint32_t)K;
    for (uint32_t slot = 0; slot < K; ++slot) {
      if (!((o->chg[sb * 4 + (slot >> 5)] >> (slot & 31)) & 1u)) continue;
      const uint32_t f = slot < n ? o->res[2 * (sb * K + slot)] : 0u;
      const uint32_t d = slot >= nd ? 0u
                         : (o->split ? o->dur[2 * (sb * K + slot)]
                                     : (o->dur ? o->dur[sb * K + slot] : f));
      if ((f > d ? f : d) >= PACK_LIMIT) o->hc[sb] |= HC_BIG;
    }
  }
}

/* Emptied reservoirs (reset, failure): split handles drop the duration count and the pending
 * guesses; reservoir_mode VPP zeroes every bin (VPP's zeroed shm, shm_proxy.py:518-543 reads all
 * 128). */
static void clear_reservoirs(oracle_t* o, size_t sb) {
  if (o->split) {
    o->res_count_dur[sb] = 0u;
    o->pend_hc[sb] = 0u;
  }
  if (o->res_vpp) {
    memset(o->res + sb * K * 2, 0, (size_t)K * 8);
    if (o->dur) memset(o->dur + sb * K * (o->split ? 2 : 1), 0, (size_t)K * (o->split ? 8 : 4));
  }
}

static void pop_until(env_ctx* e, int s, int32_t t, uint64_t base_us, double den) {
  oracle_t* o = e->o;
  const size_t sb = e->b * (size_t)o->S + (size_t)s;
  int head = ring_head(o, sb), cnt = ring_count(o, sb);
  while (cnt > 0) {
    const int32_t* ent = &o->ring[(sb * o->Q + (size_t)head) * 2];
    const int32_t tc = ent[0], ta = ent[1];
    if (tc > t) break;
    const int32_t start = ta > o->last_tc[sb] ? ta : o->last_tc[sb];
    /* the sample is (float)(int32_t)fct * 1e-6f seconds */
    /* n_flow_on_mode VPP: a lost-FIN flow (the test of oracle_lost_fin_fct) is counted at its
     * completion, sampled or not */
    if (o->leak && oracle_lost_fin_fct(0u, (uint32_t)base_us + (uint32_t)ta, e->gid,
                                       o->episode[e->b], o->key[0], o->key[1], o->lf_thr, 1, 0.0f) != 0u)
      o->lost_on[sb] += 1u;
    const uint32_t fct = oracle_lost_fin_fct((uint32_t)(tc - ta), (uint32_t)base_us + (uint32_t)ta,
                                             e->gid, o->episode[e->b], o->key[0], o->key[1],
                                             o->lf_thr, o->lf_off_us, o->lf_wait_us);
    /* the flow-duration sample: VPP records time_now - t_init on every plain ACK after the first
     * (lbhash.h:129-136: states ACKed / PSHACKed), the last one at the flow's last data packet --
     * its completion here -- so the sample is the flow's age tc - ta, queueing wait included
     * (problem-01 README "from first packet to last packet"); duration_mode SERVICE keeps the
     * service time tc - max(ta, predecessor's tc) */
    const uint32_t dur =
        (uint32_t)(tc - (o->cfg.duration_mode == LBSIM_DURATION_SERVICE ? start : ta));
    o->last_tc[sb] = tc;
    const uint32_t ts_ms = (uint32_t)((base_us + (uint64_t)(int64_t)tc) / 1000u);
    /* ta >= 0: arrived in this step (times are relative to the step start) */
    const uint32_t r = o->flow_r[sb * o->Q + (size_t)head];
    if (o->split) {
      /* lost-FIN (lbhash.h:175-217): the guesses due by tc first, then this flow's duration
       * sample (its age at its last packet, lbhash.h:129-136: recorded now), then its fct -- now
       * (RSTACK seen, :116-124) or, lost, as a guess due at the wrap-up: the entry expires
       * flow_timeout after this last packet and the next flow hashed into the bucket, after the
       * wait, records now - t_init - 40 s (:182-192, :204-213) */
      pend_flush(e, s, tc, base_us);
      split_add(e, s, 1, dur, ts_ms, ta >= 0, r);
      int32_t wait = 0;
      if (lf_test((uint32_t)base_us + (uint32_t)ta, e->gid, o->episode[e->b], o->key[0], o->key[1],
                  o->lf_thr, o->lf_wait_us, &wait))
        pend_push(e, s, (uint32_t)base_us + (uint32_t)tc + (uint32_t)(o->lf_off_us + 40000000) +
                            (uint32_t)wait,
                  lf_guess((uint32_t)(tc - ta), o->lf_off_us, wait));
      else
        split_add(e, s, 0, (uint32_t)(tc - ta), ts_ms, ta >= 0, r);
    } else {
      reservoir_add(e, s, fct, dur, ts_ms, ta >= 0, r);
    }
    head = head + 1 == o->Q ? 0 : head + 1;
    cnt -= 1;
  }
  ring_set(o, sb, head, cnt);
  (void)den;
}

static void draw_arrival(env_ctx* e, int32_t t_prev) {
  oracle_t* o = e->o;
  const size_t b = e->b;
  const uint32_t ctr[4] = {o->arr_idx[b], e->gid, o->episode[b], 1u << 24};
  uint32_t d[4];
  oracle_philox(ctr, o->key, d);
  if (o->cfg.arrival_source == LBSIM_ARRIVAL_TRACE) {
    /* row (gid * 7919 + (episode - 1) * 1000003 + k) mod rows of the k-th arrival */
    const uint64_t v = (uint64_t)e->gid * 7919u + (uint64_t)(o->episode[b] - 1u) * 1000003u +
                       (uint64_t)o->arr_idx[b];
    const uint32_t r = (uint32_t)(v % (uint64_t)o->trace_rows);
    o->next_arr[b] = t_prev + (int32_t)o->trace_gap[r];
    o->next_work[b] = o->trace_work[r];
  } else {
    const int32_t gap = (int32_t)(-oracle_logf(u01(d[0])) * o->mean_gap_us);
    o->next_arr[b] = t_prev + gap;
    o->next_work[b] = -oracle_logf(u01(d[1]));
  }
  o->next_u2[b] = d[2];
  o->next_u3[b] = d[3];
}

static void sim_step(env_ctx* e, const float* w) {
  oracle_t* o = e->o;
  const size_t b = e->b;
  const int S = o->S, Q = o->Q;
  const int policy = o->cfg.assign_policy;
  const uint64_t base_us = (uint64_t)o->clock[b] * (uint64_t)o->dt_us;
  double den[LBSIM_MAX_SERVERS];
  for (int s = 0; s < S; ++s) den[s] = (double)w[s] + 1e-9;
  /* ALIAS: the table over the servers with weight > 0 (register_as_weights, shm_proxy.py:642-648),
   * alias indices are positions in that active list (node.c:449-460 as_indexes) */
  int n_act = 0, act[LBSIM_MAX_SERVERS];
  float w_act[LBSIM_MAX_SERVERS], odd[LBSIM_MAX_SERVERS];
  int32_t alias[LBSIM_MAX_SERVERS];
  if (policy == LBSIM_POLICY_ALIAS) {
    for (int s = 0; s < S; ++s)
      if (w[s] > 0.0f) { act[n_act] = s; w_act[n_act] = w[s]; ++n_act; }
    double odd64[LBSIM_MAX_SERVERS];
    oracle_gen_alias(w_act, n_act, odd64, alias);
    for (int k = 0; k < n_act; ++k) odd[k] = (float)odd64[k];
  }
  /* server failure / recovery at the step start (THEORY.md §6.4): one draw per server, stream 5,
   * counter (clock, gid, episode); a failing server loses its queued flows (counted as dropped)
   * and its reservoirs, and takes no flows while down (capacity 0, as a full server) */
  int qcap[LBSIM_MAX_SERVERS];
  for (int s = 0; s < S; ++s) qcap[s] = Q;
  if (o->down) {
    for (int s = 0; s < S; ++s) {
      const size_t sb = b * (size_t)S + (size_t)s;
      const uint32_t ctr[4] = {o->clock[b], e->gid, o->episode[b], (5u << 24) | (uint32_t)s};
      uint32_t d[4];
      oracle_philox(ctr, o->key, d);
      const uint32_t u = d[0] >> 8;
      if (o->down[sb]) {
        if (u < o->rec_thr) o->down[sb] = 0u;
      } else if (u < o->fail_thr) {
        o->down[sb] = 1u;
        o->dropped[b] += (uint32_t)ring_count(o, sb);
        o->hc[sb] = (uint32_t)ring_head(o, sb); /* empty queue, reservoirs emptied: no HC_BIG */
        o->last_tc[sb] = LAST_NONE;
        o->res_count[sb] = 0u;
        if (o->lost_on) o->lost_on[sb] = 0u;
        o->chg[sb * 4] |= 1u; /* emptied: the next observe recomputes the (zero) features */
        clear_reservoirs(o, sb);
      }
      if (o->down[sb]) qcap[s] = 0;
    }
  }

  while (o->next_arr[b] < o->dt_us) {
    const int32_t ta = o->next_arr[b];
    for (int s = 0; s < S; ++s) pop_until(e, s, ta, base_us, den[s]);
    int cnt[LBSIM_MAX_SERVERS];
    float sc[LBSIM_MAX_SERVERS];
    for (int s = 0; s < S; ++s) {
      const size_t sb = b * (size_t)S + (size_t)s;
      cnt[s] = ring_count(o, sb);
      /* node.c:395-437 score on the as_stat n_flow_on, which never drops a lost-FIN flow
       * (lbhash.h:193,214): under n_flow_on_mode VPP the queue plus the server's lost flows
       * completed so far (counted at their pop, pop_until); eligibility stays the queue */
      sc[s] = score_of(policy, cnt[s] + (o->lost_on ? (int32_t)o->lost_on[sb] : 0), den[s]);
    }
    int chosen = -1;
    if (policy == LBSIM_POLICY_ALIAS) {
      /* node.c:442-460: rand_num = U * n, bucket = (int)rand_num, alias if the fraction exceeds
       * odd[bucket]; U = 24 bits of the arrival's hash word (never 1, unlike rand()/RAND_MAX).
       * A full server drops the flow (ALIAS has no eligibility test). */
      if (n_act > 0) {
        const float rn = (float)(o->next_u2[b] >> 8) * 5.9604644775390625e-8f * (float)n_act;
        int bucket = (int)rn;
        if (bucket > n_act - 1) bucket = n_act - 1;
        const int k = (rn - (float)bucket) > odd[bucket] ? alias[bucket] : bucket;
        if (cnt[act[k]] < qcap[act[k]]) chosen = act[k];
      }
    } else if (policy == LBSIM_POLICY_SED2 || policy == LBSIM_POLICY_LSQ2) {
      /* node.c:409-417 / 433-441: two candidates, keep the second only if strictly better; the
       * candidates are the hash word's high and low 16 bits mapped to [0, S) */
      const int h1 = (int)(((o->next_u2[b] >> 16) * (uint32_t)S) >> 16);
      const int h2 = (int)(((o->next_u2[b] & 0xFFFFu) * (uint32_t)S) >> 16);
      const int ok1 = cnt[h1] < qcap[h1], ok2 = cnt[h2] < qcap[h2];
      if (ok1 && ok2) chosen = sc[h2] < sc[h1] ? h2 : h1;
      else if (ok1) chosen = h1;
      else if (ok2) chosen = h2;
    } else {
      /* node.c:393-404: start at the hashed (Maglev) server, replace on strictly lower score */
      const int h = (int)(((uint64_t)o->next_u2[b] * (uint64_t)S) >> 32);
      float best = 0.0f;
      if (cnt[h] < qcap[h]) { chosen = h; best = sc[h]; }
      for (int s = 0; s < S; ++s)
        if (cnt[s] < qcap[s] && (chosen < 0 || sc[s] < best)) { chosen = s; best = sc[s]; }
    }
    if (chosen < 0) {
      o->dropped[b] += 1u;
    } else {
      const int s = chosen;
      const size_t sb = b * (size_t)S + (size_t)s;
      const int head = ring_head(o, sb), c = ring_count(o, sb);
      int32_t start = ta;
      if (c > 0) {
        int tp = head + c - 1;
        if (tp >= Q) tp -= Q;
        const int32_t tail_tc = o->ring[(sb * Q + (size_t)tp) * 2];
        start = tail_tc > ta ? tail_tc : ta;
      }
      int32_t svc = (int32_t)(o->next_work[b] * o->svc_scale[s]);
      if (svc < 1) svc = 1;
      int pos = head + c;
      if (pos >= Q) pos -= Q;
      o->ring[(sb * Q + (size_t)pos) * 2] = start + svc;
      o->ring[(sb * Q + (size_t)pos) * 2 + 1] = ta;
      o->flow_r[sb * Q + (size_t)pos] = o->next_u3[b];
      ring_set(o, sb, head, c + 1);
      e->assigned[s] += 1;
    }
    o->arr_idx[b] += 1u;
    draw_arrival(e, ta);
  }
  for (int s = 0; s < S; ++s) pop_until(e, s, o->dt_us, base_us, den[s]);
  /* split handles: the guesses due by the step's end */
  if (o->split)
    for (int s = 0; s < S; ++s) pend_flush(e, s, o->dt_us, base_us);
  /* rebase to the next step */
  const int32_t dt = o->dt_us;
  o->next_arr[b] -= dt;
  for (int s = 0; s < S; ++s) {
    const size_t sb = b * (size_t)S + (size_t)s;
    int pos = ring_head(o, sb);
    const int c = ring_count(o, sb);
    for (int i = 0; i < c; ++i) {
      o->ring[(sb * Q + (size_t)pos) * 2] -= dt;
      o->ring[(sb * Q + (size_t)pos) * 2 + 1] -= dt;
      pos = pos + 1 == Q ? 0 : pos + 1;
    }
    o->last_tc[sb] = o->last_tc[sb] < LAST_NONE + dt ? LAST_NONE : o->last_tc[sb] - dt;
  }
  o->clock[b] += 1u;
}

static float action_weight(const oracle_t* o, const void* action, int dtype, size_t idx) {
  const lbsim_config_t* c = &o->cfg;
  if (c->action_type == LBSIM_ACTION_DISCRETE) {
    int64_t a = dtype == LBSIM_DTYPE_I64 ? ((const int64_t*)action)[idx]
                                         : (int64_t)((const int32_t*)action)[idx];
    if (a < 0) a += c->num_discrete;
    if (a < 0) a = 0;
    if (a >= c->num_discrete) a = c->num_discrete - 1;
    return c->discrete_weights[a];
  }
  const float a = ((const float*)action)[idx];
  return a < c->min_weight ? c->min_weight : (a > c->max_weight ? c->max_weight : a);
}

/* env.py:460-468: running mean/std in float64; count is incremented first; out = float32 cast. */
void oracle_normalize(const float* raw, int n, int32_t* count, double* mean, double* std,
                      float* out) {
  const int32_t cnt = *count + 1;
  for (int e = 0; e < n; ++e) {
    const double ob = (double)raw[e];
    double m = mean[e];
    const double sd = std[e];
    const double delta = ob - m;
    m = m + delta / (double)cnt;
    const double delta2 = ob - m;
    double v = (sd * sd * (double)(cnt - 1) + delta * delta2) / (double)cnt;
    v = v > 1e-8 ? v : 1e-8;
    const double ns = sqrt(v);
    mean[e] = m;
    std[e] = ns;
    out[e] = (float)((ob - m) / (ns + 1e-8));
  }
  *count = cnt;
}

/* Observation (S, 11), reward, bookkeeping and normalisation of env b. */
static void observe(oracle_t* o, size_t b, float* obs_out, float* reward_out, uint8_t* done_out,
                    int step_mode) {
  const int S = o->S;
  float raw[LBSIM_MAX_SERVERS * NF];
  for (int s = 0; s < S; ++s) {
    const size_t sb = b * (size_t)S + (size_t)s;
    const uint32_t rc = o->res_count[sb];
    const int n = rc < (uint32_t)K ? (int)rc : K;
    float w[K];
    uint64_t wq[K];
    uint32_t ts[K];
    for (int i = 0; i < n; ++i) ts[i] = o->res[2 * (sb * K + (size_t)i) + 1];
    slot_weights(ts, n, o->decay_c, w, wq);
    float ff[5], fd[5], vf[K], vd[K];
    for (int i = 0; i < n; ++i) {
      vf[i] = us_to_seconds(o->res[2 * (sb * K + (size_t)i)]);
      /* paired records (no duration plane): the duration reservoir is the fct reservoir */
      vd[i] = o->dur && !o->split ? us_to_seconds(o->dur[sb * K + (size_t)i]) : vf[i];
    }
    features_one(vf, w, wq, n, ff);
    if (o->split) {
      /* the duration reservoir of a split handle: its own count and timestamps */
      const uint32_t cd = o->res_count_dur[sb];
      const int nd = cd < (uint32_t)K ? (int)cd : K;
      float wd[K];
      uint64_t wqd[K];
      for (int i = 0; i < nd; ++i) {
        vd[i] = us_to_seconds(o->dur[2 * (sb * K + (size_t)i)]);
        ts[i] = o->dur[2 * (sb * K + (size_t)i) + 1];
      }
      slot_weights(ts, nd, o->decay_c, wd, wqd);
      features_one(vd, wd, wqd, nd, fd);
    } else {
      features_one(vd, w, wq, n, fd);
    }
    for (int f = 0; f < 5; ++f) { o->fcache[sb * 10 + (size_t)f] = ff[f]; o->fcache[sb * 10 + 5 + (size_t)f] = fd[f]; }
    /* n_flow_on: flows in flight, plus the lost-FIN flows VPP never decrements (n_flow_on_mode
     * VPP, lbhash.h:193,214) */
    raw[s * NF + 0] = (float)((uint32_t)ring_count(o, sb) + (o->lost_on ? o->lost_on[sb] : 0u));
    for (int f = 0; f < 5; ++f) { raw[s * NF + 1 + f] = ff[f]; raw[s * NF + 6 + f] = fd[f]; }
  }
  if (step_mode) {
    const double r = oracle_reward(raw, S, o->cfg.reward_metric, o->cfg.reward_field);
    reward_out[b] = (float)r;
    o->ep_step[b] += 1;
    o->ep_return[b] += r;
    done_out[b] = (uint8_t)(o->ep_step[b] >= o->cfg.max_steps);
  }
  float* row = obs_out + b * (size_t)S * NF;
  if (o->cfg.normalize_obs) {
    const size_t off = b * (size_t)S * NF;
    oracle_normalize(raw, S * NF, &o->norm_count[b], o->norm_mean + off, o->norm_std + off, row);
  } else {
    memcpy(row, raw, sizeof(float) * (size_t)S * NF);
  }
}

static void reset_env(oracle_t* o, size_t b) {
  env_ctx e;
  memset(&e, 0, sizeof(e));
  e.o = o; e.b = b; e.gid = (uint32_t)(o->cfg.env_id_offset + (int64_t)b);
  const int S = o->S;
  o->episode[b] += 1u;
  o->clock[b] = 0u;
  o->dropped[b] = 0u;
  o->arr_idx[b] = 0u;
  draw_arrival(&e, 0);
  for (int s = 0; s < S; ++s) {
    const size_t sb = b * (size_t)S + (size_t)s;
    o->hc[sb] = 0u;
    o->last_tc[sb] = LAST_NONE;
    o->res_count[sb] = 0u;
    /* emptied reservoirs: slot 0 marked written (the GPU's next observe recomputes every server
     * of the env instead of reusing the last episode's cached features) */
    for (int w = 0; w < 4; ++w) o->chg[sb * 4 + (size_t)w] = w == 0 ? 1u : 0u;
    if (o->down) o->down[sb] = 0u; /* every server is up at the episode start */
    if (o->lost_on) o->lost_on[sb] = 0u;
    clear_reservoirs(o, sb);
  }
  if (o->split) o->lf_over[b] = 0u;
  float w1[LBSIM_MAX_SERVERS];
  for (int s = 0; s < LBSIM_MAX_SERVERS; ++s) w1[s] = 1.0f;
  for (int k = 0; k < o->cfg.warmup_steps; ++k) sim_step(&e, w1);
  big_scan(o, b);
  o->ep_step[b] = 0;
  o->ep_return[b] = 0.0;
}

int oracle_reset(oracle_t* o, const uint8_t* mask, float* obs_out) {
  const long B = o->B;
  if (o->cfg.arrival_source == LBSIM_ARRIVAL_TRACE && o->trace_rows == 0) return -2;
#pragma omp parallel for schedule(dynamic, 16) num_threads(o->threads)
  for (long b = 0; b < B; ++b) {
    if (mask && !mask[b]) continue;
    reset_env(o, (size_t)b);
    observe(o, (size_t)b, obs_out, NULL, NULL, 0);
  }
  if (!mask) o->initialised = 1;
  return 0;
}

int oracle_step(oracle_t* o, const void* action, int dtype, float* obs_out, float* reward_out,
                uint8_t* done_out, int32_t* assign_out) {
  if (!o->initialised) return LBSIM_EINVAL;
  const long B = o->B;
  const int S = o->S;
#pragma omp parallel for schedule(dynamic, 16) num_threads(o->threads)
  for (long b = 0; b < B; ++b) {
    env_ctx e;
    memset(&e, 0, sizeof(e));
    e.o = o; e.b = (size_t)b; e.gid = (uint32_t)(o->cfg.env_id_offset + (int64_t)b);
    for (size_t i = 0; i < (size_t)S * 4; ++i) o->chg[(size_t)b * S * 4 + i] = 0u;
    if (o->cfg.next_step_reset && o->ep_step[b] >= o->cfg.max_steps) {
      /* gymnasium NEXT_STEP autoreset: the env that returned done last step resets instead of
       * stepping (its action is ignored): reset observation, reward 0, done 0, counts 0 */
      reset_env(o, (size_t)b);
      if (assign_out)
        for (int s = 0; s < S; ++s) assign_out[(size_t)b * S + (size_t)s] = 0;
      observe(o, (size_t)b, obs_out, NULL, NULL, 0);
      reward_out[b] = 0.0f;
      done_out[b] = 0u;
      continue;
    }
    float w[LBSIM_MAX_SERVERS];
    for (int s = 0; s < S; ++s) w[s] = action_weight(o, action, dtype, (size_t)b * S + (size_t)s);
    sim_step(&e, w);
    big_scan(o, (size_t)b);
    if (assign_out)
      for (int s = 0; s < S; ++s) assign_out[(size_t)b * S + (size_t)s] = e.assigned[s];
    observe(o, (size_t)b, obs_out, reward_out, done_out, 1);
  }
  return 0;
}

void oracle_episode_stats(const oracle_t* o, int32_t* len_out, double* ret_out) {
  for (int b = 0; b < o->B; ++b) {
    if (len_out) len_out[b] = o->ep_step[b];
    if (ret_out) ret_out[b] = o->ep_return[b];
  }
}

/* Stateless batch helpers used by the golden tests. */
void oracle_reward_batch(const float* obs, long n, int S, int metric, int field, float* out) {
  for (long i = 0; i < n; ++i) out[i] = (float)oracle_reward(obs + i * (long)S * NF, S, metric, field);
}

void oracle_reward_batch64(const float* obs, long n, int S, int metric, int field, double* out) {
  for (long i = 0; i < n; ++i) out[i] = oracle_reward(obs + i * (long)S * NF, S, metric, field);
}

void oracle_features_batch(const float* values, const uint32_t* ts, const uint32_t* counts, long n,
                           float decay_factor, float* out) {
  for (long r = 0; r < n; ++r)
    oracle_reservoir_features(values + r * K, ts + r * K, counts[r], decay_factor, out + r * 5);
}

/* Algorithm R slot for the insert that sees `count` earlier samples (-1 = rejected); exposes the
 * decision rule alone for the uniformity test (test_reservoir.py:243-287 analogue). */
long oracle_algr_slot(uint32_t count, uint32_t gid, uint32_t episode, uint32_t server,
                      const uint32_t key[2]) {
  if (count < (uint32_t)K) return (long)count;
  const uint32_t ctr[4] = {count >> 1, gid, episode, (2u << 24) | server};
  uint32_t d[4];
  oracle_philox(ctr, key, d);
  const uint32_t hi = (count & 1u) ? d[3] : d[1];
  const uint32_t lo = (count & 1u) ? d[2] : d[0];
  const unsigned __int128 prod = (unsigned __int128)(((uint64_t)hi << 32) | lo) * ((uint64_t)count + 1u);
  const uint64_t j = (uint64_t)(prod >> 64);
  return j < (uint64_t)K ? (long)j : -1;
}

/* ------------------------------------------------------------------ VPP shm (upstream) features */
/* Shm_Manager.process_reservoir (src/lb/shm_proxy.py:518-543) of n raw VPP reservoirs: tv[r][128]
 * (t, v) f32 pairs (reservoir_as_t, src/vpp/lb/shm.h:35-37), frame time ts[r / res_per_ts] (the
 * msg_out_t f32, a Python float).  Over all 128 bins in float64, numpy's order:
 *   mean = pairwise(v) / 128; p90 = 'linear' percentile (virtual index 127 * 0.9, _lerp);
 *   std = sqrt(pairwise((v - mean)^2) / 128); vd = v * pow(decay, ts - t); mean(vd), p90(vd). */
static int cmp_f64(const void* a, const void* b) {
  const double x = *(const double*)a, y = *(const double*)b;
  return (x > y) - (x < y);
}

static double np_p90_128(double* s) {
  qsort(s, 128, sizeof(double), cmp_f64);
  const double vi = 127.0 * 0.9, gamma = vi - 114.0;
  const double a = s[114], d = s[115] - a;
  return a + d * gamma; /* gamma < 0.5: _lerp's add branch */
}

void oracle_vpp_features(const float* tv, const float* ts, long res_per_ts, long n, double decay,
                         double* out) {
  for (long r = 0; r < n; ++r) {
    const float* p = tv + r * 256;
    const double now = (double)ts[r / res_per_ts];
    double v[128], vd[128], x2[128], s[128];
    for (int i = 0; i < 128; ++i) {
      v[i] = (double)p[2 * i + 1];
      vd[i] = v[i] * pow(decay, now - (double)p[2 * i]);
    }
    const double mean = pw64(v, 128) / 128.0;
    for (int i = 0; i < 128; ++i) {
      const double x = v[i] - mean;
      x2[i] = x * x;
    }
    double* o = out + r * 5;
    o[0] = mean;
    memcpy(s, v, sizeof(s));
    o[1] = np_p90_128(s);
    o[2] = sqrt(pw64(x2, 128) / 128.0);
    o[3] = pw64(vd, 128) / 128.0;
    memcpy(s, vd, sizeof(s));
    o[4] = np_p90_128(s);
  }
}
