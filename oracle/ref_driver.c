/*
 * ref_driver.c — exports the reference's header-only C reservoir twin
 * (simulation-mode/problem-01-reservoir-sampling/src/reservoir.h, included IN PLACE from the
 * reference tree via -DREF_RESERVOIR_H) as a shared library under oracle/_ref/.
 * TEST INFRASTRUCTURE ONLY: used by tests/test_ref_twin.py to cross-check the oracle's
 * Algorithm R fill/replacement rule and reservoir statistics against the reference's own C.
 * No reference source is copied into this repository.
 */
#include REF_RESERVOIR_H

size_t ref_reservoir_sizeof(void) { return sizeof(reservoir_t); }
void ref_reservoir_init(reservoir_t* r, uint64_t seed) { reservoir_init(r, seed); }
int ref_reservoir_add(reservoir_t* r, float v, uint64_t ts_us) { return reservoir_add(r, v, ts_us); }
uint64_t ref_reservoir_count(const reservoir_t* r) { return r->count; }
const float* ref_reservoir_values(const reservoir_t* r) { return r->values; }
void ref_reservoir_stats(const reservoir_t* r, float decay, uint64_t now_us, float out[5]) {
  reservoir_stats_t s;
  memset(&s, 0, sizeof(s));
  reservoir_compute_stats(r, &s, decay, now_us);
  out[0] = s.mean; out[1] = s.p90; out[2] = s.std; out[3] = s.mean_decay; out[4] = s.p90_decay;
}
