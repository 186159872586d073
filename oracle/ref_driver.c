/*
 * ref_driver.c -- TEST INFRASTRUCTURE ONLY (CPU baseline + oracle cross-check).
 *
 * Drives the reference's OWN compiled SIMD kernel (simd_c/reedsolomon.c, compiled
 * from /root/reference by oracle/Makefile into oracle/_ref/, never copied) the way
 * the reference's Rust code does:
 *   - galois_8.rs:291-327  mul_slice / mul_slice_xor: SIMD prefix through the FFI,
 *     then the pure-Rust tail (galois_8.rs:137-219) from `bytes_done`;
 *   - core.rs:481-509      code_some_slices loop order (input-major, first input
 *     overwrites, later inputs accumulate).
 * Tables come from the build.rs restatement in rse_oracle.c (pinned by the
 * reference's LOG-table known answer, galois_8.rs:339-363).
 */
#include <stddef.h>
#include <stdint.h>

#include "rse_oracle.h"

/* simd_c/reedsolomon.h:30-42 */
size_t reedsolomon_gal_mul(const uint8_t low[16], const uint8_t high[16],
                           const uint8_t *restrict in, uint8_t *restrict out,
                           size_t len);
size_t reedsolomon_gal_mul_xor(const uint8_t low[16], const uint8_t high[16],
                               const uint8_t *restrict in, uint8_t *restrict out,
                               size_t len);

static uint8_t MUL[256 * 256], LOW[256 * 16], HIGH[256 * 16];
static int ready = 0;

static void init(void) {
  if (ready) return;
  oracle_gf8_tables(0, 0, MUL, LOW, HIGH);
  ready = 1;
}

/* galois_8.rs:291-305 */
void ref_gf8_mul_slice(uint8_t c, const uint8_t *in, uint8_t *out, size_t len) {
  init();
  size_t done = reedsolomon_gal_mul(&LOW[c * 16], &HIGH[c * 16], in, out, len);
  const uint8_t *row = &MUL[c * 256];
  for (size_t j = done; j < len; j++) out[j] = row[in[j]];
}

/* galois_8.rs:313-327 */
void ref_gf8_mul_slice_xor(uint8_t c, const uint8_t *in, uint8_t *out, size_t len) {
  init();
  size_t done = reedsolomon_gal_mul_xor(&LOW[c * 16], &HIGH[c * 16], in, out, len);
  const uint8_t *row = &MUL[c * 256];
  for (size_t j = done; j < len; j++) out[j] ^= row[in[j]];
}

/* bytes the SIMD kernel itself covers for a given length (its vector width) */
size_t ref_gf8_simd_bytes(size_t len) {
  static uint8_t in[512], out[512];
  init();
  if (len > sizeof in) len = sizeof in;
  return reedsolomon_gal_mul(&LOW[16], &HIGH[16], in, out, len);
}

/* core.rs:481-509 code_some_slices over GF(2^8) */
void ref_gf8_code_some_slices(const uint8_t *rows, size_t n_out, size_t n_in,
                              const uint8_t *const *inputs, uint8_t *const *outputs,
                              size_t len) {
  init();
  for (size_t i = 0; i < n_in; i++)
    for (size_t r = 0; r < n_out; r++) {
      uint8_t c = rows[r * n_in + i];
      if (i == 0) ref_gf8_mul_slice(c, inputs[i], outputs[r], len);
      else ref_gf8_mul_slice_xor(c, inputs[i], outputs[r], len);
    }
}

/* `reps` back-to-back code_some_slices calls (a per-call CPU timing without
 * the caller's per-call FFI overhead; bench.py's reference bench matrix) */
void ref_gf8_code_repeat(const uint8_t *rows, size_t n_out, size_t n_in,
                         const uint8_t *const *inputs, uint8_t *const *outputs, size_t len,
                         size_t reps) {
  for (size_t t = 0; t < reps; t++) ref_gf8_code_some_slices(rows, n_out, n_in, inputs, outputs, len);
}
