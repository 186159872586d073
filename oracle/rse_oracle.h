/*
 * rse_oracle.h -- TEST INFRASTRUCTURE ONLY (the checker, never the product).
 *
 * A plain-C restatement of rust-rse/reed-solomon-erasure v6.0.0's arithmetic and
 * codec semantics, used by tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg to check the HIP library.  Nothing under reed-solomon-erasure_amd/
 * links, includes or calls this file.
 *
 * Pinning: tests/test_oracle_golden.py checks this restatement against every
 * known-answer vector the reference's own tests hold (galois_8.rs:339-363,
 * 482-552; matrix.rs:372-411; tests/mod.rs:249-353, 851-893; README 3+2;
 * sage/galois_ext_test.sage:10-26) and against the reference's own compiled
 * SIMD kernel (simd_c/reedsolomon.c, built by oracle/Makefile into oracle/_ref/).
 *
 * Lengths are in field ELEMENTS (1 byte for GF(2^8), 2 bytes for GF(2^16)),
 * exactly as Rust slice lengths are in the reference.
 * Return codes: 0 = Ok, 1..13 = errors.rs:4-18 Error variants in declaration order.
 */
#ifndef RSE_ORACLE_H
#define RSE_ORACLE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- GF(2^8): build.rs:13-94, galois_8.rs:56-103 ---------------------- */
void oracle_gf8_tables(uint8_t log_table[256], uint8_t exp_table[510],
                       uint8_t mul_table[256 * 256], uint8_t mul_low[256 * 16],
                       uint8_t mul_high[256 * 16]);
uint8_t oracle_gf8_add(uint8_t a, uint8_t b);
uint8_t oracle_gf8_mul(uint8_t a, uint8_t b);
uint8_t oracle_gf8_div(uint8_t a, uint8_t b); /* b == 0 -> returns 0 and sets errno-like flag; reference panics */
uint8_t oracle_gf8_exp(uint8_t a, size_t n);
/* galois_8.rs:137-219 (pure-Rust path) */
void oracle_gf8_mul_slice(uint8_t c, const uint8_t *in, uint8_t *out, size_t n);
void oracle_gf8_mul_slice_xor(uint8_t c, const uint8_t *in, uint8_t *out, size_t n);

/* ---- GF(2^16) = GF((2^8)^2): galois_16.rs ----------------------------- */
/* Elements are [u8;2] = {coefficient of x, constant} (galois_16.rs:49-51). */
void oracle_gf16_add(const uint8_t a[2], const uint8_t b[2], uint8_t out[2]);
void oracle_gf16_mul(const uint8_t a[2], const uint8_t b[2], uint8_t out[2]);
int oracle_gf16_inverse(const uint8_t a[2], uint8_t out[2]); /* -1 on zero (reference panics) */
int oracle_gf16_div(const uint8_t a[2], const uint8_t b[2], uint8_t out[2]);
void oracle_gf16_exp(const uint8_t a[2], size_t n, uint8_t out[2]);

/* ---- Matrix: matrix.rs:119-276 (field = 8 or 16) ----------------------- */
/* row-major, elem_size 1 or 2 bytes.  Returns 0, or -1 if singular. */
int oracle_matrix_invert(int field, const uint8_t *m, size_t n, uint8_t *out);
void oracle_matrix_multiply(int field, const uint8_t *a, size_t ar, size_t ac,
                            const uint8_t *b, size_t bc, uint8_t *out);
void oracle_matrix_vandermonde(int field, size_t rows, size_t cols, uint8_t *out);

/* ---- Codec: core.rs:343-923 -------------------------------------------- */
typedef struct oracle_codec oracle_codec;

int oracle_codec_new(int field, size_t data_shards, size_t parity_shards,
                     oracle_codec **out); /* core.rs:445-467 */
void oracle_codec_free(oracle_codec *c);
/* (k+p) x k encoding matrix, elem_size bytes per element */
const uint8_t *oracle_codec_matrix(const oracle_codec *c);
size_t oracle_codec_data_shards(const oracle_codec *c);
size_t oracle_codec_parity_shards(const oracle_codec *c);

/* core.rs:481-509 code_some_slices: out_r = sum_i rows[r][i] * in_i */
void oracle_code_some_slices(int field, const uint8_t *rows, size_t n_out,
                             size_t n_in, const uint8_t *const *inputs,
                             uint8_t *const *outputs, size_t len_elems);

int oracle_encode(const oracle_codec *c, uint8_t *const *shards,
                  const size_t *lens, size_t n); /* core.rs:597-611 */
int oracle_encode_sep(const oracle_codec *c, const uint8_t *const *data,
                      const size_t *data_lens, size_t n_data,
                      uint8_t *const *parity, const size_t *parity_lens,
                      size_t n_parity); /* core.rs:617-632 */
int oracle_encode_single(const oracle_codec *c, size_t i_data,
                         uint8_t *const *shards, const size_t *lens,
                         size_t n); /* core.rs:545-562 */
int oracle_encode_single_sep(const oracle_codec *c, size_t i_data,
                             const uint8_t *single, size_t single_len,
                             uint8_t *const *parity, const size_t *parity_lens,
                             size_t n_parity); /* core.rs:576-592 */
int oracle_verify(const oracle_codec *c, const uint8_t *const *shards,
                  const size_t *lens, size_t n, int *ok); /* core.rs:637-651 */
int oracle_verify_with_buffer(const oracle_codec *c,
                              const uint8_t *const *shards, const size_t *lens,
                              size_t n, uint8_t *const *buffer,
                              const size_t *buf_lens, size_t n_buf,
                              int *ok); /* core.rs:654-669 */
/* (T, bool) ReconstructShard semantics (lib.rs:168-200): a missing shard's
 * buffer must have the common length or IncorrectShardSize is returned. */
int oracle_reconstruct(const oracle_codec *c, uint8_t *const *shards,
                       const size_t *lens, const uint8_t *present, size_t n,
                       int data_only); /* core.rs:733-923 */

#ifdef __cplusplus
}
#endif
#endif
