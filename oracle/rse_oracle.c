/*
 * rse_oracle.c -- TEST INFRASTRUCTURE ONLY: the CPU checker for the HIP library.
 *
 * Plain-C restatement of rust-rse/reed-solomon-erasure v6.0.0 (the reference is
 * Rust; no Rust toolchain exists in this image, so the crate itself cannot run).
 * Every function cites the reference file:line it follows.  It is pinned by the
 * reference's own known-answer tests and by the reference's own compiled SIMD
 * kernel (see rse_oracle.h and tests/test_oracle_golden.py).
 *
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load
 * this code.  The shipped library (reed-solomon-erasure_amd/) never does.
 */
#include "rse_oracle.h"

#include <stdlib.h>
#include <string.h>

/* errors.rs:4-18, numbered as wasm/src/lib.rs:11-24 */
enum {
  E_OK = 0,
  E_TOO_FEW_SHARDS = 1,
  E_TOO_MANY_SHARDS = 2,
  E_TOO_FEW_DATA_SHARDS = 3,
  E_TOO_MANY_DATA_SHARDS = 4,
  E_TOO_FEW_PARITY_SHARDS = 5,
  E_TOO_MANY_PARITY_SHARDS = 6,
  E_TOO_FEW_BUFFER_SHARDS = 7,
  E_TOO_MANY_BUFFER_SHARDS = 8,
  E_INCORRECT_SHARD_SIZE = 9,
  E_TOO_FEW_SHARDS_PRESENT = 10,
  E_EMPTY_SHARD = 11,
  E_INVALID_SHARD_FLAGS = 12,
  E_INVALID_INDEX = 13,
};

/* ======================= GF(2^8) tables: build.rs ======================= */
#define FIELD_SIZE 256
#define GENERATING_POLYNOMIAL 29 /* build.rs:11 */
#define EXP_TABLE_SIZE (FIELD_SIZE * 2 - 2)

static uint8_t LOG_TABLE[FIELD_SIZE];
static uint8_t EXP_TABLE[EXP_TABLE_SIZE];
static uint8_t MUL_TABLE[FIELD_SIZE][FIELD_SIZE];
static uint8_t MUL_LOW[FIELD_SIZE][16];
static uint8_t MUL_HIGH[FIELD_SIZE][16];
static int tables_ready = 0;

/* build.rs:13-29 gen_log_table */
static void gen_log_table(void) {
  memset(LOG_TABLE, 0, sizeof LOG_TABLE);
  size_t b = 1;
  for (size_t log = 0; log < FIELD_SIZE - 1; log++) {
    LOG_TABLE[b] = (uint8_t)log;
    b = b << 1;
    if (FIELD_SIZE <= b) b = (b - FIELD_SIZE) ^ GENERATING_POLYNOMIAL;
  }
}

/* build.rs:33-43 gen_exp_table */
static void gen_exp_table(void) {
  memset(EXP_TABLE, 0, sizeof EXP_TABLE);
  for (size_t i = 1; i < FIELD_SIZE; i++) {
    size_t log = LOG_TABLE[i];
    EXP_TABLE[log] = (uint8_t)i;
    EXP_TABLE[log + FIELD_SIZE - 1] = (uint8_t)i;
  }
}

/* build.rs:45-54 multiply */
static uint8_t table_multiply(uint8_t a, uint8_t b) {
  if (a == 0 || b == 0) return 0;
  return EXP_TABLE[(size_t)LOG_TABLE[a] + (size_t)LOG_TABLE[b]];
}

static void init_tables(void) {
  if (tables_ready) return;
  gen_log_table();
  gen_exp_table();
  /* build.rs:56-69 gen_mul_table */
  for (int a = 0; a < FIELD_SIZE; a++)
    for (int b = 0; b < FIELD_SIZE; b++)
      MUL_TABLE[a][b] = table_multiply((uint8_t)a, (uint8_t)b);
  /* build.rs:71-94 gen_mul_table_half */
  for (int a = 0; a < FIELD_SIZE; a++)
    for (int b = 0; b < FIELD_SIZE; b++) {
      uint8_t r = table_multiply((uint8_t)a, (uint8_t)b);
      if ((b & 0x0F) == b) MUL_LOW[a][b] = r;
      if ((b & 0xF0) == b) MUL_HIGH[a][b >> 4] = r;
    }
  tables_ready = 1;
}

void oracle_gf8_tables(uint8_t log_table[256], uint8_t exp_table[510],
                       uint8_t mul_table[256 * 256], uint8_t mul_low[256 * 16],
                       uint8_t mul_high[256 * 16]) {
  init_tables();
  if (log_table) memcpy(log_table, LOG_TABLE, sizeof LOG_TABLE);
  if (exp_table) memcpy(exp_table, EXP_TABLE, sizeof EXP_TABLE);
  if (mul_table) memcpy(mul_table, MUL_TABLE, sizeof MUL_TABLE);
  if (mul_low) memcpy(mul_low, MUL_LOW, sizeof MUL_LOW);
  if (mul_high) memcpy(mul_high, MUL_HIGH, sizeof MUL_HIGH);
}

/* ======================= GF(2^8) ops: galois_8.rs ======================= */
/* galois_8.rs:57-59 */
uint8_t oracle_gf8_add(uint8_t a, uint8_t b) { return a ^ b; }
/* galois_8.rs:68-70 */
uint8_t oracle_gf8_mul(uint8_t a, uint8_t b) {
  init_tables();
  return MUL_TABLE[a][b];
}
/* galois_8.rs:73-87 (b == 0 panics in the reference; callers never do it) */
uint8_t oracle_gf8_div(uint8_t a, uint8_t b) {
  init_tables();
  if (a == 0) return 0;
  if (b == 0) return 0;
  int log_result = (int)LOG_TABLE[a] - (int)LOG_TABLE[b];
  if (log_result < 0) log_result += 255;
  return EXP_TABLE[log_result];
}
/* galois_8.rs:90-103 */
uint8_t oracle_gf8_exp(uint8_t a, size_t n) {
  init_tables();
  if (n == 0) return 1;
  if (a == 0) return 0;
  size_t log_result = (size_t)LOG_TABLE[a] * n;
  while (255 <= log_result) log_result -= 255;
  return EXP_TABLE[log_result];
}
/* galois_8.rs:137-175 mul_slice_pure_rust (unroll is a speed detail) */
void oracle_gf8_mul_slice(uint8_t c, const uint8_t *in, uint8_t *out, size_t n) {
  init_tables();
  const uint8_t *row = MUL_TABLE[c];
  for (size_t j = 0; j < n; j++) out[j] = row[in[j]];
}
/* galois_8.rs:177-219 mul_slice_xor_pure_rust */
void oracle_gf8_mul_slice_xor(uint8_t c, const uint8_t *in, uint8_t *out,
                              size_t n) {
  init_tables();
  const uint8_t *row = MUL_TABLE[c];
  for (size_t j = 0; j < n; j++) out[j] ^= row[in[j]];
}

/* ======================= GF(2^16): galois_16.rs ========================= */
typedef struct {
  uint8_t v[2]; /* v[0] = coefficient of x, v[1] = constant (galois_16.rs:49-51) */
} elem16;

static const uint8_t EXT_POLY[3] = {1, 2, 128}; /* galois_16.rs:14 */

static elem16 e16(uint8_t a, uint8_t b) {
  elem16 e;
  e.v[0] = a;
  e.v[1] = b;
  return e;
}
static elem16 e16_const(uint8_t n) { return e16(0, n); } /* :71-73 */
static int e16_is_zero(elem16 e) { return e.v[0] == 0 && e.v[1] == 0; }
static size_t e16_degree(elem16 e) { return e.v[0] != 0 ? 1 : 0; } /* :109-115 */

/* galois_16.rs:133-135 */
static elem16 e16_add(elem16 a, elem16 b) {
  return e16(a.v[0] ^ b.v[0], a.v[1] ^ b.v[1]);
}
/* galois_16.rs:97-107 reduce_from */
static elem16 e16_reduce_from(uint8_t x0, uint8_t x1, uint8_t x2) {
  if (x0 != 0) {
    x1 ^= oracle_gf8_mul(EXT_POLY[1], x0);
    x2 ^= oracle_gf8_mul(EXT_POLY[2], x0);
  }
  return e16(x1, x2);
}
/* galois_16.rs:149-161 */
static elem16 e16_mul(elem16 a, elem16 b) {
  uint8_t o0 = oracle_gf8_mul(a.v[0], b.v[0]);
  uint8_t o1 = oracle_gf8_add(oracle_gf8_mul(a.v[1], b.v[0]),
                              oracle_gf8_mul(a.v[0], b.v[1]));
  uint8_t o2 = oracle_gf8_mul(a.v[1], b.v[1]);
  return e16_reduce_from(o0, o1, o2);
}
/* galois_16.rs:167-169  Element * u8 */
static elem16 e16_mul_u8(elem16 a, uint8_t r) {
  return e16(oracle_gf8_mul(r, a.v[0]), oracle_gf8_mul(r, a.v[1]));
}
/* galois_16.rs:80-93 */
static elem16 e16_exp(elem16 self, size_t n) {
  if (n == 0) return e16_const(1);
  if (e16_is_zero(self)) return e16(0, 0);
  elem16 x = self;
  for (size_t i = 1; i < n; i++) self = e16_mul(self, x);
  return self;
}

/* galois_16.rs:211-239 div_ext_by: divide EXT_POLY by rhs */
static void e16_div_ext_by(elem16 rhs, elem16 *q, elem16 *r) {
  if (e16_degree(rhs) == 0) {
    *q = e16(0, 0);
    *r = e16(0, 0);
    return;
  }
  uint8_t leading_mul_inv = oracle_gf8_div(1, rhs.v[0]);
  elem16 monictized = e16_mul_u8(rhs, leading_mul_inv);
  uint8_t poly[3] = {EXT_POLY[0], EXT_POLY[1], EXT_POLY[2]};
  for (size_t i = 0; i < 2; i++) {
    uint8_t coef = poly[i];
    for (size_t j = 1; j < 2; j++) {
      if (rhs.v[j] != 0) poly[i + j] ^= oracle_gf8_mul(monictized.v[j], coef);
    }
  }
  *r = e16_const(poly[2]);
  *q = e16_mul_u8(e16(poly[0], poly[1]), leading_mul_inv);
}

/* galois_16.rs:241-282 polynom_div: self / rhs */
static int e16_polynom_div(elem16 self, elem16 rhs, elem16 *q, elem16 *r) {
  size_t divisor_degree = e16_degree(rhs);
  if (e16_is_zero(rhs)) return -1; /* reference panics "divide by 0" */
  if (e16_degree(self) < divisor_degree) {
    *q = e16(0, 0);
    *r = self;
  } else if (divisor_degree == 0) {
    uint8_t invert = oracle_gf8_div(1, rhs.v[1]);
    *q = e16(oracle_gf8_mul(invert, self.v[0]), oracle_gf8_mul(invert, self.v[1]));
    *r = e16(0, 0);
  } else {
    uint8_t leading_mul_inv = oracle_gf8_div(1, rhs.v[0]);
    elem16 monic = e16(oracle_gf8_mul(leading_mul_inv, rhs.v[0]),
                       oracle_gf8_mul(leading_mul_inv, rhs.v[1]));
    uint8_t leading_coeff = self.v[0];
    uint8_t remainder = self.v[1];
    if (monic.v[1] != 0) remainder ^= oracle_gf8_mul(monic.v[1], self.v[0]);
    *q = e16_const(oracle_gf8_mul(leading_mul_inv, leading_coeff));
    *r = e16_const(remainder);
  }
  return 0;
}

/* galois_16.rs:191-208 const_egcd; rhs_is_ext selects EgcdRhs::ExtPoly */
static int e16_const_egcd(elem16 self, int rhs_is_ext, elem16 rhs, uint8_t *g,
                          elem16 *x, elem16 *y) {
  if (e16_is_zero(self)) {
    if (rhs_is_ext) return -1; /* reference panics */
    *g = rhs.v[1];
    *x = e16_const(0);
    *y = e16_const(1);
    return 0;
  }
  elem16 cur_q, cur_r;
  if (rhs_is_ext) {
    e16_div_ext_by(self, &cur_q, &cur_r);
  } else if (e16_polynom_div(rhs, self, &cur_q, &cur_r) != 0) {
    return -1;
  }
  uint8_t gg;
  elem16 xx, yy;
  if (e16_const_egcd(cur_r, 0, self, &gg, &xx, &yy) != 0) return -1;
  *g = gg;
  *x = e16_add(yy, e16_mul(cur_q, xx));
  *y = xx;
  return 0;
}

/* galois_16.rs:285-315 inverse */
static int e16_inverse(elem16 self, elem16 *out) {
  if (e16_is_zero(self)) return -1;
  uint8_t gcd;
  elem16 x, unused;
  if (e16_const_egcd(self, 1, e16(0, 0), &gcd, &x, &unused) != 0) return -1;
  if (gcd == 0) return -1;
  uint8_t normalizer = oracle_gf8_div(1, gcd);
  *out = e16_mul_u8(x, normalizer);
  return 0;
}

void oracle_gf16_add(const uint8_t a[2], const uint8_t b[2], uint8_t out[2]) {
  elem16 r = e16_add(e16(a[0], a[1]), e16(b[0], b[1]));
  out[0] = r.v[0];
  out[1] = r.v[1];
}
void oracle_gf16_mul(const uint8_t a[2], const uint8_t b[2], uint8_t out[2]) {
  elem16 r = e16_mul(e16(a[0], a[1]), e16(b[0], b[1]));
  out[0] = r.v[0];
  out[1] = r.v[1];
}
int oracle_gf16_inverse(const uint8_t a[2], uint8_t out[2]) {
  elem16 r;
  if (e16_inverse(e16(a[0], a[1]), &r) != 0) return -1;
  out[0] = r.v[0];
  out[1] = r.v[1];
  return 0;
}
/* galois_16.rs:175-177 */
int oracle_gf16_div(const uint8_t a[2], const uint8_t b[2], uint8_t out[2]) {
  elem16 inv;
  if (e16_inverse(e16(b[0], b[1]), &inv) != 0) return -1;
  elem16 r = e16_mul(e16(a[0], a[1]), inv);
  out[0] = r.v[0];
  out[1] = r.v[1];
  return 0;
}
void oracle_gf16_exp(const uint8_t a[2], size_t n, uint8_t out[2]) {
  elem16 r = e16_exp(e16(a[0], a[1]), n);
  out[0] = r.v[0];
  out[1] = r.v[1];
}

/* ============ Field dispatch (lib.rs:56-119 trait Field) ================== */
static size_t esize(int field) { return field == 16 ? 2 : 1; }
static size_t field_order(int field) { return field == 16 ? 65536 : 256; }

static void f_zero(int field, uint8_t *o) { memset(o, 0, esize(field)); }
static void f_one(int field, uint8_t *o) {
  if (field == 16) { o[0] = 0; o[1] = 1; } /* galois_16.rs:45-47 */
  else o[0] = 1;
}
static int f_is_zero(int field, const uint8_t *a) {
  return field == 16 ? (a[0] == 0 && a[1] == 0) : a[0] == 0;
}
static int f_eq(int field, const uint8_t *a, const uint8_t *b) {
  return memcmp(a, b, esize(field)) == 0;
}
static void f_add(int field, const uint8_t *a, const uint8_t *b, uint8_t *o) {
  if (field == 16) oracle_gf16_add(a, b, o);
  else o[0] = oracle_gf8_add(a[0], b[0]);
}
static void f_mul(int field, const uint8_t *a, const uint8_t *b, uint8_t *o) {
  if (field == 16) oracle_gf16_mul(a, b, o);
  else o[0] = oracle_gf8_mul(a[0], b[0]);
}
static void f_div(int field, const uint8_t *a, const uint8_t *b, uint8_t *o) {
  if (field == 16) (void)oracle_gf16_div(a, b, o);
  else o[0] = oracle_gf8_div(a[0], b[0]);
}
static void f_exp(int field, const uint8_t *a, size_t n, uint8_t *o) {
  if (field == 16) oracle_gf16_exp(a, n, o);
  else o[0] = oracle_gf8_exp(a[0], n);
}
/* galois_8.rs:37-39 (n as u8), galois_16.rs:49-51 ([n>>8, n&255]) */
static void f_nth(int field, size_t n, uint8_t *o) {
  if (field == 16) { o[0] = (uint8_t)(n >> 8); o[1] = (uint8_t)n; }
  else o[0] = (uint8_t)n;
}

/* ====================== Matrix: matrix.rs =============================== */
#define AT(m, cols, r, c, es) ((m) + (((r) * (cols) + (c)) * (es)))

/* matrix.rs:119-139 */
void oracle_matrix_multiply(int field, const uint8_t *a, size_t ar, size_t ac,
                            const uint8_t *b, size_t bc, uint8_t *out) {
  size_t es = esize(field);
  uint8_t val[2], mul[2];
  for (size_t r = 0; r < ar; r++)
    for (size_t c = 0; c < bc; c++) {
      f_zero(field, val);
      for (size_t i = 0; i < ac; i++) {
        f_mul(field, AT(a, ac, r, i, es), AT(b, bc, i, c, es), mul);
        f_add(field, val, mul, val);
      }
      memcpy(AT(out, bc, r, c, es), val, es);
    }
}

/* matrix.rs:178-189 */
static void swap_rows(uint8_t *m, size_t cols, size_t es, size_t r1, size_t r2) {
  if (r1 == r2) return;
  for (size_t i = 0; i < cols * es; i++) {
    uint8_t t = m[r1 * cols * es + i];
    m[r1 * cols * es + i] = m[r2 * cols * es + i];
    m[r2 * cols * es + i] = t;
  }
}

/* matrix.rs:195-247 gaussian_elim on a rows x cols matrix */
static int gaussian_elim(int field, uint8_t *m, size_t rows, size_t cols) {
  size_t es = esize(field);
  uint8_t one[2], scale[2], tmp[2];
  f_one(field, one);
  for (size_t r = 0; r < rows; r++) {
    if (f_is_zero(field, AT(m, cols, r, r, es))) {
      for (size_t rb = r + 1; rb < rows; rb++) {
        if (!f_is_zero(field, AT(m, cols, rb, r, es))) {
          swap_rows(m, cols, es, r, rb);
          break;
        }
      }
    }
    if (f_is_zero(field, AT(m, cols, r, r, es))) return -1; /* SingularMatrix */
    if (!f_eq(field, AT(m, cols, r, r, es), one)) {
      f_div(field, one, AT(m, cols, r, r, es), scale);
      for (size_t c = 0; c < cols; c++)
        f_mul(field, scale, AT(m, cols, r, c, es), AT(m, cols, r, c, es));
    }
    for (size_t rb = r + 1; rb < rows; rb++) {
      if (!f_is_zero(field, AT(m, cols, rb, r, es))) {
        memcpy(scale, AT(m, cols, rb, r, es), es);
        for (size_t c = 0; c < cols; c++) {
          f_mul(field, scale, AT(m, cols, r, c, es), tmp);
          f_add(field, AT(m, cols, rb, c, es), tmp, AT(m, cols, rb, c, es));
        }
      }
    }
  }
  for (size_t d = 0; d < rows; d++)
    for (size_t ra = 0; ra < d; ra++) {
      if (!f_is_zero(field, AT(m, cols, ra, d, es))) {
        memcpy(scale, AT(m, cols, ra, d, es), es);
        for (size_t c = 0; c < cols; c++) {
          f_mul(field, scale, AT(m, cols, d, c, es), tmp);
          f_add(field, AT(m, cols, ra, c, es), tmp, AT(m, cols, ra, c, es));
        }
      }
    }
  return 0;
}

/* matrix.rs:249-261 invert = augment with identity, eliminate, take right half */
int oracle_matrix_invert(int field, const uint8_t *m, size_t n, uint8_t *out) {
  size_t es = esize(field);
  uint8_t *work = (uint8_t *)calloc(n * 2 * n, es);
  if (!work) return -2;
  for (size_t r = 0; r < n; r++) {
    memcpy(AT(work, 2 * n, r, 0, es), AT(m, n, r, 0, es), n * es);
    f_one(field, AT(work, 2 * n, r, n + r, es));
  }
  int rc = gaussian_elim(field, work, n, 2 * n);
  if (rc == 0)
    for (size_t r = 0; r < n; r++)
      memcpy(AT(out, n, r, 0, es), AT(work, 2 * n, r, n, es), n * es);
  free(work);
  return rc;
}

/* matrix.rs:263-276 */
void oracle_matrix_vandermonde(int field, size_t rows, size_t cols, uint8_t *out) {
  size_t es = esize(field);
  uint8_t ra[2];
  for (size_t r = 0; r < rows; r++) {
    f_nth(field, r, ra);
    for (size_t c = 0; c < cols; c++) f_exp(field, ra, c, AT(out, cols, r, c, es));
  }
}

/* ========================== Codec: core.rs ============================== */
struct oracle_codec {
  int field;
  size_t k, p, total;
  uint8_t *matrix; /* total x k */
};

/* core.rs:430-436 build_matrix */
static int build_matrix(int field, size_t k, size_t total, uint8_t *out) {
  size_t es = esize(field);
  uint8_t *v = (uint8_t *)malloc(total * k * es);
  uint8_t *top = (uint8_t *)malloc(k * k * es);
  uint8_t *inv = (uint8_t *)malloc(k * k * es);
  int rc = -2;
  if (v && top && inv) {
    oracle_matrix_vandermonde(field, total, k, v);
    memcpy(top, v, k * k * es); /* sub_matrix(0,0,k,k): first k rows */
    rc = oracle_matrix_invert(field, top, k, inv);
    if (rc == 0) oracle_matrix_multiply(field, v, total, k, inv, k, out);
  }
  free(v);
  free(top);
  free(inv);
  return rc;
}

/* core.rs:445-467 */
int oracle_codec_new(int field, size_t data_shards, size_t parity_shards,
                     oracle_codec **out) {
  init_tables();
  if (field != 8 && field != 16) return -1;
  if (data_shards == 0) return E_TOO_FEW_DATA_SHARDS;
  if (parity_shards == 0) return E_TOO_FEW_PARITY_SHARDS;
  if (data_shards + parity_shards > field_order(field)) return E_TOO_MANY_SHARDS;
  oracle_codec *c = (oracle_codec *)calloc(1, sizeof *c);
  if (!c) return -2;
  c->field = field;
  c->k = data_shards;
  c->p = parity_shards;
  c->total = data_shards + parity_shards;
  c->matrix = (uint8_t *)malloc(c->total * c->k * esize(field));
  if (!c->matrix || build_matrix(field, c->k, c->total, c->matrix) != 0) {
    free(c->matrix);
    free(c);
    return -2;
  }
  *out = c;
  return E_OK;
}

void oracle_codec_free(oracle_codec *c) {
  if (!c) return;
  free(c->matrix);
  free(c);
}
const uint8_t *oracle_codec_matrix(const oracle_codec *c) { return c->matrix; }
size_t oracle_codec_data_shards(const oracle_codec *c) { return c->k; }
size_t oracle_codec_parity_shards(const oracle_codec *c) { return c->p; }

/* lib.rs:99-118 default mul_slice / mul_slice_add (GF(2^16) uses these) */
static void f_mul_slice(int field, const uint8_t *c, const uint8_t *in,
                        uint8_t *out, size_t n, int add) {
  if (field == 8) {
    if (add) oracle_gf8_mul_slice_xor(c[0], in, out, n);
    else oracle_gf8_mul_slice(c[0], in, out, n);
    return;
  }
  uint8_t t[2];
  for (size_t j = 0; j < n; j++) {
    f_mul(field, c, in + 2 * j, t);
    if (add) f_add(field, out + 2 * j, t, out + 2 * j);
    else memcpy(out + 2 * j, t, 2);
  }
}

/* core.rs:492-509 code_single_slice */
static void code_single_slice(int field, const uint8_t *rows, size_t n_out,
                              size_t n_in, size_t i_input, const uint8_t *input,
                              uint8_t *const *outputs, size_t len) {
  size_t es = esize(field);
  for (size_t r = 0; r < n_out; r++)
    f_mul_slice(field, rows + (r * n_in + i_input) * es, input, outputs[r], len,
                i_input != 0);
}

/* core.rs:481-490 code_some_slices */
void oracle_code_some_slices(int field, const uint8_t *rows, size_t n_out,
                             size_t n_in, const uint8_t *const *inputs,
                             uint8_t *const *outputs, size_t len_elems) {
  init_tables();
  for (size_t i = 0; i < n_in; i++)
    code_single_slice(field, rows, n_out, n_in, i, inputs[i], outputs, len_elems);
}

/* ----- validation macros: macros.rs:142-245 ----- */
static int check_count(size_t got, size_t want, int too_few, int too_many) {
  if (got < want) return too_few;
  if (got > want) return too_many;
  return E_OK;
}
static int check_multi(const size_t *lens, size_t n) { /* macros.rs:144-155 */
  size_t size = lens[0];
  if (size == 0) return E_EMPTY_SHARD;
  for (size_t i = 0; i < n; i++)
    if (lens[i] != size) return E_INCORRECT_SHARD_SIZE;
  return E_OK;
}

static const uint8_t *parity_rows(const oracle_codec *c) {
  return c->matrix + c->k * c->k * esize(c->field); /* core.rs:420-428 */
}

/* core.rs:617-632 */
int oracle_encode_sep(const oracle_codec *c, const uint8_t *const *data,
                      const size_t *data_lens, size_t n_data,
                      uint8_t *const *parity, const size_t *parity_lens,
                      size_t n_parity) {
  int rc;
  if ((rc = check_count(n_data, c->k, E_TOO_FEW_DATA_SHARDS, E_TOO_MANY_DATA_SHARDS))) return rc;
  if ((rc = check_count(n_parity, c->p, E_TOO_FEW_PARITY_SHARDS, E_TOO_MANY_PARITY_SHARDS))) return rc;
  if ((rc = check_multi(data_lens, n_data))) return rc;
  if ((rc = check_multi(parity_lens, n_parity))) return rc;
  if (data_lens[0] != parity_lens[0]) return E_INCORRECT_SHARD_SIZE;
  oracle_code_some_slices(c->field, parity_rows(c), c->p, c->k, data, parity,
                          data_lens[0]);
  return E_OK;
}

/* core.rs:597-611 */
int oracle_encode(const oracle_codec *c, uint8_t *const *shards,
                  const size_t *lens, size_t n) {
  int rc;
  if ((rc = check_count(n, c->total, E_TOO_FEW_SHARDS, E_TOO_MANY_SHARDS))) return rc;
  if ((rc = check_multi(lens, n))) return rc;
  return oracle_encode_sep(c, (const uint8_t *const *)shards, lens, c->k,
                           shards + c->k, lens + c->k, c->p);
}

/* core.rs:576-592 */
int oracle_encode_single_sep(const oracle_codec *c, size_t i_data,
                             const uint8_t *single, size_t single_len,
                             uint8_t *const *parity, const size_t *parity_lens,
                             size_t n_parity) {
  int rc;
  if (i_data >= c->k) return E_INVALID_INDEX;
  if ((rc = check_count(n_parity, c->p, E_TOO_FEW_PARITY_SHARDS, E_TOO_MANY_PARITY_SHARDS))) return rc;
  if ((rc = check_multi(parity_lens, n_parity))) return rc;
  if (parity_lens[0] != single_len) return E_INCORRECT_SHARD_SIZE;
  code_single_slice(c->field, parity_rows(c), c->p, c->k, i_data, single, parity,
                    single_len);
  return E_OK;
}

/* core.rs:545-562 */
int oracle_encode_single(const oracle_codec *c, size_t i_data,
                         uint8_t *const *shards, const size_t *lens, size_t n) {
  int rc;
  if (i_data >= c->k) return E_INVALID_INDEX;
  if ((rc = check_count(n, c->total, E_TOO_FEW_SHARDS, E_TOO_MANY_SHARDS))) return rc;
  if ((rc = check_multi(lens, n))) return rc;
  return oracle_encode_single_sep(c, i_data, shards[i_data], lens[i_data],
                                  shards + c->k, lens + c->k, c->p);
}

/* core.rs:654-669 + check_some_slices_with_buffer core.rs:511-532 */
int oracle_verify_with_buffer(const oracle_codec *c,
                              const uint8_t *const *shards, const size_t *lens,
                              size_t n, uint8_t *const *buffer,
                              const size_t *buf_lens, size_t n_buf, int *ok) {
  int rc;
  if ((rc = check_count(n, c->total, E_TOO_FEW_SHARDS, E_TOO_MANY_SHARDS))) return rc;
  if ((rc = check_count(n_buf, c->p, E_TOO_FEW_BUFFER_SHARDS, E_TOO_MANY_BUFFER_SHARDS))) return rc;
  if ((rc = check_multi(lens, n))) return rc;
  if ((rc = check_multi(buf_lens, n_buf))) return rc;
  if (lens[0] != buf_lens[0]) return E_INCORRECT_SHARD_SIZE;
  size_t len = lens[0], es = esize(c->field);
  oracle_code_some_slices(c->field, parity_rows(c), c->p, c->k, shards, buffer, len);
  int all = 1;
  for (size_t i = 0; i < c->p; i++)
    if (memcmp(buffer[i], shards[c->k + i], len * es) != 0) all = 0;
  *ok = all;
  return E_OK;
}

/* core.rs:637-651 */
int oracle_verify(const oracle_codec *c, const uint8_t *const *shards,
                  const size_t *lens, size_t n, int *ok) {
  int rc;
  if ((rc = check_count(n, c->total, E_TOO_FEW_SHARDS, E_TOO_MANY_SHARDS))) return rc;
  if ((rc = check_multi(lens, n))) return rc;
  size_t len = lens[0], es = esize(c->field);
  uint8_t **buf = (uint8_t **)calloc(c->p, sizeof *buf);
  size_t *bl = (size_t *)calloc(c->p, sizeof *bl);
  for (size_t i = 0; i < c->p; i++) {
    buf[i] = (uint8_t *)calloc(len, es);
    bl[i] = len;
  }
  rc = oracle_verify_with_buffer(c, shards, lens, n, buf, bl, c->p, ok);
  for (size_t i = 0; i < c->p; i++) free(buf[i]);
  free(buf);
  free(bl);
  return rc;
}

/* core.rs:733-923 reconstruct_internal with (T, bool) shards (lib.rs:168-200).
 * The LRU decode-matrix cache (core.rs:697-731) only memoises the inversion;
 * it cannot change results, so the checker recomputes every time. */
int oracle_reconstruct(const oracle_codec *c, uint8_t *const *shards,
                       const size_t *lens, const uint8_t *present, size_t n,
                       int data_only) {
  int rc;
  size_t k = c->k, es = esize(c->field);
  if ((rc = check_count(n, c->total, E_TOO_FEW_SHARDS, E_TOO_MANY_SHARDS))) return rc;

  size_t number_present = 0, shard_len = 0;
  int have_len = 0;
  for (size_t i = 0; i < n; i++) { /* core.rs:747-761 */
    if (present[i]) {
      if (lens[i] == 0) return E_EMPTY_SHARD;
      number_present++;
      if (have_len && lens[i] != shard_len) return E_INCORRECT_SHARD_SIZE;
      shard_len = lens[i];
      have_len = 1;
    }
  }
  if (number_present == c->total) return E_OK; /* core.rs:763-767 */
  if (number_present < k) return E_TOO_FEW_SHARDS_PRESENT; /* :770-772 */

  const uint8_t **sub_shards = (const uint8_t **)calloc(k, sizeof *sub_shards);
  uint8_t **missing_data = (uint8_t **)calloc(c->total, sizeof(uint8_t *));
  uint8_t **missing_parity = (uint8_t **)calloc(c->total, sizeof(uint8_t *));
  size_t *valid = (size_t *)calloc(k, sizeof(size_t));
  size_t *invalid = (size_t *)calloc(c->total, sizeof(size_t));
  uint8_t *sub_matrix = (uint8_t *)calloc(k * k, es);
  uint8_t *decode = (uint8_t *)calloc(k * k, es);
  uint8_t *rows = (uint8_t *)calloc(c->total * k, es);
  const uint8_t **all_data = (const uint8_t **)calloc(k, sizeof(uint8_t *));
  size_t n_sub = 0, n_inv = 0, n_md = 0, n_mp = 0;
  rc = E_OK;

  for (size_t row = 0; row < n; row++) { /* core.rs:801-841 */
    if (row >= k && data_only) {
      if (present[row]) {
        if (n_sub < k) { sub_shards[n_sub] = shards[row]; valid[n_sub++] = row; }
      } else {
        invalid[n_inv++] = row;
      }
      continue;
    }
    /* get_or_initialize, lib.rs:185-199 */
    if (lens[row] != shard_len) { rc = E_INCORRECT_SHARD_SIZE; goto out; }
    if (present[row]) {
      if (n_sub < k) { sub_shards[n_sub] = shards[row]; valid[n_sub++] = row; }
    } else {
      if (row < k) missing_data[n_md++] = shards[row];
      else missing_parity[n_mp++] = shards[row];
      invalid[n_inv++] = row;
    }
  }

  /* core.rs:711-722: sub-matrix of the valid rows, inverted */
  for (size_t r = 0; r < k; r++)
    memcpy(sub_matrix + r * k * es, c->matrix + valid[r] * k * es, k * es);
  if (oracle_matrix_invert(c->field, sub_matrix, k, decode) != 0) { rc = -2; goto out; }

  /* core.rs:850-861: missing data = decode rows x sub_shards */
  {
    size_t nr = 0;
    for (size_t j = 0; j < n_inv && invalid[j] < k; j++, nr++)
      memcpy(rows + nr * k * es, decode + invalid[j] * k * es, k * es);
    oracle_code_some_slices(c->field, rows, nr, k, sub_shards, missing_data, shard_len);
  }
  if (!data_only) { /* core.rs:872-918 */
    size_t nr = 0;
    for (size_t j = 0; j < n_inv; j++) {
      if (invalid[j] < k) continue;
      memcpy(rows + nr * k * es, parity_rows(c) + (invalid[j] - k) * k * es, k * es);
      nr++;
    }
    size_t i_old = 0, i_new = 0, next_maybe_good = 0, na = 0;
    for (size_t j = 0; j < n_inv && invalid[j] < k; j++) {
      for (size_t t = next_maybe_good; t < invalid[j]; t++) all_data[na++] = sub_shards[i_old++];
      next_maybe_good = invalid[j] + 1;
      all_data[na++] = missing_data[i_new++];
    }
    for (size_t t = next_maybe_good; t < k; t++) all_data[na++] = sub_shards[i_old++];
    oracle_code_some_slices(c->field, rows, nr, k, all_data, missing_parity, shard_len);
  }
out:
  free(sub_shards);
  free(missing_data);
  free(missing_parity);
  free(valid);
  free(invalid);
  free(sub_matrix);
  free(decode);
  free(rows);
  free(all_data);
  return rc;
}
