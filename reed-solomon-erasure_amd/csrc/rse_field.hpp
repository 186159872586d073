// rse_field.hpp -- host-side field arithmetic and matrix algebra for the codec.
//
// Elements are held as uint16_t: GF(2^8) uses the low byte; GF(2^16) packs the
// reference's [u8;2] = {coefficient of x, constant} (galois_16.rs:49-51) as
// (coef_x << 8) | constant, so nth(n) of both fields is simply n
// (galois_8.rs:37-39, galois_16.rs:49-51).
//
// GF(2^8): polynomial basis modulo x^8+x^4+x^3+x^2+1 (0x11D, build.rs:11), the
// field the reference's LOG/EXP/MUL tables tabulate (build.rs:13-94).
// GF(2^16): GF(2^8)[x] / (x^2 + 2x + 128) (galois_16.rs:9-14).  Every field
// operation has a unique result, so the matrices built here (Vandermonde,
// product, Gauss-Jordan inverse) are byte-identical to matrix.rs:119-276.
#pragma once

#include <stddef.h>
#include <stdint.h>

#include <vector>

namespace rse {

class Gf8 {
 public:
  static uint8_t mul(uint8_t a, uint8_t b) {
    if (a == 0 || b == 0) return 0;
    return t().exp[t().log[a] + t().log[b]];
  }
  static uint8_t inv(uint8_t a) { return t().exp[255 - t().log[a]]; }  // a != 0
  static uint8_t pow(uint8_t a, size_t n) {                            // galois_8.rs:90-103
    if (n == 0) return 1;
    if (a == 0) return 0;
    return t().exp[(size_t)t().log[a] * (n % 255) % 255];
  }

 private:
  struct Tables {
    uint8_t log[256];
    uint8_t exp[512];
    Tables() {
      unsigned b = 1;
      for (unsigned l = 0; l < 255; ++l) {
        log[b] = (uint8_t)l;
        exp[l] = exp[l + 255] = (uint8_t)b;
        b <<= 1;
        if (b & 0x100u) b ^= 0x11Du;
      }
      log[0] = 0;
      exp[510] = exp[511] = 0;
    }
  };
  static const Tables& t() {
    static const Tables tables;
    return tables;
  }
};

// Field policy: F::mul/add/inv/pow/one/order over uint16_t elements.
struct Gf8Field {
  static constexpr int kBits = 8;
  static constexpr size_t kOrder = 256;
  static uint16_t mul(uint16_t a, uint16_t b) { return Gf8::mul((uint8_t)a, (uint8_t)b); }
  static uint16_t inv(uint16_t a) { return Gf8::inv((uint8_t)a); }
  static uint16_t pow(uint16_t a, size_t n) { return Gf8::pow((uint8_t)a, n); }
};

struct Gf16Field {
  static constexpr int kBits = 16;
  static constexpr size_t kOrder = 65536;
  // (a1 x + a0)(b1 x + b0) with x^2 = 2x + 128  (galois_16.rs:146-162, 97-107)
  static uint16_t mul(uint16_t a, uint16_t b) {
    const uint8_t a1 = a >> 8, a0 = a & 0xFF, b1 = b >> 8, b0 = b & 0xFF;
    const uint8_t hh = Gf8::mul(a1, b1);
    const uint8_t x = Gf8::mul(a1, b0) ^ Gf8::mul(a0, b1) ^ Gf8::mul(2, hh);
    const uint8_t c = Gf8::mul(a0, b0) ^ Gf8::mul(128, hh);
    return (uint16_t)((x << 8) | c);
  }
  static uint16_t pow(uint16_t a, size_t n) {  // galois_16.rs:80-93: exp(0,0)=1
    if (n == 0) return 1;
    if (a == 0) return 0;
    n %= 65535;
    if (n == 0) return 1;
    uint16_t r = 1, b = a;
    while (n) {
      if (n & 1) r = mul(r, b);
      b = mul(b, b);
      n >>= 1;
    }
    return r;
  }
  // The reference's extended-Euclid inverse (galois_16.rs:285-315) returns the
  // unique field inverse for every nonzero element (checked exhaustively in
  // tests/test_oracle_golden.py), so a^(2^16 - 2) is identical.
  static uint16_t inv(uint16_t a) { return pow(a, 65534); }
};

// Row-major dense matrix over a field policy F (matrix.rs:33-39).
template <class F>
struct Matrix {
  size_t rows = 0, cols = 0;
  std::vector<uint16_t> d;
  Matrix() = default;
  Matrix(size_t r, size_t c) : rows(r), cols(c), d(r * c, 0) {}
  uint16_t& at(size_t r, size_t c) { return d[r * cols + c]; }
  uint16_t at(size_t r, size_t c) const { return d[r * cols + c]; }

  static Matrix identity(size_t n) {
    Matrix m(n, n);
    for (size_t i = 0; i < n; ++i) m.at(i, i) = 1;
    return m;
  }
  // matrix.rs:263-276: V[r][c] = nth(r)^c
  static Matrix vandermonde(size_t r, size_t c) {
    Matrix m(r, c);
    for (size_t i = 0; i < r; ++i)
      for (size_t j = 0; j < c; ++j) m.at(i, j) = F::pow((uint16_t)i, j);
    return m;
  }
  // matrix.rs:119-139
  Matrix multiply(const Matrix& rhs) const {
    Matrix out(rows, rhs.cols);
    for (size_t r = 0; r < rows; ++r)
      for (size_t c = 0; c < rhs.cols; ++c) {
        uint16_t v = 0;
        for (size_t i = 0; i < cols; ++i) v ^= F::mul(at(r, i), rhs.at(i, c));
        out.at(r, c) = v;
      }
    return out;
  }
  // Gauss-Jordan inverse (matrix.rs:195-261).  Returns false if singular.
  bool invert(Matrix& out) const {
    const size_t n = rows;
    Matrix w(n, 2 * n);
    for (size_t r = 0; r < n; ++r) {
      for (size_t c = 0; c < n; ++c) w.at(r, c) = at(r, c);
      w.at(r, n + r) = 1;
    }
    for (size_t col = 0; col < n; ++col) {
      size_t piv = col;
      while (piv < n && w.at(piv, col) == 0) ++piv;
      if (piv == n) return false;
      if (piv != col)
        for (size_t c = 0; c < 2 * n; ++c) std::swap(w.at(piv, c), w.at(col, c));
      const uint16_t s = F::inv(w.at(col, col));
      for (size_t c = 0; c < 2 * n; ++c) w.at(col, c) = F::mul(s, w.at(col, c));
      for (size_t r = 0; r < n; ++r) {
        const uint16_t f = w.at(r, col);
        if (r == col || f == 0) continue;
        for (size_t c = 0; c < 2 * n; ++c) w.at(r, c) ^= F::mul(f, w.at(col, c));
      }
    }
    out = Matrix(n, n);
    for (size_t r = 0; r < n; ++r)
      for (size_t c = 0; c < n; ++c) out.at(r, c) = w.at(r, n + c);
    return true;
  }
};

}  // namespace rse
