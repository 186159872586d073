// CPU check of the XOR-network generator (rse_netgen.hpp), built and run by
// tests/test_netgen.py: for several codecs, both fields, every budget and both
// factorings, expanding each output plane's sources (temporaries into the
// planes they XOR) must give back the plane's row of the coefficient's bit
// matrix, and the exact factoring must not cost more ops than the greedy.
// Prints one line per case; exits non-zero on the first mismatch.
#include <cstdio>
#include <cstdlib>

#include "rse_netgen.hpp"

using namespace rse;

template <class F>
std::vector<uint16_t> parity(size_t k, size_t p) {  // core.rs:430-436
  auto v = Matrix<F>::vandermonde(k + p, k);
  Matrix<F> top(k, k);
  for (size_t r = 0; r < k; ++r)
    for (size_t c = 0; c < k; ++c) top.at(r, c) = v.at(r, c);
  Matrix<F> inv;
  if (!top.invert(inv)) std::exit(3);
  auto m = v.multiply(inv);
  std::vector<uint16_t> rows;
  for (size_t r = k; r < k + p; ++r)
    for (size_t c = 0; c < k; ++c) rows.push_back(m.at(r, c));
  return rows;
}

// Value (over network input i's plane sources) of source j of input i.
uint64_t source_value(const netgen::Net& net, uint32_t i, int j) {
  if (j < net.nsrc()) return 1ull << j;
  const auto& t = net.tmp[(size_t)i * (net.temps > 0 ? net.temps : 1) + (j - net.nsrc())];
  uint64_t v = source_value(net, i, t[0]) ^ source_value(net, i, t[1]);
  if (t[2] != 255) v ^= source_value(net, i, t[2]);
  return v;
}

int check(int field, uint32_t k, uint32_t p, int budget) {
  const auto rows = field == 16 ? parity<Gf16Field>(k, p) : parity<Gf8Field>(k, p);
  const netgen::Net plain = netgen::build(field, k, p, rows.data(), 0);
  size_t ops[2] = {0, 0};
  for (int exact = 0; exact < 2; ++exact) {
    const netgen::Net net = netgen::build(field, k, p, rows.data(), budget, exact != 0);
    for (uint32_t i = 0; i < k; ++i) {
      if (net.ntmp[i] > net.temps) return 1;
      for (int t = 0; t < net.ntmp[i]; ++t) {  // a temporary uses earlier sources only
        const auto& x = net.tmp[(size_t)i * (net.temps > 0 ? net.temps : 1) + t];
        if (x[0] >= net.np + t || x[1] >= net.np + t || (x[2] != 255 && x[2] >= net.np + t))
          return 2;
      }
      for (uint32_t o = 0; o < p; ++o)
        for (int q = 0; q < net.np; ++q) {
          uint64_t v = 0;
          for (uint64_t m = net.at(o, i, q); m; m &= m - 1) {
            const int j = __builtin_ctzll(m);
            if (j >= net.np + net.ntmp[i]) return 4;
            v ^= source_value(net, i, j);
          }
          if (v != plain.at(o, i, q)) {
            std::printf("MISMATCH field %d %u+%u budget %d exact %d o %u i %u q %d\n", field, k, p,
                        budget, exact, o, i, q);
            return 5;
          }
        }
    }
    ops[exact] = net.ops();
  }
  std::printf("field %d %u+%u budget %d: greedy %zu exact %zu plain %zu\n", field, k, p, budget,
              ops[0], ops[1], plain.ops());
  return ops[1] <= ops[0] ? 0 : 6;
}

// Paired GF(2^8) networks (build_pairs): network input j's rows are inputs 2j
// and 2j + 1's bit-matrix rows side by side (sources 0..7 and 8..15).
int check_pairs(uint32_t k, uint32_t p, int budget) {
  const auto rows = parity<Gf8Field>(k, p);
  const netgen::Net plain = netgen::build(8, k, p, rows.data(), 0);
  const netgen::Net net = netgen::build_pairs(k, p, rows.data(), budget);
  if (!net.pairs || net.ki != (k + 1) / 2) return 11;
  const int ns = net.nsrc();
  for (uint32_t j = 0; j < net.ki; ++j) {
    if (net.ntmp[j] > net.temps) return 12;
    for (int t = 0; t < net.ntmp[j]; ++t) {
      const auto& x = net.tmp[(size_t)j * (net.temps > 0 ? net.temps : 1) + t];
      if (x[0] >= ns + t || x[1] >= ns + t || (x[2] != 255 && x[2] >= ns + t)) return 13;
    }
    for (uint32_t o = 0; o < p; ++o)
      for (int q = 0; q < 8; ++q) {
        uint64_t v = 0;
        for (uint64_t m = net.at(o, j, q); m; m &= m - 1) {
          const int s = __builtin_ctzll(m);
          if (s >= ns + net.ntmp[j]) return 14;
          v ^= source_value(net, j, s);
        }
        uint64_t want = plain.at(o, 2 * j, q);
        if (2 * j + 1 < k) want |= plain.at(o, 2 * j + 1, q) << 8;
        if (v != want) {
          std::printf("MISMATCH pairs %u+%u budget %d o %u j %u q %d\n", k, p, budget, o, j, q);
          return 15;
        }
      }
  }
  const netgen::Net one = netgen::build(8, k, p, rows.data(), budget);
  std::printf("pairs 8 %u+%u budget %d: paired %zu, per input %zu\n", k, p, budget, net.ops(),
              one.ops());
  return 0;
}

int main() {
  const struct { int field; uint32_t k, p; } cases[] = {
      {8, 10, 4}, {8, 12, 8}, {8, 50, 5}, {8, 3, 2}, {16, 20, 8}, {16, 40, 3}, {16, 7, 5}};
  for (const auto& c : cases)
    for (int budget : {0, 4, 16, 32}) {
      const int rc = check(c.field, c.k, c.p, budget);
      if (rc) {
        std::printf("FAIL rc %d field %d %u+%u budget %d\n", rc, c.field, c.k, c.p, budget);
        return rc;
      }
    }
  const struct { uint32_t k, p; } pcases[] = {{50, 5}, {51, 7}, {3, 2}, {1, 4}, {12, 8}};
  for (const auto& c : pcases)
    for (int budget : {0, 4, 16, 32}) {
      const int rc = check_pairs(c.k, c.p, budget);
      if (rc) {
        std::printf("FAIL rc %d pairs %u+%u budget %d\n", rc, c.k, c.p, budget);
        return rc;
      }
    }
  std::printf("OK\n");
  return 0;
}
