// rse_netgen.hpp -- host-side generator of the bit-sliced XOR networks.
//
// Multiplying by a constant c is GF(2)-linear: an 8x8 (GF(2^8)) or 16x16
// (GF(2^16)) bit matrix.  With the data bit-sliced (rse_bitslice_core.hpp), the
// contribution of input i to output plane q of output o is the XOR of the input
// planes that row q of the bit matrix of coefficient (o, i) selects: the mask
// sel[o][i][q] (bit j = source j).  All outputs' rows of one input draw on the
// same sources, so shared subexpressions are factored out first: temporaries
// t = a ^ b or a ^ b ^ c of the input's sources (one v_bitop3 each, computed
// once per input and chunk) that become new sources.
//
// Cost model: an output plane with w sources costs ceil(w / 2) v_bitop3
// (acc ^ x ^ y), so replacing a pair by a temporary saves one op in exactly
// the rows of odd weight that contain it, and replacing a triple saves one op
// in every row that contains it.  The generator greedily adds the temporary
// with the largest net saving (rows saved - 1 for the temporary), pairs and
// triples alike, until none saves anything or the budget is used.  For
// GF(2^16) 20+8 this takes the network from 5816 v_bitop3 (no temporaries)
// past 4224 (pairs by row count, 16 temporaries; round 1) to 3592 (32).
// The default since is factor8 / factor16 below: the same greedy, but every
// row re-expressed by its exact fewest-source decomposition over the current
// sources (3144 for 20+8).
//
// Used by rse_jit.cpp for the codecs specialised at run time and by
// rse_gen_tables.cpp, at build time, for the codecs compiled into
// rse_bitslice.hip -- one generator, one table format, one set of kernels.
#pragma once

#include <stdint.h>

#include <algorithm>
#include <array>
#include <cstdio>
#include <string>
#include <vector>

#include "rse_field.hpp"

namespace rse {
namespace netgen {

constexpr int kMaxTemps = 32;  // sources per mask: planes (<= 16) + temporaries <= 48 < 64

struct Net {
  int field = 8;
  int np = 8;  // planes per group: 8 (GF(2^8), two groups per 16 dwords) or 16
  uint32_t k = 0, p = 0;
  // paired inputs (GF(2^8) wide modules, build_pairs): network input j is data
  // inputs 2j and 2j + 1, sources 0..7 the planes of the first, 8..15 of the
  // second, so temporaries may combine planes of both; ki = (k + 1) / 2
  bool pairs = false;
  uint32_t ki = 0;                                // network inputs: k, or (k + 1) / 2
  int temps = 0;                                  // budget per network input
  std::vector<uint64_t> sel;                      // [o][ki][q]
  std::vector<uint8_t> ntmp;                      // [ki]
  std::vector<std::array<uint8_t, 3>> tmp;        // [ki][t]: sources {a, b, c}; c = 255: a pair
  int nsrc() const { return pairs ? 16 : np; }    // plane sources per network input
  uint64_t& at(uint32_t o, uint32_t i, int q) { return sel[((size_t)o * ki + i) * np + q]; }
  uint64_t at(uint32_t o, uint32_t i, int q) const { return sel[((size_t)o * ki + i) * np + q]; }
  // v_bitop3 count of one chunk's network (the cost model above)
  size_t ops() const {
    size_t n = 0;
    for (uint32_t i = 0; i < ki; ++i) n += ntmp[i];
    for (uint64_t m : sel) n += ((size_t)__builtin_popcountll(m) + 1) / 2;
    return n;
  }
};

inline int popc(uint64_t m) { return __builtin_popcountll(m); }

// Greedy temporaries over one input's rows (see above); returns the count and
// fills tmp.  planes = the input's own sources (np).
inline int factor(std::vector<uint64_t>& rows, int budget, int planes,
                  std::array<uint8_t, 3>* tmp) {
  int n = 0;
  std::vector<int> c2, c3;
  while (n < budget && n < kMaxTemps) {
    const int ns = planes + n;
    c2.assign((size_t)ns * ns, 0);
    c3.assign((size_t)ns * ns * ns, 0);
    int src[64];
    for (uint64_t r : rows) {
      int w = 0;
      for (uint64_t m = r; m; m &= m - 1) src[w++] = __builtin_ctzll(m);
      for (int x = 0; x < w; ++x)
        for (int y = x + 1; y < w; ++y) {
          if (w & 1) ++c2[(size_t)src[x] * ns + src[y]];
          for (int z = y + 1; z < w; ++z) ++c3[((size_t)src[x] * ns + src[y]) * ns + src[z]];
        }
    }
    int best = 0, ba = -1, bb = -1, bc = -1;
    for (int a = 0; a < ns; ++a)
      for (int b = a + 1; b < ns; ++b) {
        if (c2[(size_t)a * ns + b] - 1 > best) {
          best = c2[(size_t)a * ns + b] - 1;
          ba = a, bb = b, bc = -1;
        }
        for (int c = b + 1; c < ns; ++c)
          if (c3[((size_t)a * ns + b) * ns + c] - 1 > best) {
            best = c3[((size_t)a * ns + b) * ns + c] - 1;
            ba = a, bb = b, bc = c;
          }
      }
    if (best <= 0) break;
    const uint64_t m = (1ull << ba) | (1ull << bb) | (bc >= 0 ? 1ull << bc : 0ull);
    for (uint64_t& r : rows)
      if ((r & m) == m) r = (r & ~m) | (1ull << ns);
    tmp[n] = {(uint8_t)ba, (uint8_t)bb, (uint8_t)(bc >= 0 ? bc : 255)};
    ++n;
  }
  return n;
}

// GF(2^8): exact decompositions.  With 8 planes there are only 256 masks, so
// for a set of sources (planes and temporaries) the fewest sources whose XOR is
// each mask follows from one pass per source, D'[x] = min(D[x], D[x ^ s] + 1),
// and a row costs ceil(D[row] / 2).  The generator greedily adds the temporary
// (any mask one v_bitop3 away: D = 2 or 3) that saves the most, rows re-expressed
// over every source set rather than only where the temporary's bits appear --
// for GF(2^8) 50+20 in 5-output shares 20586 ops per chunk against 23012 for
// factor() above.  rows: masks over the 8 planes in, over the sources out.
inline int factor8(std::vector<uint64_t>& rows, int budget, std::array<uint8_t, 3>* tmp) {
  constexpr int kInf = 1 << 20;
  std::vector<uint32_t> src;                 // source values (8-bit masks)
  std::vector<std::array<int, 256>> stage;   // stage[j][x]: D over the first j sources
  std::array<int, 256> d{};
  d.fill(kInf);
  d[0] = 0;
  stage.push_back(d);
  auto add = [&](uint32_t m) {
    std::array<int, 256> nd;
    for (int x = 0; x < 256; ++x) nd[x] = std::min(d[x], d[x ^ m] + 1);
    d = nd;
    src.push_back(m);
    stage.push_back(d);
  };
  for (int j = 0; j < 8; ++j) add(1u << j);
  // the fewest sources whose XOR is x: bit j = source j
  auto decompose = [&](uint32_t x) {
    uint64_t used = 0;
    for (size_t j = src.size(); j > 0 && x; --j)
      if (stage[j][x] != stage[j - 1][x]) {
        used |= 1ull << (j - 1);
        x ^= src[j - 1];
      }
    return used;
  };
  int count[256] = {};
  for (uint64_t r : rows) ++count[r & 0xFFu];
  auto cost = [&](const std::array<int, 256>& dd) {
    int c = 0;
    for (int x = 1; x < 256; ++x)
      if (count[x]) c += count[x] * ((dd[x] + 1) / 2);
    return c;
  };
  int n = 0, cur = cost(d);
  while (n < budget && n < kMaxTemps) {
    int best = 0;
    uint32_t bm = 0;
    for (uint32_t m = 1; m < 256; ++m) {
      if (d[m] < 2 || d[m] > 3) continue;  // one op from the current sources
      std::array<int, 256> nd;
      for (int x = 0; x < 256; ++x) nd[x] = std::min(d[x], d[x ^ m] + 1);
      const int save = cur - cost(nd) - 1;
      if (save > best) {
        best = save;
        bm = m;
      }
    }
    if (!bm) break;
    const uint64_t parts = decompose(bm);
    int a[3], w = 0;
    for (uint64_t q = parts; q; q &= q - 1) a[w++] = __builtin_ctzll(q);
    tmp[n] = {(uint8_t)a[0], (uint8_t)a[1], (uint8_t)(w == 3 ? a[2] : 255)};
    add(bm);
    cur = cost(d);
    ++n;
  }
  for (uint64_t& r : rows) r = decompose((uint32_t)(r & 0xFFu));
  return n;
}

// GF(2^16): the same with a 65536-entry D.  Candidates are the XORs of two or
// three current sources (one v_bitop3); a row's new cost needs only D[r] and
// D[r ^ m].  A decomposition follows D downhill (a source s with
// D[x ^ s] = D[x] - 1; minimality rules out reusing one).  For GF(2^16) 20+8
// 3144 ops per chunk against 3592 for factor(); 40+12 in 3-output shares
// 10728 against 11806.
inline int factor16(std::vector<uint64_t>& rows, int budget, std::array<uint8_t, 3>* tmp) {
  std::vector<uint8_t> d(65536, 0xFF), nd(65536);
  d[0] = 0;
  std::vector<uint32_t> src;
  auto add = [&](uint32_t m) {
    for (uint32_t x = 0; x < 65536; ++x) {
      const int via = d[x ^ m] == 0xFF ? 0xFF : d[x ^ m] + 1;
      nd[x] = (uint8_t)std::min<int>(d[x], via);
    }
    d.swap(nd);
    src.push_back(m);
  };
  for (int j = 0; j < 16; ++j) add(1u << j);
  auto decompose = [&](uint32_t x) {
    uint64_t used = 0;
    while (x) {
      bool step = false;
      for (size_t j = 0; j < src.size() && !step; ++j)
        if (!((used >> j) & 1u) && d[x ^ src[j]] + 1 == d[x]) {
          used |= 1ull << j;
          x ^= src[j];
          step = true;
        }
      if (!step) break;  // cannot happen: d is exact
    }
    return used;
  };
  std::vector<std::pair<uint32_t, int>> rc;  // distinct rows and their counts
  {
    std::vector<uint32_t> v;
    for (uint64_t r : rows) v.push_back((uint32_t)(r & 0xFFFFu));
    std::sort(v.begin(), v.end());
    for (size_t i = 0; i < v.size();) {
      size_t j = i;
      while (j < v.size() && v[j] == v[i]) ++j;
      if (v[i]) rc.push_back({v[i], (int)(j - i)});
      i = j;
    }
  }
  auto cost_with = [&](uint32_t m) {
    int c = 0;
    for (const auto& [r, n] : rc) c += n * ((std::min<int>(d[r], d[r ^ m] + 1) + 1) / 2);
    return c;
  };
  int n = 0, cur = cost_with(0);
  while (n < budget && n < kMaxTemps) {
    int best = 0;
    uint32_t bm = 0;
    const size_t ns = src.size();
    auto eval = [&](uint32_t m) {
      if (d[m] < 2) return;  // zero or already a source
      const int save = cur - cost_with(m) - 1;
      if (save > best) {
        best = save;
        bm = m;
      }
    };
    for (size_t a = 0; a < ns; ++a)
      for (size_t b = a + 1; b < ns; ++b) {
        eval(src[a] ^ src[b]);
        for (size_t c = b + 1; c < ns; ++c) eval(src[a] ^ src[b] ^ src[c]);
      }
    if (!bm) break;
    const uint64_t parts = decompose(bm);
    int a[3], w = 0;
    for (uint64_t q = parts; q && w < 3; q &= q - 1) a[w++] = __builtin_ctzll(q);
    tmp[n] = {(uint8_t)a[0], (uint8_t)a[1], (uint8_t)(w == 3 ? a[2] : 255)};
    add(bm);
    cur = cost_with(0);
    ++n;
  }
  for (uint64_t& r : rows) r = decompose((uint32_t)(r & 0xFFFFu));
  return n;
}

// The network of p x k rows (row-major, uint16 elements as in rse_field.hpp).
// budget: temporaries per input (GF(2^8): per input, shared by its two plane
// groups, which use the same bit matrices).  exact: per input, the cheaper of
// factor8 / factor16 and factor (default); otherwise factor alone (A/B).
inline Net build(int field, uint32_t k, uint32_t p, const uint16_t* rows, int budget,
                 bool exact = true) {
  Net net;
  net.field = field;
  net.np = field == 16 ? 16 : 8;
  net.k = k;
  net.ki = k;
  net.p = p;
  net.temps = budget < 0 ? 0 : budget > kMaxTemps ? kMaxTemps : budget;
  net.sel.assign((size_t)p * k * net.np, 0);
  net.ntmp.assign(k, 0);
  net.tmp.assign((size_t)k * (net.temps > 0 ? net.temps : 1), {0, 0, 255});
  const int np = net.np;
  // GF(2^16) plane q < 8 is bit q of the coefficient-of-x byte (uint16 bit
  // q + 8), q >= 8 bit q - 8 of the constant byte (rse_bitslice_core.hpp BitsF16)
  auto bit = [&](int q) { return field == 16 ? (q ^ 8) : q; };
  auto mul = [&](uint16_t a, uint16_t b) {
    return field == 16 ? Gf16Field::mul(a, b) : Gf8Field::mul(a, b);
  };
  for (uint32_t o = 0; o < p; ++o)
    for (uint32_t i = 0; i < k; ++i)
      for (int j = 0; j < np; ++j) {
        const uint16_t col = mul(rows[(size_t)o * k + i], (uint16_t)(1u << bit(j)));
        for (int q = 0; q < np; ++q)
          if ((col >> bit(q)) & 1u) net.at(o, i, q) |= 1ull << j;
      }
  if (net.temps > 0)
    for (uint32_t i = 0; i < k; ++i) {
      std::vector<uint64_t> r;
      for (uint32_t o = 0; o < p; ++o)
        for (int q = 0; q < np; ++q) r.push_back(net.at(o, i, q));
      std::array<uint8_t, 3>* t = &net.tmp[(size_t)i * net.temps];
      net.ntmp[i] = (uint8_t)factor(r, net.temps, np, t);
      if (exact) {  // the exact factoring, unless the greedy did better on this input
        std::vector<uint64_t> r2;
        for (uint32_t o = 0; o < p; ++o)
          for (int q = 0; q < np; ++q) r2.push_back(net.at(o, i, q));
        std::vector<std::array<uint8_t, 3>> t2((size_t)net.temps);
        const int n2 = field == 8 ? factor8(r2, net.temps, t2.data())
                                  : factor16(r2, net.temps, t2.data());
        auto cost = [](const std::vector<uint64_t>& v, int n) {
          size_t c = (size_t)n;
          for (uint64_t m : v) c += ((size_t)__builtin_popcountll(m) + 1) / 2;
          return c;
        };
        if (cost(r2, n2) <= cost(r, net.ntmp[i])) {
          r.swap(r2);
          for (int x = 0; x < n2; ++x) t[x] = t2[(size_t)x];
          net.ntmp[i] = (uint8_t)n2;
        }
      }
      size_t n = 0;
      for (uint32_t o = 0; o < p; ++o)
        for (int q = 0; q < np; ++q) net.at(o, i, q) = r[n++];
    }
  return net;
}

// The GF(2^8) network of p x k rows over PAIRS of inputs (Net::pairs): the
// rows of network input j are the two inputs' bit-matrix rows side by side (16
// sources), factored like a GF(2^16) input (factor16, or the greedy if that is
// cheaper), so a temporary can serve both inputs' terms of a row.  The wide
// kernels code a round's inputs two at a time (rse_bitslice_core.hpp
// wide_code_round).  50+20 in 4 output shares: 10293 -> ~8800 ops per plane
// group at 32 temporaries (tools: offline count).
inline Net build_pairs(uint32_t k, uint32_t p, const uint16_t* rows, int budget) {
  const Net plain = build(8, k, p, rows, 0, false);
  Net net;
  net.field = 8;
  net.np = 8;
  net.k = k;
  net.p = p;
  net.pairs = true;
  net.ki = (k + 1) / 2;
  net.temps = budget < 0 ? 0 : budget > kMaxTemps ? kMaxTemps : budget;
  const int nt = net.temps > 0 ? net.temps : 1;
  net.sel.assign((size_t)p * net.ki * 8, 0);
  net.ntmp.assign(net.ki, 0);
  net.tmp.assign((size_t)net.ki * nt, {0, 0, 255});
  for (uint32_t j = 0; j < net.ki; ++j) {
    std::vector<uint64_t> r;
    for (uint32_t o = 0; o < p; ++o)
      for (int q = 0; q < 8; ++q) {
        uint64_t m = plain.at(o, 2 * j, q);
        if (2 * j + 1 < k) m |= plain.at(o, 2 * j + 1, q) << 8;
        r.push_back(m);
      }
    std::array<uint8_t, 3>* t = &net.tmp[(size_t)j * nt];
    if (net.temps > 0) {
      std::vector<uint64_t> r2 = r;
      net.ntmp[j] = (uint8_t)factor(r, net.temps, 16, t);
      std::vector<std::array<uint8_t, 3>> t2((size_t)net.temps);
      const int n2 = factor16(r2, net.temps, t2.data());
      auto cost = [](const std::vector<uint64_t>& v, int n) {
        size_t c = (size_t)n;
        for (uint64_t m : v) c += ((size_t)__builtin_popcountll(m) + 1) / 2;
        return c;
      };
      if (cost(r2, n2) <= cost(r, net.ntmp[j])) {
        r.swap(r2);
        for (int x = 0; x < n2; ++x) t[x] = t2[(size_t)x];
        net.ntmp[j] = (uint8_t)n2;
      }
    }
    size_t n = 0;
    for (uint32_t o = 0; o < p; ++o)
      for (int q = 0; q < 8; ++q) net.at(o, j, q) = r[n++];
  }
  return net;
}

// C++ source of code struct `name` for rse_bitslice_core.hpp:
//   using Field; k, p, NP, NG, kTemps (GF(2^16) per-input temporaries),
//   kGTemps (GF(2^8) per-group temporaries); planes.sel / ntmp / tmp; rows.
inline std::string emit(const Net& net, const char* name, const uint16_t* rows) {
  std::string s;
  const int nt = net.temps > 0 ? net.temps : 1;
  char buf[768];
  std::snprintf(buf, sizeof buf,
                "struct %sPlanes {\n  uint64_t sel[%u][%u][%d];\n  uint8_t ntmp[%u];\n"
                "  uint8_t tmp[%u][%d][3];\n};\n"
                "struct %s {\n  using Field = %s;\n"
                "  static constexpr int k = %u, p = %u, NP = %d, NG = %d, kTemps = %d, "
                "kGTemps = %d, kPairIn = %d;\n"
                "  static constexpr uint16_t rows[%u][%u] = {",
                name, net.p, net.ki, net.np, net.ki, net.ki, nt, name,
                net.field == 16 ? "BitsF16" : "BitsF8", net.k, net.p, net.np, 16 / net.np,
                net.field == 16 ? net.temps : 0, net.field == 16 ? 0 : net.temps,
                net.pairs ? 1 : 0, net.p, net.k);
  s += buf;
  for (uint32_t o = 0; o < net.p; ++o) {
    s += "{";
    for (uint32_t i = 0; i < net.k; ++i) {
      std::snprintf(buf, sizeof buf, "%u,", (unsigned)rows[(size_t)o * net.k + i]);
      s += buf;
    }
    s += "},";
  }
  std::snprintf(buf, sizeof buf, "};\n  static constexpr %sPlanes planes = {{", name);
  s += buf;
  for (uint32_t o = 0; o < net.p; ++o) {
    s += "{";
    for (uint32_t i = 0; i < net.ki; ++i) {
      s += "{";
      for (int q = 0; q < net.np; ++q) {
        std::snprintf(buf, sizeof buf, "%lluull,", (unsigned long long)net.at(o, i, q));
        s += buf;
      }
      s += "},";
    }
    s += "},";
  }
  s += "}, {";
  for (uint32_t i = 0; i < net.ki; ++i) {
    std::snprintf(buf, sizeof buf, "%d,", net.ntmp[i]);
    s += buf;
  }
  s += "}, {";
  for (uint32_t i = 0; i < net.ki; ++i) {
    s += "{";
    for (int t = 0; t < nt; ++t) {
      const auto& x = net.tmp[(size_t)i * nt + t];
      std::snprintf(buf, sizeof buf, "{%d,%d,%d},", x[0], x[1], x[2]);
      s += buf;
    }
    s += "},";
  }
  s += "}};\n};\n";
  return s;
}

}  // namespace netgen
}  // namespace rse
