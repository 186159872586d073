// rse_bitslice.hip -- bit-sliced GF(2^16) encode/verify kernels for codecs
// whose parity matrix is known at compile time.
//
// Why: the table kernels in rse_kernels.hip spend 4 GF(2^8) constant
// multiplies (3 v_perm_b32 each) per GF(2^16) coefficient and dword, which
// makes GF(2^16) VALU-bound far below HBM speed.  Multiplication by a constant
// c is a GF(2)-linear map on the 16 bits of an element: a 16x16 bit matrix.
// With the data bit-sliced -- register q holds bit q of 32 elements -- a
// multiply-accumulate is just the XOR of the input planes selected by each row
// of that bit matrix, ~64 v_bitop3_b32 (3-input XOR) per 32 elements instead
// of ~96 v_perm + ~64 XOR.  The encoding matrix of ReedSolomon::new (core.rs:
// 430-436, V * (V_top)^-1 over galois_16) depends only on (k, p), so for the
// configurations instantiated here its parity rows, and the bit matrices of
// every coefficient, are evaluated by constexpr code and the XOR network is
// straight-line code with no tables and no memory other than the shards.  The
// host checks that a launch's coefficients equal the compiled ones before
// dispatching here (anything else takes the table kernels), so a matrix
// mismatch can only cost speed, never correctness.
//
// Lane layout: a workgroup of 256 lanes codes a 16 KiB chunk of every shard.
// Lane t loads the 16-byte vectors t, t+256, t+512, t+768 of the chunk (each
// load instruction is 4 KiB contiguous per workgroup), i.e. 16 dwords = 32
// GF(2^16) elements.  In registers they are split into x-coefficient and
// constant byte planes with v_perm (H = byte 0, L = byte 1 of every element,
// galois_16.rs:49-51) and each plane is 8x8-bit transposed within byte lanes:
// afterwards plane q < 8 holds bit q of the H bytes, plane 8 + q bit q of the
// L bytes.  Outputs are transposed back the same way (the network is an
// involution) and merged.  Any element order works as long as input and output
// use the same one; this one keeps every global access coalesced.
#include <utility>

#include "rse_device.hpp"

namespace rse {
namespace {

constexpr int kBsBlock = 256;
constexpr uint64_t kBsChunk = 16384;  // bytes of one shard per workgroup step
constexpr int kBsDefaultVariant = 1;  // bitslice_kernel variant (tools/tune.py sweeps)

// ----------------------------------------------------------- constexpr GF
// GF(2^8), generating polynomial 0x11D (build.rs:11), log/exp built the way
// build.rs:27-48 does; GF(2^16) per galois_16.rs:146-162 (x^2 = 2x + 128).
struct Gf8Tables {
  uint8_t log[256] = {};
  uint8_t exp[512] = {};
  constexpr Gf8Tables() {
    uint32_t b = 1;
    for (int l = 0; l < 255; ++l) {
      log[b] = (uint8_t)l;
      exp[l] = exp[l + 255] = (uint8_t)b;
      b <<= 1;
      if (b & 0x100u) b ^= 0x11Du;
    }
  }
};
constexpr Gf8Tables kGf8{};

constexpr uint8_t cmul8(uint8_t a, uint8_t b) {
  return (a && b) ? kGf8.exp[kGf8.log[a] + kGf8.log[b]] : 0;
}
constexpr uint16_t cmul16(uint16_t a, uint16_t b) {
  const uint8_t a1 = a >> 8, a0 = a & 0xFF, b1 = b >> 8, b0 = b & 0xFF;
  const uint8_t hh = cmul8(a1, b1);
  const uint8_t x = cmul8(a1, b0) ^ cmul8(a0, b1) ^ cmul8(2, hh);
  const uint8_t c = cmul8(a0, b0) ^ cmul8(128, hh);
  return (uint16_t)((x << 8) | c);
}
constexpr uint16_t cpow16(uint16_t a, uint32_t n) {  // galois_16.rs:80-93
  if (n == 0) return 1;
  if (a == 0) return 0;
  n %= 65535u;
  if (n == 0) return 1;
  uint16_t r = 1, b = a;
  while (n) {
    if (n & 1) r = cmul16(r, b);
    b = cmul16(b, b);
    n >>= 1;
  }
  return r;
}
constexpr uint16_t cinv16(uint16_t a) { return cpow16(a, 65534u); }

constexpr uint8_t cexp8(uint8_t a, uint32_t n) {  // galois_8.rs:87-103
  if (n == 0) return 1;
  if (a == 0) return 0;
  return kGf8.exp[(kGf8.log[a] * n) % 255];
}

// Field policies for the constexpr matrix code.
struct CF8 {
  static constexpr int kPlanes = 8;
  static constexpr uint16_t mul(uint16_t a, uint16_t b) { return cmul8((uint8_t)a, (uint8_t)b); }
  static constexpr uint16_t pow(uint16_t a, uint32_t n) { return cexp8((uint8_t)a, n); }
  static constexpr uint16_t inv(uint16_t a) { return kGf8.exp[255 - kGf8.log[a]]; }
  // plane q = bit q of the byte
  static constexpr int bit(int q) { return q; }
};
struct CF16 {
  static constexpr int kPlanes = 16;
  static constexpr uint16_t mul(uint16_t a, uint16_t b) { return cmul16(a, b); }
  static constexpr uint16_t pow(uint16_t a, uint32_t n) { return cpow16(a, n); }
  static constexpr uint16_t inv(uint16_t a) { return cinv16(a); }
  // plane q < 8: bit q of the H (x-coefficient) byte = uint16 bit q + 8;
  // plane q >= 8: bit q - 8 of the L byte = uint16 bit q - 8
  static constexpr int bit(int q) { return q ^ 8; }
};

// Parity rows of the (K + P) x K encoding matrix V * (V[0..K])^-1 with
// V[r][c] = r^c (matrix.rs:263-276, core.rs:430-436).  The inverse is unique,
// so Gauss-Jordan here gives the same matrix as matrix.rs:195-261.
template <class F, int K, int P>
struct Parity {
  uint16_t m[P][K] = {};
  constexpr Parity() {
    uint16_t w[K][2 * K] = {};
    for (int r = 0; r < K; ++r) {
      for (int c = 0; c < K; ++c) w[r][c] = F::pow((uint16_t)r, (uint32_t)c);
      w[r][K + r] = 1;
    }
    for (int col = 0; col < K; ++col) {
      int piv = col;
      while (w[piv][col] == 0) ++piv;
      if (piv != col)
        for (int c = 0; c < 2 * K; ++c) {
          const uint16_t t = w[col][c];
          w[col][c] = w[piv][c];
          w[piv][c] = t;
        }
      const uint16_t s = F::inv(w[col][col]);
      for (int c = 0; c < 2 * K; ++c) w[col][c] = F::mul(s, w[col][c]);
      for (int r = 0; r < K; ++r) {
        const uint16_t f = w[r][col];
        if (r == col || f == 0) continue;
        for (int c = 0; c < 2 * K; ++c) w[r][c] ^= F::mul(f, w[col][c]);
      }
    }
    for (int o = 0; o < P; ++o)
      for (int i = 0; i < K; ++i) {
        uint16_t v = 0;
        for (int j = 0; j < K; ++j) v ^= F::mul(F::pow((uint16_t)(K + o), (uint32_t)j), w[j][K + i]);
        m[o][i] = v;
      }
  }
};

// sel[o][i][p] = the input planes whose XOR is output plane p of the product
// by coefficient (o, i): column q of the bit matrix is c * (element with only
// plane q's bit set).
template <class F, int K, int P>
struct Planes {
  Parity<F, K, P> par{};
  uint16_t sel[P][K][F::kPlanes] = {};
  constexpr Planes() {
    for (int o = 0; o < P; ++o)
      for (int i = 0; i < K; ++i)
        for (int q = 0; q < F::kPlanes; ++q) {
          const uint16_t col = F::mul(par.m[o][i], (uint16_t)(1u << F::bit(q)));
          for (int p = 0; p < F::kPlanes; ++p)
            if ((col >> F::bit(p)) & 1u) sel[o][i][p] |= (uint16_t)(1u << q);
        }
  }
};

// A compiled codec: NP planes per group, NG groups per lane-chunk (16 dwords).
template <class F, int K, int P>
struct Code {
  using Field = F;
  static constexpr int k = K, p = P;
  static constexpr int NP = F::kPlanes, NG = 16 / F::kPlanes;
  static constexpr Planes<F, K, P> planes{};
};

// ------------------------------------------------------------ bit slicing
// XOR of acc and the planes selected by M, two at a time.
template <uint32_t M>
__device__ __forceinline__ uint32_t xacc(uint32_t acc, const uint32_t* in) {
  if constexpr (M == 0) {
    return acc;
  } else {
    constexpr int q0 = __builtin_ctz(M);
    constexpr uint32_t m1 = M & (M - 1);
    if constexpr (m1 == 0) {
      return acc ^ in[q0];
    } else {
      constexpr int q1 = __builtin_ctz(m1);
      return xacc<m1 & (m1 - 1)>(xor3(acc, in[q0], in[q1]), in);
    }
  }
}
template <uint32_t M>
__device__ __forceinline__ uint32_t xinit(const uint32_t* in) {
  if constexpr (M == 0) {
    return 0u;
  } else {
    constexpr int q0 = __builtin_ctz(M);
    return xacc<M & (M - 1)>(in[q0], in);
  }
}

// 8x8 bit transpose inside every byte lane of h[0..7] (an involution): bit b
// of byte lane L of h[i] moves to bit i of byte lane L of h[b].
__device__ __forceinline__ void transpose8(uint32_t* h) {
#pragma unroll
  for (int s = 4, st = 0; st < 3; s >>= 1, ++st) {
    const uint32_t m = s == 4 ? 0x0F0F0F0Fu : s == 2 ? 0x33333333u : 0x55555555u;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      if (i & s) continue;
      const uint32_t a = h[i], b = h[i + s];
      h[i] = (a & ~(m << s)) | ((b & m) << s);
      h[i + s] = (b & ~m) | ((a >> s) & m);
    }
  }
}

// 4 vectors (16 dwords) -> NG groups of NP planes.
//  GF(2^16): 32 elements; split into H/L byte planes (v_perm), then 8x8
//            transposes: pl[q] = bit q of H, pl[8 + q] = bit q of L.
//  GF(2^8):  64 bytes as two groups of 8 dwords (vectors 0-1, 2-3), each
//            8x8-transposed: pl[8g + q] = bit q of group g's 32 bytes.
template <class F>
__device__ __forceinline__ void slice(const u32x4 (&v)[4], uint32_t (&pl)[16]) {
  if constexpr (F::kPlanes == 16) {
#pragma unroll
    for (int m = 0; m < 8; ++m) {
      const uint32_t x0 = v[m >> 1][(m & 1) * 2], x1 = v[m >> 1][(m & 1) * 2 + 1];
      pl[m] = __builtin_amdgcn_perm(x1, x0, 0x06040200u);      // H bytes
      pl[8 + m] = __builtin_amdgcn_perm(x1, x0, 0x07050301u);  // L bytes
    }
  } else {
#pragma unroll
    for (int d = 0; d < 16; ++d) pl[d] = v[d >> 2][d & 3];
  }
  transpose8(pl);
  transpose8(pl + 8);
}

// Inverse of slice (clobbers pl).
template <class F>
__device__ __forceinline__ void unslice(uint32_t (&pl)[16], u32x4 (&v)[4]) {
  transpose8(pl);
  transpose8(pl + 8);
  if constexpr (F::kPlanes == 16) {
#pragma unroll
    for (int m = 0; m < 8; ++m) {
      v[m >> 1][(m & 1) * 2] = __builtin_amdgcn_perm(pl[8 + m], pl[m], 0x05010400u);
      v[m >> 1][(m & 1) * 2 + 1] = __builtin_amdgcn_perm(pl[8 + m], pl[m], 0x07030602u);
    }
  } else {
#pragma unroll
    for (int d = 0; d < 16; ++d) v[d >> 2][d & 3] = pl[d];
  }
}

template <bool NT>
__device__ __forceinline__ u32x4 ldv(const uint8_t* p) {
  const u32x4* q = reinterpret_cast<const u32x4*>(p);
  if constexpr (NT) return __builtin_nontemporal_load(q);
  else return *q;
}
template <bool NT>
__device__ __forceinline__ void stv(uint8_t* p, u32x4 v) {
  u32x4* q = reinterpret_cast<u32x4*>(p);
  if constexpr (NT) __builtin_nontemporal_store(v, q);
  else *q = v;
}

template <bool NT>
__device__ __forceinline__ void load4(u32x4 (&v)[4], const uint8_t* p) {
#pragma unroll
  for (int j = 0; j < 4; ++j) v[j] = ldv<NT>(p + j * (kBsBlock * 16));
}

// acc[o*16 + g*NP + p] (^)= plane combination of group g of input I, for
// every output o, group g and plane p.
template <class C, int I, int N, int... OP>
__device__ __forceinline__ void mac_input(uint32_t (&acc)[N], const uint32_t (&in)[16],
                                          std::integer_sequence<int, OP...>) {
  if constexpr (I == 0)
    ((acc[OP] = xinit<C::planes.sel[OP / 16][I][OP % C::NP]>(in + (OP % 16) / C::NP * C::NP)),
     ...);
  else
    ((acc[OP] = xacc<C::planes.sel[OP / 16][I][OP % C::NP]>(acc[OP],
                                                              in + (OP % 16) / C::NP * C::NP)),
     ...);
}

// Output phase of one chunk: un-slice every output's planes and store them
// (kStore), compare them with the stored parity (kCheck), or both.
template <class C, bool NT>
__device__ __forceinline__ void store_outputs(uint32_t (&acc)[C::p * 16], const CodeArgs& a,
                                              uint64_t off, uint32_t mode, bool& diff) {
#pragma unroll
  for (int o = 0; o < C::p; ++o) {
    uint32_t pl[16];
#pragma unroll
    for (int q = 0; q < 16; ++q) pl[q] = acc[o * 16 + q];
    u32x4 v[4];
    unslice<typename C::Field>(pl, v);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const uint64_t o16 = off + j * (kBsBlock * 16);
      if (mode != kCheck) stv<NT>(a.out[o] + o16, v[j]);
      if (mode != kStore) {
        const u32x4 w = ldv<NT>(a.cmp[o] + o16);
        diff |= (w.x != v[j].x) | (w.y != v[j].y) | (w.z != v[j].z) | (w.w != v[j].w);
      }
    }
  }
}

// Inputs I.. of one chunk: the loads of input I + 1 are issued before input
// I is coded, so one input's worth of vectors is always in flight.
//  SB: a scheduling barrier keeps those loads ahead of input I's XOR network;
//      without it the scheduler sinks them next to their first use (register
//      pressure heuristics), which serialises HBM latency and compute.
//  XC: the last input prefetches input 0 of the workgroup's next chunk
//      (next_off, ~0 if none) into cur, so the output phase overlaps it too.
template <class C, bool NT, bool SB, bool XC, int I>
__device__ __forceinline__ void code_inputs(uint32_t (&acc)[C::p * 16], u32x4 (&cur)[4],
                                            const CodeArgs& a, uint64_t off, uint64_t next_off) {
  u32x4 nxt[4];
  if constexpr (I + 1 < C::k) {
    load4<NT>(nxt, a.in[I + 1] + off);
  } else if constexpr (XC) {
    if (next_off != ~0ull) load4<NT>(nxt, a.in[0] + next_off);
  }
  if constexpr (SB) __builtin_amdgcn_sched_barrier(0);
  uint32_t pl[16];
  slice<typename C::Field>(cur, pl);
  mac_input<C, I>(acc, pl, std::make_integer_sequence<int, C::p * 16>{});
  // keep each input's XORs together: without this the compiler reassociates
  // across inputs and keeps several inputs' planes live (spills)
#pragma unroll
  for (int q = 0; q < C::p * 16; ++q) asm volatile("" : "+v"(acc[q]));
  if constexpr (I + 1 < C::k) {
#pragma unroll
    for (int j = 0; j < 4; ++j) cur[j] = nxt[j];
    code_inputs<C, NT, SB, XC, I + 1>(acc, cur, a, off, next_off);
  } else if constexpr (XC) {
    if (next_off != ~0ull) {
#pragma unroll
      for (int j = 0; j < 4; ++j) cur[j] = nxt[j];
    }
  }
}

// One workgroup step = one 16 KiB chunk of one stripe; chunks of all stripes
// are one flat index space walked grid-stride.  a.n_vec counts whole chunks'
// vectors only (the host codes the remainder with the table kernels).
template <class C, bool NT, bool SB, bool XC>
__global__ __launch_bounds__(kBsBlock, C::p > 4 ? 2 : 3) void bitslice_kernel(
    const CodeArgs a, uint64_t chunks_per_stripe) {
  const uint64_t total = chunks_per_stripe * a.n_stripes;
  const uint32_t mode = a.mode;
  bool diff = false;
  auto chunk_off = [&](uint64_t idx) {
    const uint64_t stripe = idx / chunks_per_stripe, chunk = idx - stripe * chunks_per_stripe;
    return stripe * a.stripe_stride + chunk * kBsChunk + threadIdx.x * 16u;
  };
  u32x4 cur[4];
  if (XC && blockIdx.x < total) load4<NT>(cur, a.in[0] + chunk_off(blockIdx.x));
  for (uint64_t idx = blockIdx.x; idx < total; idx += gridDim.x) {
    const uint64_t off = chunk_off(idx);
    const uint64_t nidx = idx + gridDim.x;
    const uint64_t next_off = (XC && nidx < total) ? chunk_off(nidx) : ~0ull;
    uint32_t acc[C::p * 16];
    if (!XC) load4<NT>(cur, a.in[0] + off);
    code_inputs<C, NT, SB, XC, 0>(acc, cur, a, off, next_off);
    store_outputs<C, NT>(acc, a, off, mode, diff);
  }
  if (mode != kStore && diff) atomicOr(a.mismatch, 1u);
}

// ----------------------------------------------- LDS-DMA input ring variant
// The same kernel with the shard loads issued as global_load_lds_dwordx4
// (LDS-DMA, no VGPR destination) into a per-wave ring of D input slots, D - 1
// inputs ahead, across chunk boundaries.  Register-safe by construction: hipcc
// never sees a VGPR written by an in-flight load.  Completion is counted by
// hand (MI355X_MICROARCH.md: vmcnt counts loads, stores and LDS-DMA together,
// in issue order): waiting for step g's DMA leaves the DMAs of the steps
// issued after it plus, right after a chunk boundary, the previous chunk's
// output-phase operations (S per chunk) outstanding.

// s_waitcnt vmcnt(n), n a run-time value (wave-uniform) clamped to 63.
__device__ __forceinline__ void wait_vmcnt(uint32_t n) {
  switch (n > 63u ? 63u : n) {
#define RSE_W(N) \
  case N: asm volatile("s_waitcnt vmcnt(" #N ")" ::: "memory"); break;
    RSE_W(0) RSE_W(1) RSE_W(2) RSE_W(3) RSE_W(4) RSE_W(5) RSE_W(6) RSE_W(7) RSE_W(8) RSE_W(9)
    RSE_W(10) RSE_W(11) RSE_W(12) RSE_W(13) RSE_W(14) RSE_W(15) RSE_W(16) RSE_W(17) RSE_W(18)
    RSE_W(19) RSE_W(20) RSE_W(21) RSE_W(22) RSE_W(23) RSE_W(24) RSE_W(25) RSE_W(26) RSE_W(27)
    RSE_W(28) RSE_W(29) RSE_W(30) RSE_W(31) RSE_W(32) RSE_W(33) RSE_W(34) RSE_W(35) RSE_W(36)
    RSE_W(37) RSE_W(38) RSE_W(39) RSE_W(40) RSE_W(41) RSE_W(42) RSE_W(43) RSE_W(44) RSE_W(45)
    RSE_W(46) RSE_W(47) RSE_W(48) RSE_W(49) RSE_W(50) RSE_W(51) RSE_W(52) RSE_W(53) RSE_W(54)
    RSE_W(55) RSE_W(56) RSE_W(57) RSE_W(58) RSE_W(59) RSE_W(60) RSE_W(61) RSE_W(62)
    default: asm volatile("s_waitcnt vmcnt(63)" ::: "memory"); break;
#undef RSE_W
  }
}

// One 16-byte LDS-DMA per lane: LDS[lds + lane * 16] = *g (non-temporal).
// M0 is saved and restored in the same statement (guide §5.7).
__device__ __forceinline__ void dma16(const uint8_t* g, uint32_t lds) {
  uint32_t keep;
  asm volatile(
      "s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\t"
      "global_load_lds_dwordx4 %1, off nt\n\ts_mov_b32 m0, %0"
      : "=&s"(keep)
      : "v"(g), "s"(lds)
      : "memory");
}

template <class C, int D>
struct DmaRing {
  const CodeArgs& a;
  uint64_t cps, total, steps;
  uint32_t ring_lds;  // this wave's ring, LDS byte address (wave-uniform)
  __device__ uint64_t chunk_off(uint64_t idx) const {
    const uint64_t stripe = idx / cps, chunk = idx - stripe * cps;
    return stripe * a.stripe_stride + chunk * kBsChunk + threadIdx.x * 16u;
  }
  // step h = (chunk h / k of this workgroup, input h % k) into slot h % D
  __device__ void issue(uint64_t h) const {
    const uint64_t idx = blockIdx.x + (h / C::k) * gridDim.x;
    const uint8_t* g = a.in[h % C::k] + chunk_off(idx);
    const uint32_t l = ring_lds + (uint32_t)(h % D) * 4096u;
#pragma unroll
    for (int j = 0; j < 4; ++j) dma16(g + j * (kBsBlock * 16), l + j * 1024u);
  }
};

template <class C, int D, int I>
__device__ __forceinline__ void dma_inputs(uint32_t (&acc)[C::p * 16], const DmaRing<C, D>& ring,
                                           const uint8_t* ring_ptr, uint64_t g0, bool after_chunk,
                                           uint32_t s_ops) {
  if constexpr (I < C::k) {
    const uint64_t g = g0 + I;
    if (g + D - 1 < ring.steps) ring.issue(g + D - 1);
    const uint64_t ahead = ring.steps - 1 - g;
    uint32_t n = 4u * (uint32_t)(ahead < (uint64_t)(D - 1) ? ahead : (uint64_t)(D - 1));
    if (I < D - 1 && after_chunk) n += s_ops;
    wait_vmcnt(n);
    u32x4 cur[4];
    const uint8_t* slot = ring_ptr + (uint32_t)(g % D) * 4096u + (threadIdx.x & 63u) * 16u;
#pragma unroll
    for (int j = 0; j < 4; ++j) cur[j] = *reinterpret_cast<const u32x4*>(slot + j * 1024);
    uint32_t pl[16];
    slice<typename C::Field>(cur, pl);
    mac_input<C, I>(acc, pl, std::make_integer_sequence<int, C::p * 16>{});
#pragma unroll
    for (int q = 0; q < C::p * 16; ++q) asm volatile("" : "+v"(acc[q]));
    dma_inputs<C, D, I + 1>(acc, ring, ring_ptr, g0, after_chunk, s_ops);
  }
}

template <class C, int D>
__global__ __launch_bounds__(kBsBlock, C::p > 4 ? 2 : 3) void bitslice_dma_kernel(
    const CodeArgs a, uint64_t chunks_per_stripe) {
  __shared__ __attribute__((aligned(16))) uint8_t ring_mem[kBsBlock / 64][D][4096];
  const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint8_t* ring_ptr = &ring_mem[wave][0][0];
  DmaRing<C, D> ring{a, chunks_per_stripe, chunks_per_stripe * a.n_stripes, 0,
                     (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(uintptr_t)ring_ptr)};
  const uint64_t my_chunks =
      blockIdx.x < ring.total ? (ring.total - blockIdx.x + gridDim.x - 1) / gridDim.x : 0;
  ring.steps = my_chunks * C::k;
  const uint32_t mode = a.mode;
  const uint32_t s_ops = (mode == kCheckStore ? 8u : 4u) * C::p;  // output phase VMEM ops
  bool diff = false;
  for (uint64_t h = 0; h + 1 < (uint64_t)D && h < ring.steps; ++h) ring.issue(h);
  for (uint64_t c = 0; c < my_chunks; ++c) {
    const uint64_t off = ring.chunk_off(blockIdx.x + c * gridDim.x);
    uint32_t acc[C::p * 16];
    dma_inputs<C, D, 0>(acc, ring, ring_ptr, c * C::k, c > 0, s_ops);
    store_outputs<C, true>(acc, a, off, mode, diff);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // no DMA outlives the wave
  if (mode != kStore && diff) atomicOr(a.mismatch, 1u);
}

// ------------------------------------------------------------ reconstruct
// Bit-sliced syndrome reconstruct (BsReconArgs in rse_kernels.hpp).  The input
// sequence is the present data shards, then the syndrome parity shards; the
// next present input's loads are issued before the current one is coded.

// Input index J < k is data shard J, J >= k parity shard J - k.
__device__ __forceinline__ const uint8_t* recon_ptr(const BsReconArgs& a, uint32_t k, uint32_t j) {
  return j < k ? a.data[j] : a.par[j - k];
}
// Mask of all inputs read: data present bits, then syndrome rows shifted by k.
__device__ __forceinline__ uint64_t recon_mask(const BsReconArgs& a, uint32_t k) {
  return (uint64_t)a.present | ((uint64_t)a.synd << k);
}

// NS: sigma rows computed (rows 0..NS-1; the host picks NS above every row it
// needs), so a reconstruct pays for the rows it uses, not all p.
template <class C, bool NT, int NS, int I>
__device__ __forceinline__ void recon_inputs(uint32_t (&acc)[NS * 16], u32x4 (&cur)[4],
                                             const BsReconArgs& a, uint64_t mask, uint64_t off) {
  if constexpr (I < C::k + NS) {
    if ((mask >> I) & 1u) {
      const uint64_t rest = mask >> (I + 1);
      u32x4 nxt[4];
      if (rest) load4<NT>(nxt, recon_ptr(a, C::k, I + 1 + __builtin_ctzll(rest)) + off);
      __builtin_amdgcn_sched_barrier(0);  // as in code_inputs (SB)
      uint32_t pl[16];
      slice<typename C::Field>(cur, pl);
      if constexpr (I < C::k) {
        // every sigma row, needed or not: straight-line XOR networks (a
        // branch per row costs more in register pressure than the XORs)
        mac_input<C, I>(acc, pl, std::make_integer_sequence<int, NS * 16>{});
      } else {  // syndrome: s_r = sigma_r ^ parity_r (slicing is linear)
#pragma unroll
        for (int q = 0; q < 16; ++q) acc[(I - C::k) * 16 + q] ^= pl[q];
      }
#pragma unroll
      for (int q = 0; q < NS * 16; ++q) asm volatile("" : "+v"(acc[q]));
      if (rest) {
#pragma unroll
        for (int j = 0; j < 4; ++j) cur[j] = nxt[j];
      }
    }
    recon_inputs<C, NT, NS, I + 1>(acc, cur, a, mask, off);
  }
}

// v (4 vectors of elements) times a table-coded constant, XORed into o.
template <class F>
__device__ __forceinline__ void mac_vectors(u32x4 (&o)[4], const uint32_t* v, const uint4* tq,
                                            const uint32_t* tt2, int idx) {
  if constexpr (F::kPlanes == 8) {
    const Gf8Tab t = read_tab(tq, tt2, idx);
#pragma unroll
    for (int d = 0; d < 16; ++d) o[d >> 2][d & 3] ^= gf8_mul4(t, make_sel(v[d]));
  } else {
    const Gf8Tab hh = read_tab(tq, tt2, idx * 4 + 0), lh = read_tab(tq, tt2, idx * 4 + 1);
    const Gf8Tab hl = read_tab(tq, tt2, idx * 4 + 2), ll = read_tab(tq, tt2, idx * 4 + 3);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      uint32_t h0, l0, h1, l1;
      split_planes(make_uint4(v[4 * j], v[4 * j + 1], v[4 * j + 2], v[4 * j + 3]), h0, l0, h1, l1);
      const Sel sh0 = make_sel(h0), sl0 = make_sel(l0), sh1 = make_sel(h1), sl1 = make_sel(l1);
      const uint4 m = merge_planes(xor3(gf8_mul4(hh, sh0), gf8_mul4(lh, sl0), 0u),
                                   xor3(gf8_mul4(hl, sh0), gf8_mul4(ll, sl0), 0u),
                                   xor3(gf8_mul4(hh, sh1), gf8_mul4(lh, sl1), 0u),
                                   xor3(gf8_mul4(hl, sh1), gf8_mul4(ll, sl1), 0u));
      o[j] ^= (u32x4){m.x, m.y, m.z, m.w};
    }
  }
}

template <class C, bool NT, int NS>
__global__ __launch_bounds__(kBsBlock, NS > 4 ? 2 : 3) void bitslice_recon_kernel(
    const BsReconArgs a, uint64_t chunks_per_stripe) {
  using F = typename C::Field;
  constexpr int TPC = F::kPlanes == 16 ? 4 : 1;  // GF(2^8) tables per coefficient
  __shared__ uint4 tq[kMaxOut * NS * TPC];
  __shared__ uint32_t tt2[kMaxOut * NS * TPC];
  const uint32_t n_out = a.n_out;
  for (uint32_t t = threadIdx.x; t < n_out * NS; t += kBsBlock) {
    const uint32_t c = a.w[t / NS][t % NS];
    if constexpr (TPC == 1) {
      write_tab(tq, tt2, t, make_gf8_tab(c));
    } else {
      uint32_t sub[4];
      gf16_sub_coefs(c, sub);
#pragma unroll
      for (int q = 0; q < 4; ++q) write_tab(tq, tt2, t * 4 + q, make_gf8_tab(sub[q]));
    }
  }
  __syncthreads();
  const uint64_t mask = recon_mask(a, C::k);
  const int first = __builtin_ctzll(mask);  // host guarantees mask != 0
  const uint64_t total = chunks_per_stripe * a.n_stripes;
  for (uint64_t idx = blockIdx.x; idx < total; idx += gridDim.x) {
    const uint64_t stripe = idx / chunks_per_stripe, chunk = idx - stripe * chunks_per_stripe;
    const uint64_t off = stripe * a.stripe_stride + chunk * kBsChunk + threadIdx.x * 16u;
    uint32_t acc[NS * 16];
#pragma unroll
    for (int q = 0; q < NS * 16; ++q) acc[q] = 0u;
    u32x4 cur[4];
    load4<NT>(cur, recon_ptr(a, C::k, first) + off);
    recon_inputs<C, NT, NS, 0>(acc, cur, a, mask, off);
    // back to element order, in place
#pragma unroll
    for (int r = 0; r < NS; ++r) {
      if (!((a.sigma >> r) & 1u)) continue;
      uint32_t pl[16];
#pragma unroll
      for (int q = 0; q < 16; ++q) pl[q] = acc[r * 16 + q];
      u32x4 v[4];
      unslice<F>(pl, v);
#pragma unroll
      for (int q = 0; q < 16; ++q) acc[r * 16 + q] = v[q >> 2][q & 3];
    }
#pragma unroll 1
    for (uint32_t o = 0; o < n_out; ++o) {
      // opaque per output: otherwise LICM hoists every row's byte-plane split
      // and selectors out of this loop (hundreds of VGPRs -> scratch)
#pragma unroll
      for (int q = 0; q < NS * 16; ++q) asm volatile("" : "+v"(acc[q]));
      u32x4 v[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) v[j] = (u32x4){0u, 0u, 0u, 0u};
      const int os = a.out_sigma[o];
#pragma unroll
      for (int r = 0; r < NS; ++r) {
        if (os == r) {
#pragma unroll
          for (int q = 0; q < 16; ++q) v[q >> 2][q & 3] ^= acc[r * 16 + q];
        }
        // one row's tables at a time: the opaque offset (ordered after the
        // previous row's pins) keeps hipcc from loading every row's tables
        // up front, which spills
        const uint32_t lb = opaque_zero();
        if (((a.synd >> r) & 1u) && a.w[o][r] != 0)
          mac_vectors<F>(v, &acc[r * 16], tq, tt2, (int)(lb + o * NS + r));
#pragma unroll
        for (int j = 0; j < 4; ++j)
#pragma unroll
          for (int w = 0; w < 4; ++w) asm volatile("" : "+v"(v[j][w]));
      }
#pragma unroll
      for (int j = 0; j < 4; ++j) stv<NT>(a.out[o] + off + j * (kBsBlock * 16), v[j]);
    }
  }
}

using BsRecFn = void (*)(const BsReconArgs, uint64_t);

using BsFn = void (*)(const CodeArgs, uint64_t);
struct BsShape {
  int field;
  uint32_t k, p;
  const uint16_t* m;  // P x K parity rows compiled into the kernel
  BsFn fn[5][2];      // [variant][nt]: 0 plain, 1 +sched barrier, 2 +cross-chunk
                      // prefetch, 3/4 LDS-DMA input ring of 3/2 slots (nt only)
  BsRecFn rec[4];     // sigma rows NS = 1, 2, 4, 8 (nullptr above p); non-temporal
};

template <class C, int NS>
constexpr BsRecFn rec_fn() {
  if constexpr (NS <= C::p) return bitslice_recon_kernel<C, true, NS>;
  else return nullptr;
}
#define BS(F, FIELD, K, P)                                                      \
  {FIELD, K, P, &Code<F, K, P>::planes.par.m[0][0],                             \
   {{bitslice_kernel<Code<F, K, P>, false, false, false>,                        \
     bitslice_kernel<Code<F, K, P>, true, false, false>},                         \
    {nullptr, bitslice_kernel<Code<F, K, P>, true, true, false>},                 \
    {nullptr, bitslice_kernel<Code<F, K, P>, true, true, true>},                  \
    {nullptr, bitslice_dma_kernel<Code<F, K, P>, 3>},                             \
    {nullptr, bitslice_dma_kernel<Code<F, K, P>, 2>}},                            \
   {rec_fn<Code<F, K, P>, 1>(), rec_fn<Code<F, K, P>, 2>(), rec_fn<Code<F, K, P>, 4>(),  \
    rec_fn<Code<F, K, P>, 8>()}}
static const BsShape kBsShapes[] = {
    BS(CF8, 8, 10, 4),    // BASELINE headline: galois_8 10+4
    BS(CF8, 8, 10, 2),    // benches/bandwidth.rs 10+2
    BS(CF16, 16, 20, 8),  // BASELINE configs[4]: galois_16 20+8
};
#undef BS

}  // namespace

hipError_t launch_bitslice(int field, const CodeArgs& a, bool nt, int64_t grid,
                           hipStream_t stream, bool* handled) {
  *handled = false;
  if (a.accumulate || a.n_vec < kBsChunk / 16) return hipSuccess;
  for (const BsShape& sh : kBsShapes) {
    if (sh.field != field || sh.k != a.n_in || sh.p != a.n_out) continue;
    for (uint32_t o = 0; o < sh.p; ++o)
      for (uint32_t i = 0; i < sh.k; ++i)
        if (a.coef[o][i] != sh.m[o * sh.k + i]) return hipSuccess;
    const uint64_t cps = a.n_vec / (kBsChunk / 16);
    const uint64_t total = cps * a.n_stripes;
    uint64_t gx = grid > 0 ? (uint64_t)grid : 4096u;  // tools/tune.py sweeps
    if (gx > total) gx = total;
    if (gx > 0x7fffffffu) gx = 0x7fffffffu;
    // RSE_OPT_KERNEL_VARIANT picks a bit-sliced variant too (-1: default)
    const int64_t vopt = get_option(4);
    int v = (vopt >= 0 && vopt < 5) ? (int)vopt : kBsDefaultVariant;
    BsFn fn = sh.fn[v][nt ? 1 : 0];
    if (!fn) fn = sh.fn[v][1];
    hipLaunchKernelGGL(fn, dim3((uint32_t)gx), dim3(kBsBlock), 0, stream, a, cps);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    *handled = true;
    return hipSuccess;
  }
  return hipSuccess;
}

hipError_t launch_bitslice_recon(int field, uint32_t k, uint32_t p, const uint16_t* parity_rows,
                                 const BsReconArgs& a, uint64_t n_vec, hipStream_t stream,
                                 bool* handled) {
  *handled = false;
  if (!get_option(5) || n_vec < kBsChunk / 16 || a.n_out == 0 || a.n_out > (uint32_t)kMaxOut ||
      (a.present == 0 && a.synd == 0))
    return hipSuccess;
  for (const BsShape& sh : kBsShapes) {
    if (sh.field != field || sh.k != k || sh.p != p) continue;
    for (uint32_t i = 0; i < k * p; ++i)
      if (parity_rows[i] != sh.m[i]) return hipSuccess;
    const uint64_t cps = n_vec / (kBsChunk / 16);
    const uint64_t total = cps * a.n_stripes;
    const int64_t grid = get_option(2);
    uint64_t gx = grid > 0 ? (uint64_t)grid : 8192u;  // tools/tune.py --op reconstruct sweeps
    if (gx > total) gx = total;
    if (gx > 0x7fffffffu) gx = 0x7fffffffu;
    // rows needed: sigma (R and missing parity); NS = smallest compiled cover
    const uint32_t need = 32u - (uint32_t)__builtin_clz(a.sigma | 1u);
    int slot = -1;
    for (int q = 0; q < 4 && slot < 0; ++q)
      if (sh.rec[q] && (1u << q) >= need) slot = q;
    if (slot < 0) return hipSuccess;
    hipLaunchKernelGGL(sh.rec[slot], dim3((uint32_t)gx), dim3(kBsBlock), 0, stream, a, cps);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    count_bitslice_launch();
    *handled = true;
    return hipSuccess;
  }
  return hipSuccess;
}

uint64_t bitslice_chunk_bytes() { return kBsChunk; }

}  // namespace rse
