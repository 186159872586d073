// rse_bitslice_core.hpp -- device code of the bit-sliced coding kernels, shared
// by the codecs compiled into rse_bitslice.hip and by the modules rse_jit.cpp
// specialises at run time (hiprtc compiles this header as source text, so it
// may only depend on rse_device.hpp / rse_kernels.hpp).
//
// Multiplication by a constant c is a GF(2)-linear map: an 8x8 (GF(2^8)) or
// 16x16 (GF(2^16)) bit matrix.  With the data bit-sliced -- register q holds
// bit q of 32 bytes (GF(2^8)) or of 32 elements (GF(2^16)) -- a
// multiply-accumulate is the XOR of the input planes each row of that bit
// matrix selects, three at a time in gfx950's v_bitop3_b32: no tables, no
// v_perm in the network.  A codec type C supplies the matrices as constants:
//   using Field = BitsF8 | BitsF16 (planes per group and their bit order);
//   static constexpr int k, p, NP, kTemps;
//   static constexpr ... planes.sel[o][i][q] (uint64_t): bit j set iff
//     source j contributes to output plane q of coefficient (o, i).  Sources
//     0..NP-1 are the input's planes (of one group); with kTemps (GF(2^16))
//     or kGTemps (GF(2^8), per group) > 0, sources NP + t are shared
//     subexpressions of that input's network, planes.tmp[i][t] = {a, b, c}:
//     the XOR of sources a, b (and c unless 255), t < planes.ntmp[i]
//     (computed once per input, shared by every output plane that uses them).
//   All of it is generated on the host by rse_netgen.hpp.
//
// Lane layout: a workgroup of 256 lanes codes a 16 KiB chunk of every shard.
// Lane t loads the 16-byte vectors t, t+256, t+512, t+768 of the chunk (each
// load instruction is 4 KiB contiguous per workgroup), i.e. 16 dwords.  GF(2^8):
// two groups of 8 dwords, each 8x8-bit transposed inside byte lanes.  GF(2^16):
// 32 elements split into x-coefficient and constant byte planes with v_perm
// (galois_16.rs:49-51), each 8x8-bit transposed.  Outputs are transposed back
// the same way (the network is an involution).  Any element order works as
// long as input and output use the same one; this one keeps every global
// access coalesced.
#pragma once

#include "rse_device.hpp"

namespace rse {
namespace {

constexpr int kBsBlock = 256;
constexpr uint64_t kBsChunk = 16384;  // bytes of one shard per workgroup step

// std::integer_sequence without <utility> (hiprtc has no C++ library headers)
template <class T, T... I>
struct int_seq {};
template <int N>
using make_int_seq = __make_integer_seq<int_seq, int, N>;

// Plane order of the two fields.
struct BitsF8 {
  static constexpr int kPlanes = 8;
  // plane q = bit q of the byte
  static constexpr int bit(int q) { return q; }
};
struct BitsF16 {
  static constexpr int kPlanes = 16;
  // plane q < 8: bit q of the H (x-coefficient) byte = uint16 bit q + 8;
  // plane q >= 8: bit q - 8 of the L byte = uint16 bit q - 8
  static constexpr int bit(int q) { return q ^ 8; }
};

// ------------------------------------------------------------ bit slicing
// XOR of acc and the sources selected by M (bit j: source j -- an input
// plane or a shared temporary, rse_netgen.hpp), two at a time.
template <uint64_t M>
__device__ __forceinline__ uint32_t xacc(uint32_t acc, const uint32_t* in) {
  if constexpr (M == 0) {
    return acc;
  } else {
    constexpr int q0 = __builtin_ctzll(M);
    constexpr uint64_t m1 = M & (M - 1);
    if constexpr (m1 == 0) {
      return acc ^ in[q0];
    } else {
      constexpr int q1 = __builtin_ctzll(m1);
      return xacc<m1 & (m1 - 1)>(xor3(acc, in[q0], in[q1]), in);
    }
  }
}
template <uint64_t M>
__device__ __forceinline__ uint32_t xinit(const uint32_t* in) {
  if constexpr (M == 0) {
    return 0u;
  } else {
    constexpr int q0 = __builtin_ctzll(M);
    return xacc<M & (M - 1)>(in[q0], in);
  }
}

// Shared temporary t of input I (rse_netgen.hpp): the XOR of two or three of
// the input's earlier sources, one v_bitop3.
template <class C, int I>
__device__ __forceinline__ uint32_t temp_source(const uint32_t* src, int t) {
  const int a = C::planes.tmp[I][t][0], b = C::planes.tmp[I][t][1], c = C::planes.tmp[I][t][2];
  return c == 255 ? src[a] ^ src[b] : xor3(src[a], src[b], src[c == 255 ? 0 : c]);
}

// (x & m) | (y & ~m) in one instruction.  Written out because the C form of
// the transpose below is rewritten by the compiler into masked shifts that
// share subexpressions across the pair: ~1.4 extra v_and per select (1026 in
// the GF(2^16) 20+8 kernel; tools/isa_probe.sh).  As v_bitop3_b32 with the
// select's truth table (0xCA: S0 ? S1 : S2 per bit) rather than v_bfi_b32:
// the same issue rate with an SGPR mask (tools/valu_probe.hip), +0.5-1 % on
// the headline and wide encodes in a same-box A/B (profiles/r03/ab_bitop3/).
__device__ __forceinline__ uint32_t bfi(uint32_t m, uint32_t x, uint32_t y) {
  uint32_t r;
  asm("v_bitop3_b32 %0, %1, %2, %3 bitop3:0xca" : "=v"(r) : "s"(m), "v"(x), "v"(y));
  return r;
}

// 8x8 bit transpose inside every byte lane of h[0..7] (an involution): bit b
// of byte lane L of h[i] moves to bit i of byte lane L of h[b].  Per pair and
// stage: 2 shifts + 2 v_bfi.
__device__ __forceinline__ void transpose8(uint32_t* h) {
#pragma unroll
  for (int s = 4, st = 0; st < 3; s >>= 1, ++st) {
    const uint32_t m = s == 4 ? 0x0F0F0F0Fu : s == 2 ? 0x33333333u : 0x55555555u;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      if (i & s) continue;
      const uint32_t a = h[i], b = h[i + s];
      h[i] = bfi(m << s, b << s, a);
      h[i + s] = bfi(m, a >> s, b);
    }
  }
}

// 4 vectors (16 dwords) -> 16 planes (two groups of 8 for GF(2^8)).
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
  const gptr<const u32x4> q = (gptr<const u32x4>)(p);
  if constexpr (NT) return __builtin_nontemporal_load(q);
  else return *q;
}
template <bool NT>
__device__ __forceinline__ void stv(uint8_t* p, u32x4 v) {
  const gptr<u32x4> q = (gptr<u32x4>)(p);
  if constexpr (NT) __builtin_nontemporal_store(v, q);
  else *q = v;
}

// 16-byte store with an explicit cache policy: WT = write-through (sc1: the
// line leaves the XCD's L2 at once instead of waiting there for eviction).
template <bool NT, bool WT>
__device__ __forceinline__ void stv_policy(uint8_t* p, u32x4 v) {
  if constexpr (WT) {
    if constexpr (NT)
      asm volatile("global_store_dwordx4 %0, %1, off sc1 nt" ::"v"(p), "v"(v) : "memory");
    else
      asm volatile("global_store_dwordx4 %0, %1, off sc1" ::"v"(p), "v"(v) : "memory");
  } else {
    stv<NT>(p, v);
  }
}

// A lane's 4 vectors of one shard, S bytes apart (4 KiB: the workgroup's 256
// lanes cover a 16 KiB chunk; 1 KiB: each wave covers its own 4 KiB chunk).
template <bool NT, uint32_t S = kBsBlock * 16>
__device__ __forceinline__ void load4(u32x4 (&v)[4], const uint8_t* p) {
#pragma unroll
  for (int j = 0; j < 4; ++j) v[j] = ldv<NT>(p + j * S);
}

// acc[o*16 + g*NP + p] (^)= plane combination of group g of input I, for
// every output o, group g and plane p.
// ACC: the accumulators already hold a partial sum (accumulate mode), so
// input 0 adds to them like every other input.
// GF(2^8) with shared subexpressions (C::kGTemps > 0): both 8-plane groups
// use the same bit matrices, so the temporaries are defined once per input
// (planes.tmp[I][t] = sources {a, b}, a source j < 8 a plane of the group,
// 8 + t a temporary) and computed per group; the outputs' rows of group G are
// coded from that group's sources.
template <class C, int I, bool ACC, int G, int N, int... OP>
__device__ __forceinline__ void mac_group(uint32_t (&acc)[N], const uint32_t (&pl)[16],
                                          int_seq<int, OP...>) {
  uint32_t src[8 + C::kGTemps];
#pragma unroll
  for (int q = 0; q < 8; ++q) src[q] = pl[G * 8 + q];
#pragma unroll
  for (int t = 0; t < C::kGTemps; ++t)
    if (t < C::planes.ntmp[I]) src[8 + t] = temp_source<C, I>(src, t);
  // OP runs over outputs; plane q of group G of output o is acc[o * 16 + G * 8 + q]
  if constexpr (I == 0 && !ACC)
    ((acc[(OP / 8) * 16 + G * 8 + OP % 8] = xinit<C::planes.sel[OP / 8][I][OP % 8]>(src)), ...);
  else
    ((acc[(OP / 8) * 16 + G * 8 + OP % 8] =
          xacc<C::planes.sel[OP / 8][I][OP % 8]>(acc[(OP / 8) * 16 + G * 8 + OP % 8], src)),
     ...);
}

template <class C, int I, bool ACC, int N, int... OP>
__device__ __forceinline__ void mac_input(uint32_t (&acc)[N], const uint32_t (&pl)[16],
                                          int_seq<int, OP...>) {
  if constexpr (C::kGTemps > 0) {
    static_assert(C::NP == 8, "group temporaries are for GF(2^8)");
    mac_group<C, I, ACC, 0>(acc, pl, make_int_seq<N / 2>{});
    mac_group<C, I, ACC, 1>(acc, pl, make_int_seq<N / 2>{});
    return;
  }
  uint32_t in[16 + C::kTemps];
#pragma unroll
  for (int q = 0; q < 16; ++q) in[q] = pl[q];
  if constexpr (C::kTemps > 0) {
#pragma unroll
    for (int t = 0; t < C::kTemps; ++t)
      if (t < C::planes.ntmp[I]) in[16 + t] = temp_source<C, I>(in, t);
  }
  if constexpr (I == 0 && !ACC)
    ((acc[OP] = xinit<C::planes.sel[OP / 16][I][OP % C::NP]>(in + (OP % 16) / C::NP * C::NP)),
     ...);
  else
    ((acc[OP] = xacc<C::planes.sel[OP / 16][I][OP % C::NP]>(acc[OP],
                                                              in + (OP % 16) / C::NP * C::NP)),
     ...);
}

// Output phase of one chunk: un-slice every output's planes and store them
// (kStore), compare them with the stored parity (kCheck), or both.
// A: the argument block (CodeArgs, or a wide codec's WideArgs: O0 is then the
// first output of the wave's share).
// CE: check modes load the stored parity before un-slicing, which then covers
// part of its latency (a one-stripe verify: 60 -> 52 us per 10+4 x 16 MiB
// call).  A separate instantiation for the check kernels: in the store-mode
// kernel the reordered code cost the headline encode 1.2 % (same box A/B).
// ok: this lane's bytes belong to the launch (false only for the lanes of a
// stripe-interleaved chunk past the last stripe, SUB below): no store, no
// verdict.
template <class C, bool NT, bool WT = false, uint32_t S = kBsBlock * 16, int O0 = 0,
          class A = CodeArgs, bool CE = false>
__device__ __forceinline__ void store_outputs(uint32_t (&acc)[C::p * 16], const A& a,
                                              uint64_t off, uint32_t mode, bool& diff,
                                              bool ok = true) {
#pragma unroll
  for (int o = 0; o < C::p; ++o) {
    uint32_t pl[16];
#pragma unroll
    for (int q = 0; q < 16; ++q) pl[q] = acc[o * 16 + q];
    u32x4 w[4];
    if (CE && mode != kStore) load4<NT, S>(w, a.cmp[O0 + o] + off);
    u32x4 v[4];
    unslice<typename C::Field>(pl, v);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const uint64_t o16 = off + j * S;
      if (mode != kCheck && ok) stv_policy<NT, WT>(a.out[O0 + o] + o16, v[j]);
      if (mode != kStore) {
        if (!CE) w[j] = ldv<NT>(a.cmp[O0 + o] + o16);
        diff |= ok & ((w[j].x != v[j].x) | (w[j].y != v[j].y) | (w[j].z != v[j].z) |
                      (w[j].w != v[j].w));
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
template <class C, bool NT, bool SB, bool XC, int I, uint32_t S = kBsBlock * 16,
          bool ACC = false, class A = CodeArgs>
__device__ __forceinline__ void code_inputs(uint32_t (&acc)[C::p * 16], u32x4 (&cur)[4],
                                            const A& a, uint64_t off, uint64_t next_off) {
  u32x4 nxt[4];
  if constexpr (I + 1 < C::k) {
    load4<NT, S>(nxt, a.in[I + 1] + off);
  } else if constexpr (XC) {
    if (next_off != ~0ull) load4<NT, S>(nxt, a.in[0] + next_off);
  }
  if constexpr (SB) __builtin_amdgcn_sched_barrier(0);
  uint32_t pl[16];
  slice<typename C::Field>(cur, pl);
  mac_input<C, I, ACC>(acc, pl, make_int_seq<C::p * 16>{});
  // keep each input's XORs together: without this the compiler reassociates
  // across inputs and keeps several inputs' planes live (spills)
#pragma unroll
  for (int q = 0; q < C::p * 16; ++q) asm volatile("" : "+v"(acc[q]));
  if constexpr (I + 1 < C::k) {
#pragma unroll
    for (int j = 0; j < 4; ++j) cur[j] = nxt[j];
    code_inputs<C, NT, SB, XC, I + 1, S, ACC, A>(acc, cur, a, off, next_off);
  } else if constexpr (XC) {
    if (next_off != ~0ull) {
#pragma unroll
      for (int j = 0; j < 4; ++j) cur[j] = nxt[j];
    }
  }
}

// Encode / verify body.  One workgroup step = one 16 KiB chunk of one stripe;
// chunks of all stripes are one flat index space walked grid-stride.  a.n_vec
// counts whole chunks' vectors only (the host codes the remainder with the
// table kernels).  Launch bounds: kBsBlock lanes, C::p > 4 ? 2 : 3 waves/SIMD.
//  XM: XCD-aware order -- workgroups are dispatched round-robin over the 8
//      XCDs, so workgroup b (on XCD b % 8) takes slot (b % 8) * (G / 8) + b / 8
//      and each XCD walks its own contiguous run of chunks.
//  W4: 4 KiB chunks, one per wave (lane l loads vectors l, l+64, l+128,
//      l+192 of its wave's chunk; each load instruction still 1 KiB
//      contiguous), for shards -- or the rest of shards -- shorter than
//      16 KiB; chunks_per_stripe then counts 4 KiB chunks.
//  ACC: accumulate mode (a.accumulate): the outputs' current bytes are
//      loaded and sliced into the accumulators first -- the blocks of a wide
//      codec's parity matrix, input chunk after input chunk (rse_jit.cpp).
//  SUB: shards of exactly 1 KiB or 2 KiB (W4 only): a wave's "4 KiB chunk"
//      is 4096 / SUB consecutive stripes' shards.  64 * SUB / 4096 lanes take
//      each stripe, lane vectors SUB / 4 bytes apart (each load instruction:
//      runs of SUB / 4 contiguous bytes per stripe), so the reference's own
//      1-2 KiB blocks (benches/bandwidth.rs:88-190) run on the bit-sliced
//      networks too.  The bit-slicing never mixes bytes of different lane
//      vector positions, so lanes of different stripes are independent; lanes
//      past the last stripe load the last stripe's bytes and store nothing.
//      chunks_per_stripe is unused (the chunk count follows from n_stripes).
template <class C, bool NT, bool SB, bool XC, bool XM = false, bool WT = false, bool W4 = false,
          bool ACC = false, bool CE = false, uint32_t SUB = 0>
__device__ __forceinline__ void bitslice_body(const CodeArgs& a, uint64_t chunks_per_stripe) {
  static_assert(!(XC && W4), "cross-chunk prefetch is for 16 KiB chunks");
  static_assert(!(XC && ACC), "cross-chunk prefetch is for store mode");
  static_assert(SUB == 0 || (W4 && (SUB == 1024u || SUB == 2048u)),
                "stripe-interleaved chunks: 1 or 2 KiB shards, one chunk per wave");
  constexpr uint32_t S = SUB ? SUB / 4u : W4 ? 1024u : kBsBlock * 16u;
  constexpr uint64_t CH = W4 ? 4096u : kBsChunk;
  constexpr uint32_t SPC = SUB ? 4096u / SUB : 1u, LPS = 64u / SPC;  // stripes / chunk, lanes / stripe
  const uint64_t total = SUB ? (a.n_stripes + SPC - 1) / SPC : chunks_per_stripe * a.n_stripes;
  const uint64_t steps = W4 ? (total + 3) / 4 : total;
  const uint32_t sub = W4 ? threadIdx.x >> 6 : 0u;  // wave-uniform
  const uint32_t lane = threadIdx.x & 63u;
  const uint32_t lane_off = (SUB ? lane % LPS : W4 ? lane : threadIdx.x) * 16u;
  const uint32_t G = gridDim.x;
  const uint32_t wg = (XM && G % 8u == 0) ? (blockIdx.x % 8u) * (G / 8u) + blockIdx.x / 8u
                                           : blockIdx.x;
  const uint32_t mode = a.mode;
  bool diff = false;
  auto chunk_off = [&](uint64_t c) {
    if constexpr (SUB) {
      uint64_t stripe = c * SPC + lane / LPS;
      if (stripe >= a.n_stripes) stripe = a.n_stripes - 1;  // loaded, never stored
      return stripe * a.stripe_stride + lane_off;
    }
    const uint64_t stripe = c / chunks_per_stripe, chunk = c - stripe * chunks_per_stripe;
    return stripe * a.stripe_stride + chunk * CH + lane_off;
  };
  u32x4 cur[4];
  if (XC && wg < total) load4<NT, S>(cur, a.in[0] + chunk_off(wg));
  for (uint64_t idx = wg; idx < steps; idx += G) {
    const uint64_t c = W4 ? idx * 4 + sub : idx;
    if (W4 && c >= total) continue;  // the last step's spare waves
    const uint64_t off = chunk_off(c);
    const uint64_t nidx = idx + G;
    const uint64_t next_off = (XC && nidx < total) ? chunk_off(nidx) : ~0ull;
    uint32_t acc[C::p * 16];
    if (!XC) load4<NT, S>(cur, a.in[0] + off);
    if constexpr (ACC) {
#pragma unroll
      for (int o = 0; o < C::p; ++o) {
        u32x4 t[4];
        load4<NT, S>(t, a.out[o] + off);
        uint32_t pl[16];
        slice<typename C::Field>(t, pl);
#pragma unroll
        for (int q = 0; q < 16; ++q) acc[o * 16 + q] = pl[q];
      }
    }
    code_inputs<C, NT, SB, XC, 0, S, ACC>(acc, cur, a, off, next_off);
    const bool ok = SUB == 0 || c * SPC + lane / LPS < a.n_stripes;
    store_outputs<C, NT, WT, S, 0, CodeArgs, CE>(acc, a, off, mode, diff, ok);
    if (a.per_stripe && diff) {  // verify_flat: this chunk's stripe (SUB: this lane's)
      flag_mismatch(a.mismatch + (SUB ? c * SPC + lane / LPS : c / chunks_per_stripe));
      diff = false;
    }
  }
  if (mode != kStore && diff) flag_mismatch(a.mismatch);
}

// Inputs I.. of one chunk with D inputs in flight: input I + D is loaded
// before input I is coded (buf is a ring of D + 1 input slots, indexed at
// compile time so it stays in VGPRs).
template <class C, bool NT, int D, int I>
__device__ __forceinline__ void code_inputs_deep(uint32_t (&acc)[C::p * 16],
                                                 u32x4 (&buf)[D + 1][4], const CodeArgs& a,
                                                 uint64_t off) {
  if constexpr (I < C::k) {
    if constexpr (I + D < C::k) load4<NT>(buf[(I + D) % (D + 1)], a.in[I + D] + off);
    __builtin_amdgcn_sched_barrier(0);
    uint32_t pl[16];
    slice<typename C::Field>(buf[I % (D + 1)], pl);
    mac_input<C, I, false>(acc, pl, make_int_seq<C::p * 16>{});
#pragma unroll
    for (int q = 0; q < C::p * 16; ++q) asm volatile("" : "+v"(acc[q]));
    code_inputs_deep<C, NT, D, I + 1>(acc, buf, a, off);
  }
}

// bitslice_body with D inputs in flight per lane instead of one.
template <class C, bool NT, int D>
__device__ __forceinline__ void bitslice_body_deep(const CodeArgs& a, uint64_t chunks_per_stripe) {
  const uint64_t total = chunks_per_stripe * a.n_stripes;
  const uint32_t mode = a.mode;
  bool diff = false;
  for (uint64_t idx = blockIdx.x; idx < total; idx += gridDim.x) {
    const uint64_t stripe = idx / chunks_per_stripe, chunk = idx - stripe * chunks_per_stripe;
    const uint64_t off = stripe * a.stripe_stride + chunk * kBsChunk + threadIdx.x * 16u;
    uint32_t acc[C::p * 16];
    u32x4 buf[D + 1][4];
#pragma unroll
    for (int j = 0; j < D; ++j)
      if (j < C::k) load4<NT>(buf[j], a.in[j] + off);
    code_inputs_deep<C, NT, D, 0>(acc, buf, a, off);
    store_outputs<C, NT>(acc, a, off, mode, diff);
    if (a.per_stripe && diff) {
      flag_mismatch(a.mismatch + stripe);
      diff = false;
    }
  }
  if (mode != kStore && diff) flag_mismatch(a.mismatch);
}

// ------------------------------------------------------------ wide codecs
// Codecs with more than 8 parity rows (or 32 data shards): one workgroup of W
// waves per 4 KiB chunk of every shard, and wave w codes its own share of the
// outputs (C: those rows over ALL k inputs, O0 the first of them) from the
// same inputs.  Every wave loads every input chunk itself (plain loads: the
// workgroup's waves run side by side on one CU, so the lines are fetched from
// HBM once and served to the other waves by L1/L2); every output is written
// once.  Lane layout of the 4 KiB chunks: lane l loads vectors l, l+64,
// l+128, l+192 (each load instruction 1 KiB contiguous per wave).
// SUB: 1 or 2 KiB shards, a chunk = 4096 / SUB consecutive stripes' shards
// (bitslice_body's SUB).
template <class C, int O0, class A, uint32_t SUB = 0>
__device__ __forceinline__ void wide_body(const A& a) {
  const WideHdr& h = a.h;
  constexpr uint32_t S = SUB ? SUB / 4u : 1024u;
  constexpr uint32_t SPC = SUB ? 4096u / SUB : 1u, LPS = 64u / SPC;
  const uint64_t total = SUB ? (h.n_stripes + SPC - 1) / SPC : h.chunks_per_stripe * h.n_stripes;
  const uint32_t lane = threadIdx.x & 63u, lane_off = (SUB ? lane % LPS : lane) * 16u;
  const uint32_t mode = h.mode;
  bool diff = false;
  for (uint64_t c = blockIdx.x; c < total; c += gridDim.x) {
    uint64_t stripe, off;
    if constexpr (SUB) {
      stripe = c * SPC + lane / LPS;
      off = (stripe < h.n_stripes ? stripe : h.n_stripes - 1) * h.stripe_stride + lane_off;
    } else {
      stripe = c / h.chunks_per_stripe;
      off = stripe * h.stripe_stride + (c - stripe * h.chunks_per_stripe) * 4096u + lane_off;
    }
    const bool ok = SUB == 0 || stripe < h.n_stripes;  // lanes past the last stripe: no stores
    uint32_t acc[C::p * 16];
    u32x4 cur[4];
    load4<false, S>(cur, a.in[0] + off);
    code_inputs<C, false, true, false, 0, S, false, A>(acc, cur, a, off, ~0ull);
    store_outputs<C, true, false, S, O0, A>(acc, a, off, mode, diff, ok);
    if (h.per_stripe && diff) {
      flag_mismatch(h.mismatch + stripe);
      diff = false;
    }
  }
  if (mode != kStore && diff) flag_mismatch(h.mismatch);
}

// wide_body with the slicing shared through LDS: in round R, wave WI (of W)
// slices input R*W + WI -- only that one -- and writes its 16 planes to an LDS
// slot; after a barrier every wave codes the round's W inputs from LDS.  A
// wave thus slices k/W inputs instead of k (slicing is a third of a wide
// codec's VALU work).  Two slot sets alternate by a running round counter g,
// so a set is rewritten only two barriers after it was read, across chunks
// too: one barrier per round.
template <int W>
using WidePlanes = uint4[2][W][4][64];  // [set][slot][quad of planes][lane]

// Paired inputs (C::kPairIn, GF(2^8), rse_netgen.hpp build_pairs): network
// input J is data inputs 2J and 2J + 1, sources 0..7 the first's planes of a
// group, 8..15 the second's, then J's temporaries (per group, both groups
// sharing the bit matrices).  pb may be all zero (odd k: no second input).
template <class C, int J, int... OP>
__device__ __forceinline__ void mac_pair(uint32_t (&acc)[C::p * 16], const uint32_t (&pa)[16],
                                         const uint32_t (&pb)[16], int_seq<int, OP...>) {
#pragma unroll
  for (int g = 0; g < 2; ++g) {
    uint32_t src[16 + C::kGTemps];
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      src[q] = pa[g * 8 + q];
      src[8 + q] = pb[g * 8 + q];
    }
#pragma unroll
    for (int t = 0; t < C::kGTemps; ++t)
      if (t < C::planes.ntmp[J]) src[16 + t] = temp_source<C, J>(src, t);
    // OP < p * 8: output OP / 8, plane OP % 8 of group g; input pair 0
    // initialises the accumulators (as mac_input's input 0 does)
    if constexpr (J == 0) {
      if (g == 0)
        ((acc[(OP / 8) * 16 + OP % 8] = xinit<C::planes.sel[OP / 8][J][OP % 8]>(src)), ...);
      else
        ((acc[(OP / 8) * 16 + 8 + OP % 8] = xinit<C::planes.sel[OP / 8][J][OP % 8]>(src)), ...);
    } else {
      if (g == 0)
        ((acc[(OP / 8) * 16 + OP % 8] =
              xacc<C::planes.sel[OP / 8][J][OP % 8]>(acc[(OP / 8) * 16 + OP % 8], src)),
         ...);
      else
        ((acc[(OP / 8) * 16 + 8 + OP % 8] =
              xacc<C::planes.sel[OP / 8][J][OP % 8]>(acc[(OP / 8) * 16 + 8 + OP % 8], src)),
         ...);
    }
  }
}

template <class C, int W, int R, int S>
__device__ __forceinline__ void wide_code_round(uint32_t (&acc)[C::p * 16],
                                                const uint4 (&set)[W][4][64], uint32_t lane) {
  if constexpr (C::kPairIn) {
    // two inputs at a time (W even, so a round's inputs pair up)
    static_assert(W % 2 == 0, "paired inputs need an even number of waves");
    if constexpr (S < W && R * W + S < C::k) {
      uint32_t pa[16], pb[16];
#pragma unroll
      for (int q4 = 0; q4 < 4; ++q4) {
        const uint4 v = set[S][q4][lane];
        pa[q4 * 4 + 0] = v.x;
        pa[q4 * 4 + 1] = v.y;
        pa[q4 * 4 + 2] = v.z;
        pa[q4 * 4 + 3] = v.w;
      }
      if constexpr (R * W + S + 1 < C::k) {
#pragma unroll
        for (int q4 = 0; q4 < 4; ++q4) {
          const uint4 v = set[S + 1][q4][lane];
          pb[q4 * 4 + 0] = v.x;
          pb[q4 * 4 + 1] = v.y;
          pb[q4 * 4 + 2] = v.z;
          pb[q4 * 4 + 3] = v.w;
        }
      } else {
#pragma unroll
        for (int q = 0; q < 16; ++q) pb[q] = 0u;
      }
      mac_pair<C, (R * W + S) / 2>(acc, pa, pb, make_int_seq<C::p * 8>{});
#pragma unroll
      for (int q = 0; q < C::p * 16; ++q) asm volatile("" : "+v"(acc[q]));
      wide_code_round<C, W, R, S + 2>(acc, set, lane);
    }
  } else if constexpr (S < W && R * W + S < C::k) {
    uint32_t pl[16];
#pragma unroll
    for (int q4 = 0; q4 < 4; ++q4) {
      const uint4 v = set[S][q4][lane];
      pl[q4 * 4 + 0] = v.x;
      pl[q4 * 4 + 1] = v.y;
      pl[q4 * 4 + 2] = v.z;
      pl[q4 * 4 + 3] = v.w;
    }
    mac_input<C, R * W + S, false>(acc, pl, make_int_seq<C::p * 16>{});
#pragma unroll
    for (int q = 0; q < C::p * 16; ++q) asm volatile("" : "+v"(acc[q]));
    wide_code_round<C, W, R, S + 1>(acc, set, lane);
  }
}

template <class C, int W, int WI, int R, class A>
__device__ __forceinline__ void wide_rounds(uint32_t (&acc)[C::p * 16], u32x4 (&cur)[4],
                                            const A& a, uint64_t off, WidePlanes<W>& lds,
                                            uint32_t& g, uint32_t lane) {
  constexpr int K = C::k, NR = (K + W - 1) / W;
  if constexpr (R < NR) {
    constexpr int mine = R * W + WI, next = (R + 1) * W + WI;
    u32x4 nxt[4];
    if constexpr (next < K) load4<false, 1024u>(nxt, a.in[next] + off);
    __builtin_amdgcn_sched_barrier(0);
    uint4(&set)[W][4][64] = lds[g & 1u];
    if constexpr (mine < K) {
      uint32_t pl[16];
      slice<typename C::Field>(cur, pl);
#pragma unroll
      for (int q4 = 0; q4 < 4; ++q4)
        set[WI][q4][lane] = make_uint4(pl[q4 * 4], pl[q4 * 4 + 1], pl[q4 * 4 + 2], pl[q4 * 4 + 3]);
    }
    __syncthreads();
    wide_code_round<C, W, R, 0>(acc, set, lane);
    ++g;
    if constexpr (next < K) {
#pragma unroll
      for (int j = 0; j < 4; ++j) cur[j] = nxt[j];
    }
    wide_rounds<C, W, WI, R + 1, A>(acc, cur, a, off, lds, g, lane);
  }
}

// wide_rounds with D inputs in flight per wave instead of one.  A wave's own
// inputs are R * W + WI over the rounds R; in round R it loads round R + D's
// (ring of D + 1 slots, indexed at compile time so it stays in VGPRs).  Past
// the chunk's last round it loads the first rounds of the workgroup's next
// chunk (next_off, ~0 if none), so loads stay in flight through the output
// phase too.  Why: one 4 KiB input per wave in flight is 16 KiB per 4-wave
// workgroup, ~32 KiB per CU at 2 workgroups -- ~8 MiB over the chip, which at
// ~2 us of loaded HBM latency caps the read rate near 4 TB/s whatever the
// VALU does (Little's law); D inputs per wave raise that cap D-fold.
template <class C, int W, int WI, int D, int R, class A, uint32_t S = 1024u>
__device__ __forceinline__ void wide_rounds_deep(uint32_t (&acc)[C::p * 16],
                                                 u32x4 (&buf)[D + 1][4], const A& a, uint64_t off,
                                                 uint64_t next_off, WidePlanes<W>& lds, uint32_t& g,
                                                 uint32_t lane) {
  constexpr int K = C::k, NR = (K + W - 1) / W;
  if constexpr (R < NR) {
    constexpr int mine = R * W + WI, ahead = R + D;
    if constexpr (ahead < NR) {
      if constexpr (ahead * W + WI < K) load4<false, S>(buf[ahead % (D + 1)], a.in[ahead * W + WI] + off);
    } else if constexpr ((ahead - NR) * W + WI < K) {
      if (next_off != ~0ull) load4<false, S>(buf[ahead % (D + 1)], a.in[(ahead - NR) * W + WI] + next_off);
    }
    __builtin_amdgcn_sched_barrier(0);
    uint4(&set)[W][4][64] = lds[g & 1u];
    if constexpr (mine < K) {
      uint32_t pl[16];
      slice<typename C::Field>(buf[R % (D + 1)], pl);
#pragma unroll
      for (int q4 = 0; q4 < 4; ++q4)
        set[WI][q4][lane] = make_uint4(pl[q4 * 4], pl[q4 * 4 + 1], pl[q4 * 4 + 2], pl[q4 * 4 + 3]);
    }
    __syncthreads();
    wide_code_round<C, W, R, 0>(acc, set, lane);
    ++g;
    wide_rounds_deep<C, W, WI, D, R + 1, A, S>(acc, buf, a, off, next_off, lds, g, lane);
  }
}

// Wave WI of W; C its share of the outputs (O0 the first).  All W waves call
// this with the same `lds` (one workgroup-wide array).  D: inputs in flight
// per wave (wide_rounds_deep); 1 is wide_rounds.
// SUB: 1 or 2 KiB shards, a chunk = 4096 / SUB consecutive stripes' shards
// (bitslice_body's SUB).
template <class C, int O0, int W, int WI, int D, class A, uint32_t SUB = 0>
__device__ __forceinline__ void wide_body_lds_deep(const A& a, WidePlanes<W>& lds) {
  const WideHdr& h = a.h;
  constexpr int K = C::k, NR = (K + W - 1) / W;
  constexpr uint32_t S = SUB ? SUB / 4u : 1024u;
  constexpr uint32_t SPC = SUB ? 4096u / SUB : 1u, LPS = 64u / SPC;
  const uint64_t total = SUB ? (h.n_stripes + SPC - 1) / SPC : h.chunks_per_stripe * h.n_stripes;
  const uint32_t lane = threadIdx.x & 63u, lane_off = (SUB ? lane % LPS : lane) * 16u;
  const uint32_t mode = h.mode;
  bool diff = false;
  uint32_t g = 0;
  auto chunk_off = [&](uint64_t c) {
    if constexpr (SUB) {
      uint64_t stripe = c * SPC + lane / LPS;
      if (stripe >= h.n_stripes) stripe = h.n_stripes - 1;  // loaded, never stored
      return stripe * h.stripe_stride + lane_off;
    }
    const uint64_t stripe = c / h.chunks_per_stripe, chunk = c - stripe * h.chunks_per_stripe;
    return stripe * h.stripe_stride + chunk * 4096u + lane_off;
  };
  u32x4 buf[D + 1][4];
  if (blockIdx.x < total) {
    const uint64_t off0 = chunk_off(blockIdx.x);
#pragma unroll
    for (int j = 0; j < D; ++j)
      if (j < NR && j * W + WI < K) load4<false, S>(buf[j], a.in[j * W + WI] + off0);
  }
  for (uint64_t c = blockIdx.x; c < total; c += gridDim.x) {
    const uint64_t off = chunk_off(c);
    const uint64_t next = c + gridDim.x;
    const uint64_t next_off = next < total ? chunk_off(next) : ~0ull;
    uint32_t acc[C::p * 16];
    wide_rounds_deep<C, W, WI, D, 0, A, S>(acc, buf, a, off, next_off, lds, g, lane);
    if constexpr (NR % (D + 1) != 0) {  // the next chunk's rounds j into slots j
      u32x4 t[D][4];
#pragma unroll
      for (int j = 0; j < D; ++j)
#pragma unroll
        for (int q = 0; q < 4; ++q) t[j][q] = buf[(NR + j) % (D + 1)][q];
#pragma unroll
      for (int j = 0; j < D; ++j)
#pragma unroll
        for (int q = 0; q < 4; ++q) buf[j][q] = t[j][q];
    }
    store_outputs<C, true, false, S, O0, A>(acc, a, off, mode, diff,
                                            SUB == 0 || c * SPC + lane / LPS < h.n_stripes);
    if (h.per_stripe && diff) {
      flag_mismatch(h.mismatch + (SUB ? c * SPC + lane / LPS : c / h.chunks_per_stripe));
      diff = false;
    }
  }
  if (mode != kStore && diff) flag_mismatch(h.mismatch);
}

// Wave WI of W; C its share of the outputs (O0 the first).  All W waves call
// this with the same `lds` (one workgroup-wide array).
template <class C, int O0, int W, int WI, class A>
__device__ __forceinline__ void wide_body_lds(const A& a, WidePlanes<W>& lds) {
  const WideHdr& h = a.h;
  const uint64_t total = h.chunks_per_stripe * h.n_stripes;
  const uint32_t lane = threadIdx.x & 63u, lane_off = lane * 16u;
  const uint32_t mode = h.mode;
  bool diff = false;
  uint32_t g = 0;
  for (uint64_t c = blockIdx.x; c < total; c += gridDim.x) {
    const uint64_t stripe = c / h.chunks_per_stripe, chunk = c - stripe * h.chunks_per_stripe;
    const uint64_t off = stripe * h.stripe_stride + chunk * 4096u + lane_off;
    uint32_t acc[C::p * 16];
    u32x4 cur[4];
    if constexpr (WI < C::k) load4<false, 1024u>(cur, a.in[WI] + off);
    wide_rounds<C, W, WI, 0, A>(acc, cur, a, off, lds, g, lane);
    store_outputs<C, true, false, 1024u, O0, A>(acc, a, off, mode, diff);
    if (h.per_stripe && diff) {
      flag_mismatch(h.mismatch + stripe);
      diff = false;
    }
  }
  if (mode != kStore && diff) flag_mismatch(h.mismatch);
}

// ------------------------------------- GF(2^8) wide codecs on half chunks
// wide_body_lds_deep gives each lane 16 dwords of every shard (a 4 KiB chunk
// per wave): two 8-plane groups, so a wave's share of o outputs holds 16 o
// accumulators.  At 8 outputs per wave (32+32, 64+64: the reference's widest
// bench shapes, benches/bandwidth.rs:94-95, 154-155) that is 128 VGPRs before
// the input pair's 16 planes and 32 temporaries, and the module spilled 172
// (32+32) / 274 (64+64) VGPRs to scratch.  Here a wave's chunk is 2 KiB: lane
// l loads vectors l and l + 64 (each load instruction still 1 KiB contiguous
// per wave) -- 8 dwords, ONE plane group -- so the accumulators halve, and the
// network code (written once per group in mac_pair) is half as long.  The
// networks themselves are the paired GF(2^8) ones (C::kPairIn): the same
// XORs per byte.  SUB: 1 or 2 KiB shards, a chunk = 2048 / SUB consecutive
// stripes' shards (32 lanes per stripe for 1 KiB, vectors 512 B apart).
template <int W>
using WideHalfPlanes = uint4[2][W][2][64];  // [set][slot][quad of planes][lane]

// 2 vectors (8 dwords) -> 8 planes, and back (clobbers pl).
__device__ __forceinline__ void slice8(const u32x4 (&v)[2], uint32_t (&pl)[8]) {
#pragma unroll
  for (int d = 0; d < 8; ++d) pl[d] = v[d >> 2][d & 3];
  transpose8(pl);
}
__device__ __forceinline__ void unslice8(uint32_t (&pl)[8], u32x4 (&v)[2]) {
  transpose8(pl);
#pragma unroll
  for (int d = 0; d < 8; ++d) v[d >> 2][d & 3] = pl[d];
}
template <uint32_t S>
__device__ __forceinline__ void load2(u32x4 (&v)[2], const uint8_t* p) {
  v[0] = ldv<false>(p);
  v[1] = ldv<false>(p + S);
}

// mac_pair on one plane group: acc[o * 8 + q] (^)= plane q of output o's
// terms of network input J (data inputs 2J, 2J + 1).
template <class C, int J, int... OP>
__device__ __forceinline__ void mac_pair_half(uint32_t (&acc)[C::p * 8], const uint32_t (&pa)[8],
                                              const uint32_t (&pb)[8], int_seq<int, OP...>) {
  uint32_t src[16 + C::kGTemps];
#pragma unroll
  for (int q = 0; q < 8; ++q) {
    src[q] = pa[q];
    src[8 + q] = pb[q];
  }
#pragma unroll
  for (int t = 0; t < C::kGTemps; ++t)
    if (t < C::planes.ntmp[J]) src[16 + t] = temp_source<C, J>(src, t);
  if constexpr (J == 0)
    ((acc[OP] = xinit<C::planes.sel[OP / 8][J][OP % 8]>(src)), ...);
  else
    ((acc[OP] = xacc<C::planes.sel[OP / 8][J][OP % 8]>(acc[OP], src)), ...);
}

template <class C, int W, int R, int S>
__device__ __forceinline__ void wide_code_round_half(uint32_t (&acc)[C::p * 8],
                                                     const uint4 (&set)[W][2][64], uint32_t lane) {
  static_assert(C::kPairIn && W % 2 == 0, "half chunks: paired GF(2^8) networks, W even");
  if constexpr (S < W && R * W + S < C::k) {
    uint32_t pa[8], pb[8];
#pragma unroll
    for (int q4 = 0; q4 < 2; ++q4) {
      const uint4 v = set[S][q4][lane];
      pa[q4 * 4 + 0] = v.x;
      pa[q4 * 4 + 1] = v.y;
      pa[q4 * 4 + 2] = v.z;
      pa[q4 * 4 + 3] = v.w;
    }
    if constexpr (R * W + S + 1 < C::k) {
#pragma unroll
      for (int q4 = 0; q4 < 2; ++q4) {
        const uint4 v = set[S + 1][q4][lane];
        pb[q4 * 4 + 0] = v.x;
        pb[q4 * 4 + 1] = v.y;
        pb[q4 * 4 + 2] = v.z;
        pb[q4 * 4 + 3] = v.w;
      }
    } else {
#pragma unroll
      for (int q = 0; q < 8; ++q) pb[q] = 0u;
    }
    mac_pair_half<C, (R * W + S) / 2>(acc, pa, pb, make_int_seq<C::p * 8>{});
#pragma unroll
    for (int q = 0; q < C::p * 8; ++q) asm volatile("" : "+v"(acc[q]));
    wide_code_round_half<C, W, R, S + 2>(acc, set, lane);
  }
}

// The rounds of one half chunk, D own inputs in flight per wave (as
// wide_rounds_deep: ring of D + 1 slots; past the last round, the next
// chunk's first rounds).
template <class C, int W, int WI, int D, int R, class A, uint32_t S>
__device__ __forceinline__ void wide_rounds_half(uint32_t (&acc)[C::p * 8], u32x4 (&buf)[D + 1][2],
                                                 const A& a, uint64_t off, uint64_t next_off,
                                                 WideHalfPlanes<W>& lds, uint32_t& g, uint32_t lane) {
  constexpr int K = C::k, NR = (K + W - 1) / W;
  if constexpr (R < NR) {
    constexpr int mine = R * W + WI, ahead = R + D;
    if constexpr (ahead < NR) {
      if constexpr (ahead * W + WI < K) load2<S>(buf[ahead % (D + 1)], a.in[ahead * W + WI] + off);
    } else if constexpr ((ahead - NR) * W + WI < K) {
      if (next_off != ~0ull) load2<S>(buf[ahead % (D + 1)], a.in[(ahead - NR) * W + WI] + next_off);
    }
    __builtin_amdgcn_sched_barrier(0);
    uint4(&set)[W][2][64] = lds[g & 1u];
    if constexpr (mine < K) {
      uint32_t pl[8];
      slice8(buf[R % (D + 1)], pl);
      set[WI][0][lane] = make_uint4(pl[0], pl[1], pl[2], pl[3]);
      set[WI][1][lane] = make_uint4(pl[4], pl[5], pl[6], pl[7]);
    }
    __syncthreads();
    wide_code_round_half<C, W, R, 0>(acc, set, lane);
    ++g;
    wide_rounds_half<C, W, WI, D, R + 1, A, S>(acc, buf, a, off, next_off, lds, g, lane);
  }
}

// Wave WI of W; C its share of the outputs (O0 the first).  All W waves call
// this with the same `lds`.  The launch's chunk count is in 2 KiB units
// (rse_jit.cpp launch_wide: twice the 4 KiB chunks, or ceil(n_stripes /
// (2048 / SUB))).
template <class C, int O0, int W, int WI, int D, class A, uint32_t SUB = 0>
__device__ __forceinline__ void wide_body_half(const A& a, WideHalfPlanes<W>& lds) {
  static_assert(SUB == 0 || SUB == 1024u || SUB == 2048u, "1 or 2 KiB shards");
  const WideHdr& h = a.h;
  constexpr int K = C::k, NR = (K + W - 1) / W;
  constexpr uint32_t S = SUB ? SUB / 2u : 1024u;  // a lane's two vectors, S bytes apart
  constexpr uint32_t SPC = SUB ? 2048u / SUB : 1u, LPS = 64u / SPC;  // stripes / chunk, lanes / stripe
  const uint64_t halves = 2 * h.chunks_per_stripe;  // 2 KiB chunks per stripe
  const uint64_t total = SUB ? (h.n_stripes + SPC - 1) / SPC : halves * h.n_stripes;
  const uint32_t lane = threadIdx.x & 63u, lane_off = (SUB ? lane % LPS : lane) * 16u;
  const uint32_t mode = h.mode;
  bool diff = false;
  uint32_t g = 0;
  auto chunk_off = [&](uint64_t c) {
    if constexpr (SUB) {
      uint64_t stripe = c * SPC + lane / LPS;
      if (stripe >= h.n_stripes) stripe = h.n_stripes - 1;  // loaded, never stored
      return stripe * h.stripe_stride + lane_off;
    }
    const uint64_t stripe = c / halves, half = c - stripe * halves;
    return stripe * h.stripe_stride + half * 2048u + lane_off;
  };
  u32x4 buf[D + 1][2];
  if (blockIdx.x < total) {
    const uint64_t off0 = chunk_off(blockIdx.x);
#pragma unroll
    for (int j = 0; j < D; ++j)
      if (j < NR && j * W + WI < K) load2<S>(buf[j], a.in[j * W + WI] + off0);
  }
  for (uint64_t c = blockIdx.x; c < total; c += gridDim.x) {
    const uint64_t off = chunk_off(c);
    const uint64_t next = c + gridDim.x;
    const uint64_t next_off = next < total ? chunk_off(next) : ~0ull;
    uint32_t acc[C::p * 8];
    wide_rounds_half<C, W, WI, D, 0, A, S>(acc, buf, a, off, next_off, lds, g, lane);
    if constexpr (NR % (D + 1) != 0) {  // the next chunk's rounds j into slots j
      u32x4 t[D][2];
#pragma unroll
      for (int j = 0; j < D; ++j)
#pragma unroll
        for (int q = 0; q < 2; ++q) t[j][q] = buf[(NR + j) % (D + 1)][q];
#pragma unroll
      for (int j = 0; j < D; ++j)
#pragma unroll
        for (int q = 0; q < 2; ++q) buf[j][q] = t[j][q];
    }
    const bool ok = SUB == 0 || c * SPC + lane / LPS < h.n_stripes;
#pragma unroll
    for (int o = 0; o < C::p; ++o) {
      uint32_t pl[8];
#pragma unroll
      for (int q = 0; q < 8; ++q) pl[q] = acc[o * 8 + q];
      u32x4 v[2];
      unslice8(pl, v);
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const uint64_t o16 = off + j * S;
        if (mode != kCheck && ok) stv<true>(a.out[O0 + o] + o16, v[j]);
        if (mode != kStore) {
          const u32x4 w = ldv<true>(a.cmp[O0 + o] + o16);
          diff |= ok & ((w.x != v[j].x) | (w.y != v[j].y) | (w.z != v[j].z) | (w.w != v[j].w));
        }
      }
    }
    if (h.per_stripe && diff) {
      flag_mismatch(h.mismatch + (SUB ? c * SPC + lane / LPS : c / halves));
      diff = false;
    }
  }
  if (mode != kStore && diff) flag_mismatch(h.mismatch);
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
template <class C, bool NT, int NS, int I, uint32_t S = kBsBlock * 16>
__device__ __forceinline__ void recon_inputs(uint32_t (&acc)[NS * 16], u32x4 (&cur)[4],
                                             const BsReconArgs& a, uint64_t mask, uint64_t off) {
  if constexpr (I < C::k + NS) {
    if ((mask >> I) & 1u) {
      const uint64_t rest = mask >> (I + 1);
      u32x4 nxt[4];
      if (rest) load4<NT, S>(nxt, recon_ptr(a, C::k, I + 1 + __builtin_ctzll(rest)) + off);
      __builtin_amdgcn_sched_barrier(0);  // as in code_inputs (SB)
      uint32_t pl[16];
      slice<typename C::Field>(cur, pl);
      if constexpr (I < C::k) {
        // every sigma row, needed or not: straight-line XOR networks (a
        // branch per row costs more in register pressure than the XORs)
        mac_input<C, I, false>(acc, pl, make_int_seq<NS * 16>{});
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
    recon_inputs<C, NT, NS, I + 1, S>(acc, cur, a, mask, off);
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

// The per-(output, syndrome row) GF(2^8) tables of the run-time mixing, for
// one set of reconstruct arguments (all lanes; the caller synchronises).
template <class C, int NS>
__device__ __forceinline__ void recon_tables(const BsReconArgs& a, uint4* tq, uint32_t* tt2) {
  using F = typename C::Field;
  const uint32_t n_out = a.n_out;
  for (uint32_t t = threadIdx.x; t < n_out * NS; t += kBsBlock) {
    const uint32_t c = a.w[t / NS][t % NS];
    if constexpr (F::kPlanes == 8) {
      write_tab(tq, tt2, t, make_gf8_tab(c));
    } else {
      uint32_t sub[4];
      gf16_sub_coefs(c, sub);
#pragma unroll
      for (int q = 0; q < 4; ++q) write_tab(tq, tt2, t * 4 + q, make_gf8_tab(sub[q]));
    }
  }
}

// ---- bit-sliced run-time mixing -------------------------------------------
// A run-time constant c times sliced planes s, accumulated: c*s is the XOR of
// y_b = e_b * s over the set bits b of c, e_b the element with only bit b set.
// The y_b follow from s by compile-time maps: doubling every byte (xtime,
// generator polynomial 0x11D, build.rs:11) -- a renaming of the 8 planes of a
// byte plus 3 XORs -- and, for GF(2^16), one multiplication by x
// (galois_16.rs:146-162: x*(H x + L) = (2H + L) x + 128 H).  The bits of c are
// wave-uniform, so each selects its XORs with a scalar branch: ~half of c's
// 8/16 bits are set, each costing 16 planes of XOR (two bits per v_bitop3),
// with no tables, no v_perm and no un-slicing of the syndromes.

// y *= 2 in every byte (planes 8g..8g+7 are bits 0..7 of byte group g).
__device__ __forceinline__ void xtime_planes(uint32_t (&y)[16]) {
#pragma unroll
  for (int g = 0; g < 2; ++g) {
    uint32_t* b = y + 8 * g;
    const uint32_t t = b[7];
#pragma unroll
    for (int q = 7; q > 0; --q) b[q] = b[q - 1];
    b[0] = t;
    b[2] ^= t;
    b[3] ^= t;
    b[4] ^= t;
  }
}

// y = x * s for GF(2^16) planes (0..7: H = coefficient of x, 8..15: L).
__device__ __forceinline__ void mul_x_planes(const uint32_t (&s)[16], uint32_t (&y)[16]) {
  uint32_t h[16];
#pragma unroll
  for (int q = 0; q < 8; ++q) {
    h[q] = s[q];
    h[8 + q] = s[q];
  }
  xtime_planes(h);  // h[0..7] = 2H (h[8..15] = 2H too: the 128 H chain below starts there)
#pragma unroll
  for (int q = 0; q < 8; ++q) y[q] = h[q] ^ s[8 + q];
#pragma unroll
  for (int i = 0; i < 6; ++i) xtime_planes(h);  // h[8..15] = 2^7 H = 128 H
#pragma unroll
  for (int q = 0; q < 8; ++q) y[8 + q] = h[8 + q];
}

// out[g] ^= (bits b, b+1 of c[g]) selection of y0 = e_b s, y1 = e_{b+1} s.
template <int G>
__device__ __forceinline__ void mix_pair(uint32_t (&out)[G][16], const uint32_t (&c)[G], int b,
                                         const uint32_t (&y0)[16], const uint32_t (&y1)[16]) {
#pragma unroll
  for (int g = 0; g < G; ++g) {
    const uint32_t m = (c[g] >> b) & 3u;  // wave-uniform
    // (the pins keep each case a real branch: speculated into selects, the
    // three cases' temporaries would all be live at once and spill)
    if (m == 3u) {
#pragma unroll
      for (int q = 0; q < 16; ++q) {
        out[g][q] = xor3(out[g][q], y0[q], y1[q]);
        asm volatile("" : "+v"(out[g][q]));
      }
    } else if (m == 1u) {
#pragma unroll
      for (int q = 0; q < 16; ++q) {
        out[g][q] ^= y0[q];
        asm volatile("" : "+v"(out[g][q]));
      }
    } else if (m == 2u) {
#pragma unroll
      for (int q = 0; q < 16; ++q) {
        out[g][q] ^= y1[q];
        asm volatile("" : "+v"(out[g][q]));
      }
    }
  }
}

// out[g] ^= c[g] * s for G outputs at once (one y chain for all of them).
// Byte j of c: e_b = 2^(b - 8j) for j = 0 (GF(2^8), and GF(2^16)'s constant
// part), x * 2^(b - 8j) for j = 1.  A byte's 8 doublings rotate the planes
// back onto their registers, so the byte loop stays rolled (half the code)
// at no cost in moves, while the steps inside it are unrolled (a doubling is
// then a renaming plus 3 XORs per byte group).
template <class F, int G>
__device__ __forceinline__ void mix_row(uint32_t (&out)[G][16], const uint32_t (&c)[G],
                                        const uint32_t (&s)[16]) {
#pragma unroll 1
  for (int j = 0; j < F::kPlanes / 8; ++j) {
    uint32_t y0[16], y1[16];
    if (j == 0) {
#pragma unroll
      for (int q = 0; q < 16; ++q) y0[q] = s[q];
    } else {
      mul_x_planes(s, y0);
    }
    uint32_t cj[G];
#pragma unroll
    for (int g = 0; g < G; ++g) cj[g] = c[g] >> (8 * j);
#pragma unroll
    for (int b = 0; b < 8; b += 2) {
#pragma unroll
      for (int q = 0; q < 16; ++q) y1[q] = y0[q];
      xtime_planes(y1);
      mix_pair<G>(out, cj, b, y0, y1);
#pragma unroll
      for (int q = 0; q < 16; ++q) y0[q] = y1[q];
      xtime_planes(y0);
#pragma unroll
      for (int q = 0; q < 16; ++q) asm volatile("" : "+v"(y0[q]));
    }
  }
}

// The mixing of recon_chunk on sliced syndromes, outputs in groups of G
// (NS rows + G outputs + the y pair fit the VGPR budget at NS = 8); each
// output un-sliced once and stored.  A: BsReconArgs (kernarg or a per-stripe
// descriptor in memory: read uniform either way).
template <class C, bool NT, int NS, int G>
__device__ __forceinline__ void recon_mix_bitsliced(const BsReconArgs& a,
                                                    const uint32_t (&acc)[NS * 16], uint64_t off) {
  using F = typename C::Field;
  const uint32_t n_out = __builtin_amdgcn_readfirstlane(a.n_out);
  const uint32_t synd = __builtin_amdgcn_readfirstlane(a.synd);
#pragma unroll 1
  for (uint32_t o0 = 0; o0 < n_out; o0 += G) {
    uint32_t out[G][16];
#pragma unroll
    for (int g = 0; g < G; ++g)
#pragma unroll
      for (int q = 0; q < 16; ++q) out[g][q] = 0u;
#pragma unroll
    for (int r = 0; r < NS; ++r) {
      uint32_t c[G];
      uint32_t any = 0;
#pragma unroll
      for (int g = 0; g < G; ++g) {
        const uint32_t o = o0 + g;
        const bool live = o < n_out;
        // a missing parity output starts from its sigma row
        if (live && __builtin_amdgcn_readfirstlane(a.out_sigma[live ? o : 0]) == r) {
#pragma unroll
          for (int q = 0; q < 16; ++q) out[g][q] ^= acc[r * 16 + q];
        }
        c[g] = (live && ((synd >> r) & 1u)) ? __builtin_amdgcn_readfirstlane(a.w[live ? o : 0][r]) : 0u;
        any |= c[g];
      }
      if (any) {
        // a fresh copy per pass (the pin): otherwise LICM hoists the y chains
        // of every row out of the pass loop, NS x 16 more live VGPRs
        uint32_t s[16];
#pragma unroll
        for (int q = 0; q < 16; ++q) {
          s[q] = acc[r * 16 + q];
          asm volatile("" : "+v"(s[q]));
        }
        mix_row<F, G>(out, c, s);
      }
      // keep each row's work together (as recon_inputs does across inputs)
#pragma unroll
      for (int g = 0; g < G; ++g)
#pragma unroll
        for (int q = 0; q < 16; ++q) asm volatile("" : "+v"(out[g][q]));
    }
#pragma unroll
    for (int g = 0; g < G; ++g) {
      if (o0 + g >= n_out) break;
      u32x4 v[4];
      unslice<F>(out[g], v);
      uint8_t* dst = a.out[o0 + g];
#pragma unroll
      for (int j = 0; j < 4; ++j) stv<NT>(dst + off + j * (kBsBlock * 16), v[j]);
    }
  }
}

// The e x e mixing of a reconstruct kernel (RSE_OPT_RECON_MIX):
//  kReconMixTables  v_perm tables in LDS after un-slicing (round 1);
//  kReconMixChain   bit-sliced doubling chains above 4 syndrome rows, tables
//                   below (round 2: +11 % at 8 rows);
//  kReconMixHorner  bit-sliced Horner's rule (below), any number of rows.
//  kReconMixHorner4 the same, four steps per mask word unrolled (the step
//                   bytes by constant shifts, no 64-bit mask shifting or
//                   per-step loop control; A/B).
constexpr int kReconMixTables = 0, kReconMixChain = 1, kReconMixHorner = 2, kReconMixHorner4 = 3;
constexpr int kReconMixDefault = kReconMixHorner4;
constexpr bool recon_mix_tables(int ns, int mix) {
  return mix == kReconMixTables || (mix == kReconMixChain && ns <= 4);
}

// ---- Horner mixing (rse_kernels.hpp: the basis, BsReconArgs::hm) ----------
// Output o = sum_r w[o][r] s_r, evaluated by Horner's rule over the basis
// coordinates i (high to low) of the w[o][r]:
//   v = z * v ^ (XOR of the syndromes s_r whose w[o][r] has coordinate i)
// with the row set of step j in byte j of hm[o].  Multiplying by z moves plane
// q of a group to q + 1 and XORs the group's top plane into the taps; it is
// fused into the first row group's selection (new plane q = old plane q - 1
// ^ the selected sources, one v_bitop3).  For each pair of rows {2t, 2t + 1}
// the XOR d_t is precomputed, so a pair adds at most one source and a group
// of two pairs (a nibble of the step's mask) at most two: one op per plane
// per group, the nibble picking the case by a scalar branch.  No per-row y
// chains (the doubling chains of recon_mix_bitsliced) and one output live at
// a time: ~(NS / 4) x 16 + 4 ops per step, NB steps per output.
template <class F>
struct HornerF;
template <>
struct HornerF<BitsF8> {
  static constexpr int N = 8;  // planes per group = coordinates
  static constexpr uint32_t taps = kHornerTaps8;
};
template <>
struct HornerF<BitsF16> {
  static constexpr int N = 16;
  static constexpr uint32_t taps = kHornerTaps16;
};

// Plane masks of the GF(2^16) basis conversions (plane q <-> element bit q ^ 8).
constexpr uint64_t to_b_planes(int i) {  // z-coordinate plane i from element planes
  uint64_t m = 0;
  for (int j = 0; j < 16; ++j)
    if ((kHornerBasis16.to_b[i] >> j) & 1u) m |= 1ull << (j ^ 8);
  return m;
}
constexpr uint64_t from_b_planes(int q) {  // element plane q from z-coordinate planes
  return kHornerBasis16.from_b[q ^ 8];
}
template <int... I>
__device__ __forceinline__ void to_basis16(uint32_t* pl, int_seq<int, I...>) {
  uint32_t in[16];
#pragma unroll
  for (int q = 0; q < 16; ++q) in[q] = pl[q];
  ((pl[I] = xinit<to_b_planes(I)>(in)), ...);
}
template <int... I>
__device__ __forceinline__ void from_basis16(uint32_t* pl, int_seq<int, I...>) {
  uint32_t in[16];
#pragma unroll
  for (int q = 0; q < 16; ++q) in[q] = pl[q];
  ((pl[I] = xinit<from_b_planes(I)>(in)), ...);
}

// Source of pair P selected by SEL (1: row 2P, 2: row 2P + 1, 3: d_P), or none.
template <int SEL, int P, int NS>
constexpr bool h_has() {
  return (SEL == 1 && 2 * P < NS) || (SEL >= 2 && 2 * P + 1 < NS);
}
template <int SEL, int P, int NS, int ND>
__device__ __forceinline__ const uint32_t* h_src(const uint32_t (&s)[NS * 16],
                                                 const uint32_t (&d)[ND][16]) {
  if constexpr (SEL == 1 && 2 * P < NS) return &s[2 * P * 16];
  else if constexpr (SEL == 2 && 2 * P + 1 < NS) return &s[(2 * P + 1) * 16];
  else if constexpr (SEL == 3 && 2 * P + 1 < NS) return d[P];
  else return nullptr;
}

// v = (SH ? z * v : v) ^ the sources of nibble NIB of row group G.
template <class F, bool SH, int NIB, int G, int NS, int ND>
__device__ __forceinline__ void h_case(uint32_t (&v)[16], const uint32_t (&s)[NS * 16],
                                       const uint32_t (&d)[ND][16]) {
  constexpr int N = HornerF<F>::N;
  constexpr bool hasA = h_has<NIB & 3, 2 * G, NS>(), hasB = h_has<(NIB >> 2) & 3, 2 * G + 1, NS>();
  if constexpr (!SH && !hasA && !hasB) return;
  const uint32_t* A = h_src<NIB & 3, 2 * G, NS, ND>(s, d);
  const uint32_t* B = h_src<(NIB >> 2) & 3, 2 * G + 1, NS, ND>(s, d);
  uint32_t n[16];
#pragma unroll
  for (int q = 0; q < 16; ++q) {
    const int i = q % N;
    uint32_t t[4];
    int c = 0;
    t[c++] = SH ? v[i == 0 ? q + N - 1 : q - 1] : v[q];
    if (SH && ((HornerF<F>::taps >> i) & 1u)) t[c++] = v[q - i + N - 1];
    if constexpr (hasA) t[c++] = A[q];
    if constexpr (hasB) t[c++] = B[q];
    uint32_t x = t[0];
    if (c == 2) x ^= t[1];
    if (c >= 3) x = xor3(x, t[1], t[2]);
    if (c == 4) x ^= t[3];
    n[q] = x;
  }
#pragma unroll
  for (int q = 0; q < 16; ++q) {
    v[q] = n[q];
    asm volatile("" : "+v"(v[q]));  // a real branch per case, not selects
  }
}

// The case of a nibble: a switch.  (An opaque binary tree of uniform
// branches instead -- 4 tests a step against the switch's structurized flag
// chain -- measured the same, 4.09 vs 4.08 TB/s at 8 lost, profiles/r03/s11/.)
template <class F, bool SH, int G, int NS, int ND>
__device__ __forceinline__ void h_group(uint32_t (&v)[16], const uint32_t (&s)[NS * 16],
                                        const uint32_t (&d)[ND][16], uint32_t nib) {
#define RSE_HCASE(n) \
  case n:            \
    h_case<F, SH, n, G, NS, ND>(v, s, d); \
    break;
  switch (nib) {
    RSE_HCASE(0) RSE_HCASE(1) RSE_HCASE(2) RSE_HCASE(3)
    RSE_HCASE(4) RSE_HCASE(5) RSE_HCASE(6) RSE_HCASE(7)
    RSE_HCASE(8) RSE_HCASE(9) RSE_HCASE(10) RSE_HCASE(11)
    RSE_HCASE(12) RSE_HCASE(13) RSE_HCASE(14) RSE_HCASE(15)
    default: break;
  }
#undef RSE_HCASE
}

// The mixing of recon_chunk by Horner's rule on the sliced rows acc (converted
// in place to the basis for GF(2^16)); each output un-sliced once and stored.
template <class C, bool NT, int NS, uint32_t S = kBsBlock * 16, bool U4 = false>
__device__ __forceinline__ void recon_mix_horner(const BsReconArgs& a, uint32_t (&acc)[NS * 16],
                                                 uint64_t off) {
  using F = typename C::Field;
  constexpr int NB = HornerF<F>::N;
  constexpr int ND = NS / 2 > 0 ? NS / 2 : 1;
  const uint32_t n_out = __builtin_amdgcn_readfirstlane(a.n_out);
  const uint32_t sigma = __builtin_amdgcn_readfirstlane(a.sigma);
  if constexpr (NB == 16) {
#pragma unroll
    for (int r = 0; r < NS; ++r)
      if ((sigma >> r) & 1u) to_basis16(&acc[r * 16], make_int_seq<16>{});
  }
  uint32_t d[ND][16];
#pragma unroll
  for (int t = 0; t < NS / 2; ++t)
#pragma unroll
    for (int q = 0; q < 16; ++q) d[t][q] = acc[2 * t * 16 + q] ^ acc[(2 * t + 1) * 16 + q];
#pragma unroll 1
  for (uint32_t o = 0; o < n_out; ++o) {
    // (readfirstlane returns int: widen through uint32_t, not sign-extended)
    auto word = [&](int q) { return (uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane(a.hm[o][q]); };
    uint64_t lo = word(0) | word(1) << 32;
    uint64_t hi = word(2) | word(3) << 32;
    uint32_t v[16];
#pragma unroll
    for (int q = 0; q < 16; ++q) v[q] = 0u;
    // (the fused shift writes a second register set; the case joins cost
    // 8 v_mov_b64 per step to move it back -- a tied in-place asm form and a
    // one-step lag of rows 4..7 were probed and the copies stayed)
    if constexpr (U4) {
#pragma unroll 1
      for (int w = 0; w < NB / 4; ++w) {
        const uint32_t word = (uint32_t)__builtin_amdgcn_readfirstlane(a.hm[o][w]);
#pragma unroll
        for (int b = 0; b < 4; ++b) {
          const uint32_t m = (word >> (8 * b)) & 0xFFu;
          h_group<F, true, 0, NS, ND>(v, acc, d, m & 15u);
          if constexpr (NS > 4) h_group<F, false, 1, NS, ND>(v, acc, d, m >> 4);
        }
      }
    } else {
#pragma unroll 1
      for (int j = 0; j < NB; ++j) {
        const uint32_t m = (uint32_t)lo & 0xFFu;
        lo = (lo >> 8) | (hi << 56);
        hi >>= 8;
        h_group<F, true, 0, NS, ND>(v, acc, d, m & 15u);
        if constexpr (NS > 4) h_group<F, false, 1, NS, ND>(v, acc, d, m >> 4);
      }
    }
    const int32_t os = __builtin_amdgcn_readfirstlane(a.out_sigma[o]);
#pragma unroll
    for (int r = 0; r < NS; ++r)
      if (os == r) {
#pragma unroll
        for (int q = 0; q < 16; ++q) v[q] ^= acc[r * 16 + q];
      }
    if constexpr (NB == 16) from_basis16(v, make_int_seq<16>{});
    u32x4 x[4];
    unslice<F>(v, x);
    uint8_t* dst = a.out[o];
#pragma unroll
    for (int j = 0; j < 4; ++j) stv<NT>(dst + off + j * S, x[j]);
  }
}

// One 16 KiB chunk of one stripe: off is the lane's byte offset from the
// argument block's shard pointers.  MIX: the e x e mixing (kReconMix*).
// S: bytes between a lane's 4 vectors (4 KiB: a 256-lane workgroup per 16 KiB
// chunk; 1 KiB: each wave its own 4 KiB chunk -- Horner mixing only).
template <class C, bool NT, int NS, int MIX, uint32_t S = kBsBlock * 16>
__device__ __forceinline__ void recon_chunk(const BsReconArgs& a, const uint4* tq,
                                            const uint32_t* tt2, uint64_t off) {
  static_assert(S == kBsBlock * 16 || MIX >= kReconMixHorner, "4 KiB chunks: Horner mixing");
  using F = typename C::Field;
  const uint32_t n_out = a.n_out;
  const uint64_t mask = recon_mask(a, C::k);
  const int first = __builtin_ctzll(mask);  // host / planner guarantee mask != 0
  uint32_t acc[NS * 16];
#pragma unroll
  for (int q = 0; q < NS * 16; ++q) acc[q] = 0u;
  u32x4 cur[4];
  load4<NT, S>(cur, recon_ptr(a, C::k, first) + off);
  recon_inputs<C, NT, NS, 0, S>(acc, cur, a, mask, off);
  if constexpr (MIX == kReconMixHorner || MIX == kReconMixHorner4) {
    recon_mix_horner<C, NT, NS, S, MIX == kReconMixHorner4>(a, acc, off);
    return;
  } else if constexpr (!recon_mix_tables(NS, MIX)) {  // the mixing on the sliced syndromes
    // outputs per pass: NS rows + G outputs + the y pair within the VGPR
    // budget of the launch bounds (3 waves/SIMD up to NS = 2, else 2)
    recon_mix_bitsliced<C, NT, NS, (NS <= 4 ? NS : 2)>(a, acc, off);  // (probed: G = 4 at NS = 8 spills)
    return;
  }
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

template <int NS, class F>
struct ReconLds {
  static constexpr int kTabs = kMaxOut * NS * (F::kPlanes == 16 ? 4 : 1);
};

// Reconstruct body: one argument block for every stripe of the launch.
// Launch bounds: kBsBlock lanes, NS > 4 ? 2 : 3 waves/SIMD.
template <class C, bool NT, int NS, int MIX>
__device__ __forceinline__ void bitslice_recon_body(const BsReconArgs& a,
                                                    uint64_t chunks_per_stripe) {
  const uint64_t total = chunks_per_stripe * a.n_stripes;
  if constexpr (!recon_mix_tables(NS, MIX)) {
    for (uint64_t idx = blockIdx.x; idx < total; idx += gridDim.x) {
      const uint64_t stripe = idx / chunks_per_stripe, chunk = idx - stripe * chunks_per_stripe;
      recon_chunk<C, NT, NS, MIX>(a, nullptr, nullptr,
                                  stripe * a.stripe_stride + chunk * kBsChunk + threadIdx.x * 16u);
    }
    return;
  }
  constexpr int T = ReconLds<NS, typename C::Field>::kTabs;
  __shared__ uint4 tq[T];
  __shared__ uint32_t tt2[T];
  recon_tables<C, NS>(a, tq, tt2);
  __syncthreads();
  for (uint64_t idx = blockIdx.x; idx < total; idx += gridDim.x) {
    const uint64_t stripe = idx / chunks_per_stripe, chunk = idx - stripe * chunks_per_stripe;
    recon_chunk<C, NT, NS, MIX>(a, tq, tt2,
                                stripe * a.stripe_stride + chunk * kBsChunk + threadIdx.x * 16u);
  }
}

// bitslice_recon_body (one erasure pattern for every stripe) over whole 4 KiB
// chunks, one per wave, from byte `base` of every shard on: shards of 4 to 16
// KiB, and the rest of longer ones past their 16 KiB chunks.  chunks_per_stripe
// counts 4 KiB chunks.  Horner mixing.
template <class C, bool NT, int NS>
__device__ __forceinline__ void bitslice_recon_body_w4(const BsReconArgs& a,
                                                       uint64_t chunks_per_stripe, uint64_t base) {
  const uint64_t total = chunks_per_stripe * a.n_stripes;
  const uint32_t sub = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);  // wave-uniform
  const uint32_t lane_off = (threadIdx.x & 63u) * 16u;
  for (uint64_t idx = (uint64_t)blockIdx.x * 4 + sub; idx < total; idx += (uint64_t)gridDim.x * 4) {
    const uint64_t stripe = idx / chunks_per_stripe, chunk = idx - stripe * chunks_per_stripe;
    recon_chunk<C, NT, NS, kReconMixHorner, 1024u>(
        a, nullptr, nullptr, stripe * a.stripe_stride + base + chunk * 4096u + lane_off);
  }
}

// bitslice_recon_desc_body over whole 4 KiB chunks, one per wave (lane l
// codes vectors l, l + 64, l + 128, l + 192 of its wave's chunk), for shards
// -- or the rest of shards past their 16 KiB chunks, from byte `base` on --
// shorter than 16 KiB: reconstruct_batch of small shards at bit-sliced speed.
// chunks_per_stripe counts 4 KiB chunks.  Horner mixing.
template <class C, bool NT, int NS>
__device__ __forceinline__ void bitslice_recon_desc_body_w4(const BsReconArgs* __restrict__ descs,
                                                            uint64_t chunks_per_stripe,
                                                            uint64_t n_stripes, uint64_t base);

// A stripe's descriptor through the constant address space: the planner wrote
// it before this kernel, nothing writes it during, so its fields can be scalar
// loads (through a generic pointer they were vector loads + readfirstlane).
__device__ __forceinline__ const BsReconArgs& desc_at(const BsReconArgs* descs, uint64_t s) {
  using CPtr = const __attribute__((address_space(4))) BsReconArgs*;
  return *(const BsReconArgs*)((CPtr)descs + s);
}

// Reconstruct body over per-stripe argument blocks (descs[s], written by the
// device planner of rse_reconstruct_batch: every stripe its own erasure
// pattern).  A workgroup rebuilds its mixing tables when its stripe changes.
template <class C, bool NT, int NS, int MIX = kReconMixDefault>
__device__ __forceinline__ void bitslice_recon_desc_body(const BsReconArgs* __restrict__ descs,
                                                         uint64_t chunks_per_stripe,
                                                         uint64_t n_stripes) {
  if constexpr (!recon_mix_tables(NS, MIX)) {
    const uint64_t total = chunks_per_stripe * n_stripes;
    for (uint64_t idx = blockIdx.x; idx < total; idx += gridDim.x) {
      const uint64_t stripe = idx / chunks_per_stripe, chunk = idx - stripe * chunks_per_stripe;
      const BsReconArgs& a = desc_at(descs, stripe);
      if (a.n_out == 0) continue;  // uniform: nothing to rebuild in this stripe
      recon_chunk<C, NT, NS, MIX>(a, nullptr, nullptr, chunk * kBsChunk + threadIdx.x * 16u);
    }
    return;
  }
  constexpr int T = ReconLds<NS, typename C::Field>::kTabs;
  __shared__ uint4 tq[T];
  __shared__ uint32_t tt2[T];
  uint64_t built = ~0ull;
  const uint64_t total = chunks_per_stripe * n_stripes;
  for (uint64_t idx = blockIdx.x; idx < total; idx += gridDim.x) {
    const uint64_t stripe = idx / chunks_per_stripe, chunk = idx - stripe * chunks_per_stripe;
    const BsReconArgs& a = desc_at(descs, stripe);
    if (a.n_out == 0) continue;  // uniform: nothing to rebuild in this stripe
    if (stripe != built) {
      __syncthreads();  // every lane is done with the previous stripe's tables
      recon_tables<C, NS>(a, tq, tt2);
      __syncthreads();
      built = stripe;
    }
    recon_chunk<C, NT, NS, MIX>(a, tq, tt2, chunk * kBsChunk + threadIdx.x * 16u);
  }
}

// ---- deeper input pipeline (RSE_OPT_RECON_DEPTH) ----------------------------
// recon_inputs with D inputs in flight per lane: at input index I the loads of
// index I + D are issued (if that input is read), into a ring of D + 1 slots
// indexed at compile time by the input INDEX, so the ring stays in VGPRs
// whatever the erasure pattern (an absent index just leaves its slot unused,
// so the depth in inputs actually read is at most D).  Past the chunk's last
// index the loads continue into the first X indices of the workgroup's next
// chunk (next_off, ~0 if none), so the e x e mixing overlaps them.  Why: one
// 16 KiB input in flight per 256-lane workgroup, two workgroups per CU at
// NS = 8, is ~8 MiB over the chip -- at ~2 us of loaded HBM latency a read
// cap near 4 TB/s (Little's law), while the mixing phase has no loads in
// flight at all.
template <class C, bool NT, int NS, int D, int X, int I>
__device__ __forceinline__ void recon_inputs_deep(uint32_t (&acc)[NS * 16], u32x4 (&buf)[D + 1][4],
                                                  const BsReconArgs& a, uint64_t mask,
                                                  uint64_t off, uint64_t next_off) {
  constexpr int N = C::k + NS;
  if constexpr (I < N) {
    constexpr int J = I + D;
    if constexpr (J < N) {
      if ((mask >> J) & 1u) load4<NT>(buf[J % (D + 1)], recon_ptr(a, C::k, J) + off);
    } else if constexpr (J - N < X) {
      if (next_off != ~0ull && ((mask >> (J - N)) & 1u))
        load4<NT>(buf[J % (D + 1)], recon_ptr(a, C::k, J - N) + next_off);
    }
    __builtin_amdgcn_sched_barrier(0);
    if ((mask >> I) & 1u) {
      uint32_t pl[16];
      slice<typename C::Field>(buf[I % (D + 1)], pl);
      if constexpr (I < C::k) {
        mac_input<C, I, false>(acc, pl, make_int_seq<NS * 16>{});
      } else {
#pragma unroll
        for (int q = 0; q < 16; ++q) acc[(I - C::k) * 16 + q] ^= pl[q];
      }
#pragma unroll
      for (int q = 0; q < NS * 16; ++q) asm volatile("" : "+v"(acc[q]));
    }
    recon_inputs_deep<C, NT, NS, D, X, I + 1>(acc, buf, a, mask, off, next_off);
  }
}

// Loads of the first min(D, X') input indices of a chunk (X' = D for the
// first chunk of a workgroup, when nothing was prefetched).
template <class C, bool NT, int NS, int D>
__device__ __forceinline__ void recon_prime(u32x4 (&buf)[D + 1][4], const BsReconArgs& a,
                                            uint64_t mask, uint64_t off, int from) {
#pragma unroll
  for (int j = 0; j < D; ++j)
    if (j >= from && j < C::k + NS && ((mask >> j) & 1u))
      load4<NT>(buf[j], recon_ptr(a, C::k, j) + off);
}

// recon_chunk with the deeper pipeline: buf holds the loads of this chunk's
// first indices on entry and, when next_off != ~0, of the next chunk's first X
// indices on return (moved to slots 0..X-1).
template <class C, bool NT, int NS, int MIX, int D, int X>
__device__ __forceinline__ void recon_chunk_deep(const BsReconArgs& a, const uint4* tq,
                                                 const uint32_t* tt2, uint64_t off,
                                                 uint64_t next_off, u32x4 (&buf)[D + 1][4]) {
  static_assert(MIX == kReconMixHorner, "the deeper pipeline is for Horner mixing");
  constexpr int N = C::k + NS;
  const uint64_t mask = recon_mask(a, C::k);
  uint32_t acc[NS * 16];
#pragma unroll
  for (int q = 0; q < NS * 16; ++q) acc[q] = 0u;
  recon_inputs_deep<C, NT, NS, D, X, 0>(acc, buf, a, mask, off, next_off);
  if constexpr (N % (D + 1) != 0) {
    if (next_off != ~0ull) {
      u32x4 t[X][4];
#pragma unroll
      for (int j = 0; j < X; ++j)
#pragma unroll
        for (int q = 0; q < 4; ++q) t[j][q] = buf[(N + j) % (D + 1)][q];
#pragma unroll
      for (int j = 0; j < X; ++j)
#pragma unroll
        for (int q = 0; q < 4; ++q) buf[j][q] = t[j][q];
    }
  }
  recon_mix_horner<C, NT, NS>(a, acc, off);
}

// bitslice_recon_body with the deeper pipeline (one argument block for every
// stripe: the next chunk has the same pattern, so the cross-chunk loads apply).
template <class C, bool NT, int NS, int D>
__device__ __forceinline__ void bitslice_recon_body_deep(const BsReconArgs& a,
                                                         uint64_t chunks_per_stripe) {
  constexpr int X = 1;  // the mixing's registers leave room for one input (NS = 8: 240 VGPRs)
  const uint64_t total = chunks_per_stripe * a.n_stripes;
  const uint64_t mask = recon_mask(a, C::k);
  auto chunk_off = [&](uint64_t idx) {
    const uint64_t stripe = idx / chunks_per_stripe, chunk = idx - stripe * chunks_per_stripe;
    return stripe * a.stripe_stride + chunk * kBsChunk + threadIdx.x * 16u;
  };
  u32x4 buf[D + 1][4];
  if (blockIdx.x < total) recon_prime<C, NT, NS, D>(buf, a, mask, chunk_off(blockIdx.x), 0);
  for (uint64_t idx = blockIdx.x; idx < total; idx += gridDim.x) {
    const uint64_t nidx = idx + gridDim.x;
    const uint64_t next_off = nidx < total ? chunk_off(nidx) : ~0ull;
    recon_chunk_deep<C, NT, NS, kReconMixHorner, D, X>(a, nullptr, nullptr, chunk_off(idx),
                                                       next_off, buf);
    if (next_off != ~0ull) recon_prime<C, NT, NS, D>(buf, a, mask, next_off, X);
  }
}

// bitslice_recon_desc_body with the deeper pipeline inside each chunk (the
// next chunk is usually another stripe's, with its own descriptor: no
// cross-chunk loads).
template <class C, bool NT, int NS, int D>
__device__ __forceinline__ void bitslice_recon_desc_body_deep(const BsReconArgs* __restrict__ descs,
                                                              uint64_t chunks_per_stripe,
                                                              uint64_t n_stripes) {
  const uint64_t total = chunks_per_stripe * n_stripes;
  for (uint64_t idx = blockIdx.x; idx < total; idx += gridDim.x) {
    const uint64_t stripe = idx / chunks_per_stripe, chunk = idx - stripe * chunks_per_stripe;
    const BsReconArgs& a = desc_at(descs, stripe);
    if (a.n_out == 0) continue;  // uniform: nothing to rebuild in this stripe
    const uint64_t off = chunk * kBsChunk + threadIdx.x * 16u;
    u32x4 buf[D + 1][4];
    recon_prime<C, NT, NS, D>(buf, a, recon_mask(a, C::k), off, 0);
    recon_chunk_deep<C, NT, NS, kReconMixHorner, D, 1>(a, nullptr, nullptr, off, ~0ull, buf);
  }
}

template <class C, bool NT, int NS>
__device__ __forceinline__ void bitslice_recon_desc_body_w4(const BsReconArgs* __restrict__ descs,
                                                            uint64_t chunks_per_stripe,
                                                            uint64_t n_stripes, uint64_t base) {
  const uint64_t total = chunks_per_stripe * n_stripes;
  const uint32_t sub = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);  // wave-uniform
  const uint32_t lane_off = (threadIdx.x & 63u) * 16u;
  for (uint64_t idx = (uint64_t)blockIdx.x * 4 + sub; idx < total; idx += (uint64_t)gridDim.x * 4) {
    const uint64_t stripe = idx / chunks_per_stripe, chunk = idx - stripe * chunks_per_stripe;
    const BsReconArgs& a = desc_at(descs, stripe);
    if (a.n_out == 0) continue;  // uniform: nothing to rebuild in this stripe
    recon_chunk<C, NT, NS, kReconMixHorner, 1024u>(a, nullptr, nullptr,
                                                   base + chunk * 4096u + lane_off);
  }
}

// ---- 8 sigma rows on wave pairs (RSE_OPT_RECON_PAIRS) ----------------------
// At NS = 8 one wave holds 128 VGPRs of syndromes and, in the mixing, 64 of
// pair XORs: 2 waves per SIMD, and the mixing phase (half the VALU work of an
// 8-erasure chunk) has no loads in flight.  Here two waves share one 4 KiB
// column of every shard: wave H of the pair accumulates sigma rows 4H..4H+3
// only (64 VGPRs), so 3 waves fit per SIMD.
//  * Data inputs: wave H loads and slices the present data shards of index
//    parity H and passes their planes to its partner through LDS (one barrier
//    per index pair); both code every data input into their own rows.
//  * Syndrome inputs: each wave loads the parity shards of its own rows.
//  * Mixing: output o = sum_r w[o][r] s_r splits into the two waves' partial
//    sums over their rows, each by Horner's rule over 4 rows (one nibble of the
//    step mask per step, 19 ops).  A wave computes its partner's outputs'
//    partials into LDS, then its own, adds the partner's, converts, un-slices
//    and stores (outputs split in halves).
// A workgroup of P pairs (2P waves) takes a unit of P 4 KiB columns; the
// barriers then sync P pairs (P = 1: only the pair itself).
constexpr int kPairRows = 4;
template <int P>
struct PairLds {
  u32x4 v[2][P][2][4][64];  // [buffer][pair][role][vector][lane]: 16 KiB per pair
};

template <class C, int I, int R0, int... OP>
__device__ __forceinline__ void mac_rows(uint32_t (&acc)[kPairRows * 16], const uint32_t (&pl)[16],
                                         int_seq<int, OP...>) {
  if constexpr (C::kGTemps > 0) {
#pragma unroll
    for (int g = 0; g < 2; ++g) {
      uint32_t src[8 + C::kGTemps];
#pragma unroll
      for (int q = 0; q < 8; ++q) src[q] = pl[g * 8 + q];
#pragma unroll
      for (int t = 0; t < C::kGTemps; ++t)
        if (t < C::planes.ntmp[I]) src[8 + t] = temp_source<C, I>(src, t);
      // OP < 32: row OP / 8, plane OP % 8 of group g
      if (g == 0)
        ((acc[(OP / 8) * 16 + OP % 8] =
              xacc<C::planes.sel[R0 + OP / 8][I][OP % 8]>(acc[(OP / 8) * 16 + OP % 8], src)),
         ...);
      else
        ((acc[(OP / 8) * 16 + 8 + OP % 8] =
              xacc<C::planes.sel[R0 + OP / 8][I][OP % 8]>(acc[(OP / 8) * 16 + 8 + OP % 8], src)),
         ...);
    }
  } else {
    uint32_t in[16 + C::kTemps];
#pragma unroll
    for (int q = 0; q < 16; ++q) in[q] = pl[q];
    if constexpr (C::kTemps > 0) {
#pragma unroll
      for (int t = 0; t < C::kTemps; ++t)
        if (t < C::planes.ntmp[I]) in[16 + t] = temp_source<C, I>(in, t);
    }
    ((acc[OP] = xacc<C::planes.sel[R0 + OP / 16][I][OP % C::NP]>(acc[OP],
                                                                  in + (OP % 16) / C::NP * C::NP)),
     ...);
  }
}

template <class C, int I, int R0>
__device__ __forceinline__ void mac_rows(uint32_t (&acc)[kPairRows * 16], const uint32_t (&pl)[16]) {
  if constexpr (I < C::k) {
    if constexpr (C::kGTemps > 0) mac_rows<C, I, R0>(acc, pl, make_int_seq<kPairRows * 8>{});
    else mac_rows<C, I, R0>(acc, pl, make_int_seq<kPairRows * 16>{});
  }
}

// The wave's next own input after index J (own: bit set in `own`; bits < k
// data shards, k + r parity row r), loaded into nxt; returns whether there is one.
template <class C, bool NT>
__device__ __forceinline__ bool pair_prefetch(u32x4 (&nxt)[4], const BsReconArgs& a, uint64_t own,
                                              int J, uint64_t off) {
  const uint64_t rest = own & ~((2ull << J) - 1ull);
  if (!rest) return false;
  load4<NT, 1024u>(nxt, recon_ptr(a, C::k, (uint32_t)__builtin_ctzll(rest)) + off);
  return true;
}

// The wave's own input two after index J, loaded into nxt (the depth-2
// pipeline, DBG 4); returns whether there is one.
template <class C, bool NT>
__device__ __forceinline__ bool pair_prefetch2(u32x4 (&nxt)[4], const BsReconArgs& a, uint64_t own,
                                               int J, uint64_t off) {
  uint64_t rest = own & ~((2ull << J) - 1ull);
  if (!rest) return false;
  rest &= rest - 1ull;
  if (!rest) return false;
  load4<NT, 1024u>(nxt, recon_ptr(a, C::k, (uint32_t)__builtin_ctzll(rest)) + off);
  return true;
}

// One own input of the wave: the next load(s) issued, then cur sliced into
// pl.  Depth 1: the next own input into nxt, then cur = nxt.  Depth 2 (DBG
// 4): nx1 already holds the next one in flight; the one after it is issued,
// then cur = nx1, nx1 = it.
template <class C, bool NT, int DBG>
__device__ __forceinline__ void pair_advance(u32x4 (&cur)[4], u32x4 (&nx1)[4], uint32_t (&pl)[16],
                                             const BsReconArgs& a, uint64_t own, int J, uint64_t off) {
  if constexpr (DBG == 4) {
    u32x4 nx2[4];
    const bool more2 = pair_prefetch2<C, NT>(nx2, a, own, J, off);
    __builtin_amdgcn_sched_barrier(0);
    slice<typename C::Field>(cur, pl);
#pragma unroll
    for (int j = 0; j < 4; ++j) cur[j] = nx1[j];
    if (more2) {
#pragma unroll
      for (int j = 0; j < 4; ++j) nx1[j] = nx2[j];
    }
  } else {
    u32x4 nxt[4];
    const bool more = pair_prefetch<C, NT>(nxt, a, own, J, off);
    __builtin_amdgcn_sched_barrier(0);
    slice<typename C::Field>(cur, pl);
    if (more) {
#pragma unroll
      for (int j = 0; j < 4; ++j) cur[j] = nxt[j];
    }
  }
}

// Data rounds T.. : indices 2T (role 0) and 2T + 1 (role 1).
// DBG (tune-only A/B variants, results not valid): 1 skips the Horner steps of
// the mixing, 2 the data inputs' networks (mac_rows) -- to split the kernel's
// time between its phases.
template <class C, bool NT, int H, int T, int P, int DBG = 0>
__device__ __forceinline__ void pair_data(uint32_t (&acc)[kPairRows * 16], u32x4 (&cur)[4],
                                          u32x4 (&nx1)[4],
                                          const BsReconArgs& a, uint64_t own, uint32_t present,
                                          uint64_t off, u32x4 (*mine)[64], u32x4 (*theirs)[64],
                                          uint32_t lane, uint32_t& buf) {
  if constexpr (2 * T < C::k) {
    constexpr int J = 2 * T + H, JP = 2 * T + 1 - H;
    const bool has_own = J < C::k && ((present >> J) & 1u);
    const bool has_oth = JP < C::k && ((present >> JP) & 1u);
    if (has_own || has_oth) {  // workgroup-uniform (one pattern per unit)
      uint32_t pl[16];
      // buffer `buf` of this wave's / the partner's slot: [buf][pair][role][4][64]
      u32x4* const wr = mine[buf * (P * 2 * 4)];
      const u32x4* const rd = theirs[buf * (P * 2 * 4)];
      if (has_own) {
        pair_advance<C, NT, DBG>(cur, nx1, pl, a, own, J, off);
#pragma unroll
        for (int j = 0; j < 4; ++j)
          wr[j * 64 + lane] = (u32x4){pl[4 * j], pl[4 * j + 1], pl[4 * j + 2], pl[4 * j + 3]};
      }
      __syncthreads();
      if (DBG != 2 && has_own) mac_rows<C, J, H * kPairRows>(acc, pl);
      if (DBG != 2 && has_oth) {
        uint32_t pp[16];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const u32x4 x = rd[j * 64 + lane];
          pp[4 * j] = x[0];
          pp[4 * j + 1] = x[1];
          pp[4 * j + 2] = x[2];
          pp[4 * j + 3] = x[3];
        }
        mac_rows<C, JP, H * kPairRows>(acc, pp);
      }
#pragma unroll
      for (int q = 0; q < kPairRows * 16; ++q) asm volatile("" : "+v"(acc[q]));
      buf ^= 1u;
    }
    pair_data<C, NT, H, T + 1, P, DBG>(acc, cur, nx1, a, own, present, off, mine, theirs, lane, buf);
  }
}

// The partial sum over the wave's rows of output o (Horner's rule, 4 rows),
// plus its sigma row if that is one of them.
template <class C, int H, int DBG = 0>
__device__ __forceinline__ void pair_partial(const BsReconArgs& a, uint32_t o,
                                             const uint32_t (&acc)[kPairRows * 16],
                                             const uint32_t (&d)[2][16], uint32_t (&v)[16]) {
  using F = typename C::Field;
  constexpr int NB = HornerF<F>::N;
#pragma unroll
  for (int q = 0; q < 16; ++q) v[q] = 0u;
#pragma unroll 1
  for (int w = 0; w < (DBG == 1 ? 0 : NB / 4); ++w) {
    const uint32_t word = (uint32_t)__builtin_amdgcn_readfirstlane(a.hm[o][w]);
#pragma unroll
    for (int b = 0; b < 4; ++b) {
      const uint32_t m = (word >> (8 * b)) & 0xFFu;
      h_group<F, true, 0, kPairRows, 2>(v, acc, d, H ? (m >> 4) : (m & 15u));
    }
  }
  const int32_t os = __builtin_amdgcn_readfirstlane(a.out_sigma[o]) - H * kPairRows;
#pragma unroll
  for (int r = 0; r < kPairRows; ++r)
    if (os == r) {
#pragma unroll
      for (int q = 0; q < 16; ++q) v[q] ^= acc[r * 16 + q];
    }
}

// One unit of one stripe for wave H of pair `pair`: off = the lane's byte
// offset (the pair's 4 KiB column + lane * 16) from the argument block's shard
// pointers.  cur holds the unit's first own input if `primed`; with next_off
// != ~0 (the workgroup's next unit, same argument block) that unit's first own
// input is loaded into cur before the mixing, so the mixing overlaps it, and
// the call returns true.
template <bool PF, class T>
__device__ __forceinline__ T& pick_ref(T& io, T& local) {
  if constexpr (PF) return io;
  else return local;
}
template <class C, bool NT, int H, int P, bool PF = false, int DBG = 0>
__device__ __forceinline__ bool recon_pair_unit(const BsReconArgs& a, uint64_t off,
                                                PairLds<P>& lds, uint32_t pair, uint32_t lane,
                                                u32x4 (&cur_io)[4], bool primed, uint64_t next_off) {
  // without the prefetch the unit's vectors are its own (nothing the compiler
  // must keep across units: 141 VGPRs, not 168 with 5 spilled)
  u32x4 cur_local[4];
  u32x4(&cur)[4] = pick_ref<PF>(cur_io, cur_local);
  if constexpr (!PF) {
    primed = false;
    next_off = ~0ull;
  }
  using F = typename C::Field;
  constexpr int R0 = H * kPairRows;
  const uint32_t present = a.present;
  const uint32_t synd = a.synd, sigma = a.sigma;
  const uint32_t n_out = __builtin_amdgcn_readfirstlane(a.n_out);
  // own inputs: data shards of index parity H, then the parity shards of own
  // syndrome rows
  const uint64_t par_mask = H ? 0xAAAAAAAAull : 0x55555555ull;
  const uint64_t own = ((uint64_t)present & par_mask) |
                       ((uint64_t)((synd >> R0) & 0xFu) << (C::k + R0));
  uint32_t acc[kPairRows * 16];
#pragma unroll
  for (int q = 0; q < kPairRows * 16; ++q) acc[q] = 0u;
  u32x4 nx1[4];  // depth 2 (DBG 4): the own input after cur, in flight
  if (own && !primed)
    load4<NT, 1024u>(cur, recon_ptr(a, C::k, (uint32_t)__builtin_ctzll(own)) + off);
  if constexpr (DBG == 4) {
    const uint64_t rest = own & (own - 1ull);
    if (rest) load4<NT, 1024u>(nx1, recon_ptr(a, C::k, (uint32_t)__builtin_ctzll(rest)) + off);
  }
  uint32_t buf = 0;
  u32x4(*mine)[64] = lds.v[0][pair][H];
  u32x4(*theirs)[64] = lds.v[0][pair][1 - H];
  pair_data<C, NT, H, 0, P, DBG>(acc, cur, nx1, a, own, present, off, mine, theirs, lane, buf);
  // own syndrome rows: s_r = sigma_r ^ parity_r
#pragma unroll
  for (int i = 0; i < kPairRows; ++i) {
    const int J = C::k + R0 + i;
    if ((own >> J) & 1u) {
      uint32_t pl[16];
      pair_advance<C, NT, DBG>(cur, nx1, pl, a, own, J, off);
#pragma unroll
      for (int q = 0; q < 16; ++q) acc[i * 16 + q] ^= pl[q];
    }
  }
  const bool prime = own && next_off != ~0ull;
  if (prime) load4<NT, 1024u>(cur, recon_ptr(a, C::k, (uint32_t)__builtin_ctzll(own)) + next_off);
  if constexpr (HornerF<F>::N == 16) {
#pragma unroll
    for (int r = 0; r < kPairRows; ++r)
      if ((sigma >> (R0 + r)) & 1u) to_basis16(&acc[r * 16], make_int_seq<16>{});
  }
  uint32_t d[2][16];
#pragma unroll
  for (int t = 0; t < 2; ++t)
#pragma unroll
    for (int q = 0; q < 16; ++q) d[t][q] = acc[2 * t * 16 + q] ^ acc[(2 * t + 1) * 16 + q];
  // outputs [0, half) are role 0's, [half, n_out) role 1's; exchange rounds of
  // two outputs a wave through the same LDS (the partner may still be reading
  // the last data round's planes: one barrier first)
  const uint32_t half = (n_out + 1) / 2;
  const uint32_t mine0 = H * half, theirs0 = (1 - H) * half;
  __syncthreads();
#pragma unroll 1
  for (uint32_t m = 0; m < half; m += 2) {
#pragma unroll 1
    for (uint32_t j = 0; j < 2; ++j) {
      const uint32_t po = theirs0 + m + j;
      if (m + j < half && po < n_out) {
        uint32_t v[16];
        pair_partial<C, H, DBG>(a, po, acc, d, v);
        u32x4(*x)[64] = lds.v[j][pair][H];
#pragma unroll
        for (int q = 0; q < 4; ++q) x[q][lane] = (u32x4){v[4 * q], v[4 * q + 1], v[4 * q + 2], v[4 * q + 3]};
      }
    }
    __syncthreads();
#pragma unroll 1
    for (uint32_t j = 0; j < 2; ++j) {
      const uint32_t o = mine0 + m + j;
      if (m + j < half && o < n_out) {
        uint32_t v[16];
        pair_partial<C, H, DBG>(a, o, acc, d, v);
        const u32x4(*x)[64] = lds.v[j][pair][1 - H];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const u32x4 t = x[q][lane];
          v[4 * q] ^= t[0];
          v[4 * q + 1] ^= t[1];
          v[4 * q + 2] ^= t[2];
          v[4 * q + 3] ^= t[3];
        }
        if constexpr (HornerF<F>::N == 16) from_basis16(v, make_int_seq<16>{});
        u32x4 xs[4];
        unslice<F>(v, xs);
        uint8_t* dst = a.out[o];
#pragma unroll
        for (int q = 0; q < 4; ++q) stv<NT>(dst + off + q * 1024u, xs[q]);
      }
    }
    __syncthreads();
  }
  return prime;
}

// ---- compact mixing (RSE_OPT_RECON_PAIRS 6, A/B) ----------------------------
// The same unit with ONE copy of the mixing code for both roles: the data
// phase is specialised per role (its networks code the role's rows), the
// mixing takes the role at run time, runs one Horner step per loop trip (no
// 4-step unrolling) and computes the partner's and its own partials in one
// loop, so the Horner dispatch exists once in the kernel (instruction-cache
// footprint), not four times.
template <class C, bool NT, int H, int P>
__device__ __forceinline__ void pair_inputs(const BsReconArgs& a, uint64_t off, PairLds<P>& lds,
                                            uint32_t pair, uint32_t lane,
                                            uint32_t (&acc)[kPairRows * 16]) {
  using F = typename C::Field;
  constexpr int R0 = H * kPairRows;
  const uint32_t present = a.present;
  const uint32_t synd = a.synd;
  const uint64_t par_mask = H ? 0xAAAAAAAAull : 0x55555555ull;
  const uint64_t own = ((uint64_t)present & par_mask) |
                       ((uint64_t)((synd >> R0) & 0xFu) << (C::k + R0));
  u32x4 cur[4];
  if (own) load4<NT, 1024u>(cur, recon_ptr(a, C::k, (uint32_t)__builtin_ctzll(own)) + off);
  uint32_t buf = 0;
  u32x4(*mine)[64] = lds.v[0][pair][H];
  u32x4(*theirs)[64] = lds.v[0][pair][1 - H];
  pair_data<C, NT, H, 0, P>(acc, cur, cur, a, own, present, off, mine, theirs, lane, buf);
#pragma unroll
  for (int i = 0; i < kPairRows; ++i) {
    const int J = C::k + R0 + i;
    if ((own >> J) & 1u) {
      u32x4 nxt[4];
      const bool more = pair_prefetch<C, NT>(nxt, a, own, J, off);
      __builtin_amdgcn_sched_barrier(0);
      uint32_t pl[16];
      slice<F>(cur, pl);
#pragma unroll
      for (int q = 0; q < 16; ++q) acc[i * 16 + q] ^= pl[q];
      if (more) {
#pragma unroll
        for (int j = 0; j < 4; ++j) cur[j] = nxt[j];
      }
    }
  }
}

template <class C, bool NT, int P>
__device__ __forceinline__ void recon_pair_unit_compact(const BsReconArgs& a, uint64_t off,
                                                        PairLds<P>& lds, uint32_t pair,
                                                        uint32_t lane, uint32_t H) {
  using F = typename C::Field;
  constexpr int NB = HornerF<F>::N;
  uint32_t acc[kPairRows * 16];
#pragma unroll
  for (int q = 0; q < kPairRows * 16; ++q) acc[q] = 0u;
  if (H) pair_inputs<C, NT, 1, P>(a, off, lds, pair, lane, acc);
  else pair_inputs<C, NT, 0, P>(a, off, lds, pair, lane, acc);
  const uint32_t R0 = H * kPairRows;
  const uint32_t sigma = a.sigma;
  const uint32_t n_out = __builtin_amdgcn_readfirstlane(a.n_out);
  if constexpr (NB == 16) {
#pragma unroll
    for (int r = 0; r < kPairRows; ++r)
      if ((sigma >> (R0 + r)) & 1u) to_basis16(&acc[r * 16], make_int_seq<16>{});
  }
  uint32_t d[2][16];
#pragma unroll
  for (int t = 0; t < 2; ++t)
#pragma unroll
    for (int q = 0; q < 16; ++q) d[t][q] = acc[2 * t * 16 + q] ^ acc[(2 * t + 1) * 16 + q];
  const uint32_t half = (n_out + 1) / 2;
  const uint32_t mine0 = H * half, theirs0 = (1 - H) * half;
  const uint32_t nib_shift = 4u * H;
  __syncthreads();
#pragma unroll 1
  for (uint32_t m = 0; m < half; m += 2) {
#pragma unroll 1
    for (uint32_t x = 0; x < 4; ++x) {  // 0, 1: the partner's outputs; 2, 3: own
      const uint32_t j = x & 1u;
      const bool own_out = x >= 2;
      if (x == 2) __syncthreads();
      const uint32_t o = (own_out ? mine0 : theirs0) + m + j;
      if (m + j >= half || o >= n_out) continue;
      uint32_t v[16];
#pragma unroll
      for (int q = 0; q < 16; ++q) v[q] = 0u;
#pragma unroll 1
      for (int st = 0; st < NB; ++st) {
        const uint32_t word = (uint32_t)__builtin_amdgcn_readfirstlane(a.hm[o][st >> 2]);
        h_group<F, true, 0, kPairRows, 2>(v, acc, d, (word >> (8 * (st & 3) + nib_shift)) & 15u);
      }
      const int32_t os = __builtin_amdgcn_readfirstlane(a.out_sigma[o]) - (int32_t)R0;
#pragma unroll
      for (int r = 0; r < kPairRows; ++r)
        if (os == r) {
#pragma unroll
          for (int q = 0; q < 16; ++q) v[q] ^= acc[r * 16 + q];
        }
      if (!own_out) {
        u32x4(*xw)[64] = lds.v[j][pair][H];
#pragma unroll
        for (int q = 0; q < 4; ++q) xw[q][lane] = (u32x4){v[4 * q], v[4 * q + 1], v[4 * q + 2], v[4 * q + 3]};
      } else {
        const u32x4(*xr)[64] = lds.v[j][pair][1 - H];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const u32x4 t = xr[q][lane];
          v[4 * q] ^= t[0];
          v[4 * q + 1] ^= t[1];
          v[4 * q + 2] ^= t[2];
          v[4 * q + 3] ^= t[3];
        }
        if constexpr (NB == 16) from_basis16(v, make_int_seq<16>{});
        u32x4 xs[4];
        unslice<F>(v, xs);
        uint8_t* dst = a.out[o];
#pragma unroll
        for (int q = 0; q < 4; ++q) stv<NT>(dst + off + q * 1024u, xs[q]);
      }
    }
    __syncthreads();
  }
}

// Units of P 4 KiB columns: unit u of a stripe (cps 16 KiB chunks) covers
// bytes [u * 4096P, (u + 1) * 4096P); pair q its column q.  Workgroups of
// 128P lanes.
template <class C, bool NT, int P, bool PF = false, int DBG = 0>
__device__ __forceinline__ void bitslice_recon_pair_body(const BsReconArgs& a,
                                                         uint64_t chunks_per_stripe) {
  __shared__ PairLds<P> lds;
  const uint64_t upc = chunks_per_stripe * (4 / P), total = upc * a.n_stripes;
  const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint32_t pair = wave >> 1, lane = threadIdx.x & 63u;
  auto unit_off = [&](uint64_t u) {
    const uint64_t stripe = u / upc, sub = u - stripe * upc;
    return stripe * a.stripe_stride + sub * (4096u * P) + pair * 4096u + lane * 16u;
  };
  if constexpr (PF) {
    u32x4 cur[4];
    bool primed = false;
    for (uint64_t u = blockIdx.x; u < total; u += gridDim.x) {
      const uint64_t nu = u + gridDim.x;
      const uint64_t next_off = nu < total ? unit_off(nu) : ~0ull;
      if (wave & 1u) primed = recon_pair_unit<C, NT, 1, P, true>(a, unit_off(u), lds, pair, lane, cur, primed, next_off);
      else primed = recon_pair_unit<C, NT, 0, P, true>(a, unit_off(u), lds, pair, lane, cur, primed, next_off);
    }
  } else if constexpr (DBG == 3) {
    for (uint64_t u = blockIdx.x; u < total; u += gridDim.x)
      recon_pair_unit_compact<C, NT, P>(a, unit_off(u), lds, pair, lane, wave & 1u);
  } else {
    // (a fresh vector set per unit: nothing lives across units)
    for (uint64_t u = blockIdx.x; u < total; u += gridDim.x) {
      u32x4 cur[4];
      if (wave & 1u) recon_pair_unit<C, NT, 1, P, false, DBG>(a, unit_off(u), lds, pair, lane, cur, false, ~0ull);
      else recon_pair_unit<C, NT, 0, P, false, DBG>(a, unit_off(u), lds, pair, lane, cur, false, ~0ull);
    }
  }
}

// The same over per-stripe argument blocks (rse_reconstruct_batch).
template <class C, bool NT, int P, bool PF = false, int DBG = 0>
__device__ __forceinline__ void bitslice_recon_desc_pair_body(const BsReconArgs* __restrict__ descs,
                                                              uint64_t chunks_per_stripe,
                                                              uint64_t n_stripes) {
  __shared__ PairLds<P> lds;
  const uint64_t upc = chunks_per_stripe * (4 / P), total = upc * n_stripes;
  const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint32_t pair = wave >> 1, lane = threadIdx.x & 63u;
  if constexpr (PF) {
    u32x4 cur[4];
    bool primed = false;
    for (uint64_t u = blockIdx.x; u < total; u += gridDim.x) {
      const uint64_t stripe = u / upc, sub = u - stripe * upc;
      const BsReconArgs& a = desc_at(descs, stripe);
      if (a.n_out == 0) continue;  // workgroup-uniform
      const uint64_t off = sub * (4096u * P) + pair * 4096u + lane * 16u;
      // the next unit's first input only when it is this stripe's (same block)
      const uint64_t nu = u + gridDim.x, nsub = sub + gridDim.x;
      const uint64_t next_off =
          nu < total && nsub < upc ? nsub * (4096u * P) + pair * 4096u + lane * 16u : ~0ull;
      if (wave & 1u) primed = recon_pair_unit<C, NT, 1, P, true>(a, off, lds, pair, lane, cur, primed, next_off);
      else primed = recon_pair_unit<C, NT, 0, P, true>(a, off, lds, pair, lane, cur, primed, next_off);
    }
  } else if constexpr (DBG == 3) {
    for (uint64_t u = blockIdx.x; u < total; u += gridDim.x) {
      const uint64_t stripe = u / upc, sub = u - stripe * upc;
      const BsReconArgs& a = desc_at(descs, stripe);
      if (a.n_out == 0) continue;  // workgroup-uniform
      recon_pair_unit_compact<C, NT, P>(a, sub * (4096u * P) + pair * 4096u + lane * 16u, lds,
                                        pair, lane, wave & 1u);
    }
  } else {
    for (uint64_t u = blockIdx.x; u < total; u += gridDim.x) {
      const uint64_t stripe = u / upc, sub = u - stripe * upc;
      const BsReconArgs& a = desc_at(descs, stripe);
      if (a.n_out == 0) continue;  // workgroup-uniform
      const uint64_t off = sub * (4096u * P) + pair * 4096u + lane * 16u;
      u32x4 cur[4];
      if (wave & 1u) recon_pair_unit<C, NT, 1, P>(a, off, lds, pair, lane, cur, false, ~0ull);
      else recon_pair_unit<C, NT, 0, P>(a, off, lds, pair, lane, cur, false, ~0ull);
    }
  }
}

}  // namespace
}  // namespace rse
