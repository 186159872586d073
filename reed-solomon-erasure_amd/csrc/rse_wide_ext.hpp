// rse_wide_ext.hpp -- variants of the half-chunk wide bodies
// (rse_bitslice_core.hpp wide_body_half) that run-time modules include only
// when an option asks for them (rse_jit.cpp make_source appends this text,
// kJitExtSource, after the core's): the core's text is part of every module's
// cache key, so experiments live here and leave the other modules' keys alone.
//
// PP: XOR networks of PP input pairs per scheduling region.  wide_body_half
// pins the accumulators after every pair (asm "+v"), which keeps the compiler
// from reassociating across inputs but also cuts its scheduling regions to one
// pair's network: the temporaries, then the XORs that use them 2-4
// instructions later.  At PP = 2 the scheduler can interleave two pairs'
// networks (longer dependence distance) at the cost of both pairs' sources
// and temporaries live at once.
#pragma once

namespace rse {

template <class C, int W, int R, int S, int PP>
__device__ __forceinline__ void wide_code_round_half_pp(uint32_t (&acc)[C::p * 8],
                                                        const uint4 (&set)[W][2][64],
                                                        uint32_t lane) {
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
    constexpr bool last = !(S + 2 < W && R * W + S + 2 < C::k);
    if constexpr ((S / 2) % PP == PP - 1 || last) {
#pragma unroll
      for (int q = 0; q < C::p * 8; ++q) asm volatile("" : "+v"(acc[q]));
    }
    wide_code_round_half_pp<C, W, R, S + 2, PP>(acc, set, lane);
  }
}

template <class C, int W, int WI, int D, int R, class A, uint32_t S, int PP>
__device__ __forceinline__ void wide_rounds_half_pp(uint32_t (&acc)[C::p * 8],
                                                    u32x4 (&buf)[D + 1][2], const A& a,
                                                    uint64_t off, uint64_t next_off,
                                                    WideHalfPlanes<W>& lds, uint32_t& g,
                                                    uint32_t lane) {
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
    wide_code_round_half_pp<C, W, R, 0, PP>(acc, set, lane);
    ++g;
    wide_rounds_half_pp<C, W, WI, D, R + 1, A, S, PP>(acc, buf, a, off, next_off, lds, g, lane);
  }
}

// wide_body_half with PP pairs per scheduling region.
template <class C, int O0, int W, int WI, int D, class A, uint32_t SUB, int PP>
__device__ __forceinline__ void wide_body_half_pp(const A& a, WideHalfPlanes<W>& lds) {
  static_assert(SUB == 0 || SUB == 1024u || SUB == 2048u, "1 or 2 KiB shards");
  const WideHdr& h = a.h;
  constexpr int K = C::k, NR = (K + W - 1) / W;
  constexpr uint32_t S = SUB ? SUB / 2u : 1024u;
  constexpr uint32_t SPC = SUB ? 2048u / SUB : 1u, LPS = 64u / SPC;
  const uint64_t halves = 2 * h.chunks_per_stripe;
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
    wide_rounds_half_pp<C, W, WI, D, 0, A, S, PP>(acc, buf, a, off, next_off, lds, g, lane);
    if constexpr (NR % (D + 1) != 0) {
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

}  // namespace rse
