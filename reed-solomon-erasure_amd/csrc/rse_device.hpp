// rse_device.hpp -- device helpers shared by the table kernels
// (rse_kernels.hip) and the bit-sliced kernels (rse_bitslice.hip): GF(2^8)
// constant-multiply tables for v_perm_b32, 16-byte global access, GF(2^16)
// byte-plane split/merge, and the asm fences that keep hipcc from hoisting
// table reads or re-associating XOR chains.
#pragma once

#include "rse_kernels.hpp"

namespace rse {
namespace {

// ---------------------------------------------------------------------------
// GF(2^8) constant-multiply tables (generator polynomial 0x11D, build.rs:11).
struct Gf8Tab {
  uint32_t t0lo, t0hi;  // c*j       j = 0..7
  uint32_t t1lo, t1hi;  // c*(j<<3)  j = 0..7
  uint32_t t2;          // c*(j<<6)  j = 0..3
};

__device__ __forceinline__ uint32_t xtime(uint32_t v) {
  return ((v << 1) ^ ((v & 0x80u) ? 0x1Du : 0u)) & 0xFFu;
}

__device__ __forceinline__ Gf8Tab make_gf8_tab(uint32_t c) {
  uint32_t e[8];  // e[b] = c * 2^b
  e[0] = c & 0xFFu;
#pragma unroll
  for (int b = 1; b < 8; ++b) e[b] = xtime(e[b - 1]);
  auto sub = [&](int base, int nbits, int j) {
    uint32_t r = 0;
    for (int b = 0; b < nbits; ++b)
      if ((j >> b) & 1) r ^= e[base + b];
    return r;
  };
  auto pack = [&](int base, int nbits, int j0) {
    return sub(base, nbits, j0) | (sub(base, nbits, j0 + 1) << 8) |
           (sub(base, nbits, j0 + 2) << 16) | (sub(base, nbits, j0 + 3) << 24);
  };
  Gf8Tab t;
  t.t0lo = pack(0, 3, 0);
  t.t0hi = pack(0, 3, 4);
  t.t1lo = pack(3, 3, 0);
  t.t1hi = pack(3, 3, 4);
  t.t2 = pack(6, 2, 0);
  return t;
}

// Selector bytes for the three bit groups of every byte of x.
struct Sel {
  uint32_t s0, s1, s2;
};
__device__ __forceinline__ Sel make_sel(uint32_t x) {
  Sel s;
  s.s0 = x & 0x07070707u;
  s.s1 = (x >> 3) & 0x07070707u;
  s.s2 = (x >> 6) & 0x03030303u;
  return s;
}

// a ^ b ^ c in one instruction: gfx950's v_bitop3_b32 (truth table 0x96).
__device__ __forceinline__ uint32_t xor3(uint32_t a, uint32_t b, uint32_t c) {
  return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);
}

// c * x for the four bytes of x (tables of c): 3 v_perm_b32 + 1 v_bitop3_b32.
__device__ __forceinline__ uint32_t gf8_mul4(const Gf8Tab& t, const Sel& s) {
  const uint32_t a = __builtin_amdgcn_perm(t.t0hi, t.t0lo, s.s0);
  const uint32_t b = __builtin_amdgcn_perm(t.t1hi, t.t1lo, s.s1);
  const uint32_t c = __builtin_amdgcn_perm(t.t2, t.t2, s.s2);
  return xor3(a, b, c);
}

// acc ^ c*x: 3 v_perm_b32 + 2 v_bitop3_b32-class ops (acc ^ a ^ b, then ^ c).
__device__ __forceinline__ uint32_t gf8_mac4(uint32_t acc, const Gf8Tab& t, const Sel& s) {
  const uint32_t a = __builtin_amdgcn_perm(t.t0hi, t.t0lo, s.s0);
  const uint32_t b = __builtin_amdgcn_perm(t.t1hi, t.t1lo, s.s1);
  const uint32_t c = __builtin_amdgcn_perm(t.t2, t.t2, s.s2);
  return xor3(acc, a, b) ^ c;
}

// LDS image of one table: a 16-byte part and a 4-byte part so each is one
// broadcast ds_read (b128 + b32) at a wave-uniform address.
struct TabLds {
  uint4 q;  // t0lo, t0hi, t1lo, t1hi
  uint32_t t2;
};

__device__ __forceinline__ Gf8Tab read_tab(const uint4* q, const uint32_t* t2, int idx) {
  const uint4 v = q[idx];
  Gf8Tab t;
  t.t0lo = v.x;
  t.t0hi = v.y;
  t.t1lo = v.z;
  t.t1hi = v.w;
  t.t2 = t2[idx];
  return t;
}

__device__ __forceinline__ void write_tab(uint4* q, uint32_t* t2, int idx, const Gf8Tab& t) {
  q[idx] = make_uint4(t.t0lo, t.t0hi, t.t1lo, t.t1hi);
  t2[idx] = t.t2;
}

typedef unsigned u32x4 __attribute__((ext_vector_type(4)));

// Shard accesses go through global-address-space pointers. Shard pointers read
// from memory (the per-stripe descriptors of reconstruct_batch and of the
// table path's batched reconstruct) are generic pointers, which the compiler
// otherwise accesses with flat_load/flat_store: both counters to wait on and no
// global addressing. Shards are always device-visible global memory.
template <class T>
using gptr = __attribute__((address_space(1))) T*;

// 16-byte global access.  NT = non-temporal (streaming) hint: every shard byte
// is touched exactly once, so there is nothing to keep in L2/MALL.
template <bool NT = false>
__device__ __forceinline__ uint4 ld16(const uint8_t* p) {
  if constexpr (NT) {
    const u32x4 v = __builtin_nontemporal_load((gptr<const u32x4>)(p));
    return make_uint4(v.x, v.y, v.z, v.w);
  } else {
    const u32x4 v = *(gptr<const u32x4>)(p);
    return make_uint4(v.x, v.y, v.z, v.w);
  }
}
template <bool NT = false>
__device__ __forceinline__ void st16(uint8_t* p, uint4 v) {
  if constexpr (NT) {
    const u32x4 w = {v.x, v.y, v.z, v.w};
    __builtin_nontemporal_store(w, (gptr<u32x4>)(p));
  } else {
    const u32x4 w = {v.x, v.y, v.z, v.w};
    *(gptr<u32x4>)(p) = w;
  }
}
__device__ __forceinline__ bool ne4(uint4 a, uint4 b) {
  return ((a.x ^ b.x) | (a.y ^ b.y) | (a.z ^ b.z) | (a.w ^ b.w)) != 0u;
}

// The mismatch word of the stripe at byte offset soff (CodeArgs::per_stripe).
__device__ __forceinline__ uint32_t* mismatch_word(const CodeArgs& a, uint64_t soff) {
  return a.mismatch + ((a.per_stripe && a.stripe_stride) ? soff / a.stripe_stride : 0u);
}

// A check kernel's verdict: any nonzero word means a mismatch, so lanes that
// find one store 1 (a plain vector store, idempotent: no atomic needed).  The
// word may be in pinned host memory (rse_codec.cpp run_check), where a PCIe
// atomic would need platform support.
__device__ __forceinline__ void flag_mismatch(uint32_t* p) {
  *reinterpret_cast<volatile uint32_t*>(p) = 1u;
}

// Completion of a one-launch verify (CodeArgs::done, armed by run_check): the
// last workgroup to get here stores 1 into a.done, a word of pinned host
// memory, after every workgroup's verdict stores have completed, and the host
// spins on that word instead of waiting for the end-of-kernel signal.  Each
// thread first waits until its own stores are acknowledged (the verdict words
// are uncached host memory: acknowledged means visible to the host); the
// workgroup count on the device word a.done_count (one agent-scope atomic per
// workgroup) then makes the last workgroup's completion store come after every
// acknowledgement.  No release fences: at agent scope they write back and
// invalidate L2 in every wave (a 49 us verify took 188 with them); the
// end-of-kernel release still orders everything for later work on the stream.
// The last workgroup rezeroes the count for the next launch.  Every workgroup
// of the launch calls this once, all threads.
__device__ __forceinline__ void signal_done(const CodeArgs& a) {
  if (!a.done) return;
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    const uint32_t n = __hip_atomic_fetch_add(a.done_count, 1u, __ATOMIC_RELAXED,
                                              __HIP_MEMORY_SCOPE_AGENT);
    if (n == gridDim.x - 1) {
      __hip_atomic_store(a.done_count, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(a.done, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
  }
}

// One store per wave that saw a difference, on the word of stripe offset soff.
__device__ __forceinline__ void flag_mismatch(bool diff, const CodeArgs& a, uint64_t soff) {
  const unsigned long long m = __ballot(diff);
  if (m != 0ull && (threadIdx.x & 63) == (unsigned)(__ffsll((long long)m) - 1))
    flag_mismatch(mismatch_word(a, soff));
}

__device__ __forceinline__ uint32_t opaque_zero() {
  uint32_t z = 0;
  asm volatile("" : "+s"(z));
  return z;
}

__device__ __forceinline__ void pin(uint32_t& v) { asm volatile("" : "+v"(v)); }

__device__ __forceinline__ void pin(uint4& v) {
  pin(v.x);
  pin(v.y);
  pin(v.z);
  pin(v.w);
}

// ---------------------------------------------------------------------------
// GF(2^16) byte planes.
__device__ __forceinline__ void split_planes(uint4 v, uint32_t& h0, uint32_t& l0,
                                             uint32_t& h1, uint32_t& l1) {
  // v.x = [a1_0 a0_0 a1_1 a0_1], v.y = [a1_2 a0_2 a1_3 a0_3] (little endian bytes)
  h0 = __builtin_amdgcn_perm(v.y, v.x, 0x06040200u);
  l0 = __builtin_amdgcn_perm(v.y, v.x, 0x07050301u);
  h1 = __builtin_amdgcn_perm(v.w, v.z, 0x06040200u);
  l1 = __builtin_amdgcn_perm(v.w, v.z, 0x07050301u);
}
__device__ __forceinline__ uint4 merge_planes(uint32_t h0, uint32_t l0, uint32_t h1,
                                              uint32_t l1) {
  uint4 o;
  o.x = __builtin_amdgcn_perm(l0, h0, 0x05010400u);
  o.y = __builtin_amdgcn_perm(l0, h0, 0x07030602u);
  o.z = __builtin_amdgcn_perm(l1, h1, 0x05010400u);
  o.w = __builtin_amdgcn_perm(l1, h1, 0x07030602u);
  return o;
}

__device__ __forceinline__ void gf16_sub_coefs(uint32_t c, uint32_t sub[4]) {
  const uint32_t c1 = (c >> 8) & 0xFFu, c0 = c & 0xFFu;
  uint32_t t = c1;  // 128 * c1 = c1 * 2^7
#pragma unroll
  for (int b = 0; b < 7; ++b) t = xtime(t);
  sub[0] = c0 ^ xtime(c1);  // HH = c0 + 2*c1
  sub[1] = c1;              // LH
  sub[2] = t;               // HL = 128*c1
  sub[3] = c0;              // LL
}

}  // namespace
}  // namespace rse
