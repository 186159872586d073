// rse_kernels.hip -- CDNA4 (gfx950) kernels for the Reed-Solomon hot path.
//
// Replaces, as one fused pass, the reference's
//   core.rs:481-509 code_some_slices / code_single_slice   (loop over k*p slices)
//   galois_8.rs:291-327 mul_slice / mul_slice_xor           (per-coefficient pass)
//   simd_c/reedsolomon.c:495-574 reedsolomon_gal_mul(_xor) (PSHUFB nibble kernel)
//   lib.rs:99-118 default mul_slice(_add) used by galois_16 (scalar GF(2^16))
//
// Arithmetic: multiplication by a constant c is GF(2)-linear, so
//   c*x = c*(x & 0x07) ^ c*(x & 0x38) ^ c*(x & 0xC0)
// and each term is an 8- (or 4-) entry table lookup.  CDNA's v_perm_b32 is a
// 4-lane byte gather from an 8-byte register pair, i.e. exactly an 8-entry table
// lookup for four bytes at once, so one GF(2^8) constant multiply of a dword
// costs 3 v_perm + 3 v_xor and no memory traffic.  The per-(input, output)
// tables are built once per workgroup into LDS from the coefficient bytes and
// read back as wave-uniform broadcasts (conflict-free).  Data moves as 16 B per
// lane (global_load/store_dwordx4): each wave touches 1 KiB contiguous per shard.
// No MFMA: this is XOR/table work, HBM-bound.
//
// GF(2^16) = GF(2^8)[x]/(x^2 + 2x + 128) (galois_16.rs:9-14).  For a constant
// c = c1*x + c0 and element a = a1*x + a0 (bytes [a1, a0], galois_16.rs:49-51):
//   (c*a)_x = (c0 ^ 2*c1)*a1 ^ c1*a0        (c*a)_1 = (128*c1)*a1 ^ c0*a0
// (galois_16.rs:146-162 with reduce_from :97-107 folded in), so a GF(2^16)
// shard is two GF(2^8) byte planes and one GF(2^16) coefficient is a 2x2 block
// of GF(2^8) coefficients.  Planes are split/merged in registers with v_perm.
#include <cstdarg>
#include <cstdio>

#include "rse_device.hpp"

namespace rse {
namespace {

constexpr int kBlock = 256;

// ---------------------------------------------------------------------------
// Kernel structure shared by both fields.
//   KC : inputs loaded per chunk (compile time; all KC loads are issued before
//        any arithmetic so a lane keeps KC x 16 B in flight per shard sweep)
//   NO : output capacity (accumulators live in VGPRs)
//   NOGUARD: n_out == NO and KC divides n_in -- no runtime guards.
//   VPL: 16-byte vectors per lane per span (amortises each LDS table read).
// grid = (blocks, stripes); each block grid-strides over 16-byte vectors.
//
// Table reads go through an opaque LDS offset (`lds_base`) re-materialised
// every vector iteration: otherwise LICM hoists every (input, output) table
// out of the loop into VGPRs (k*p*5 of them), which caps occupancy at one wave
// (opaque_zero / pin: rse_device.hpp).

// One span of the vector body: lane t codes the VPL vectors vfirst,
// vfirst + kBlock, ... (each wave-instruction stays a coalesced 1 KiB; a wave
// covers VPL KiB of every shard).  Every (input, output) table read from LDS
// is applied to VPL*4 dwords.
template <int KC, int NO, bool NOGUARD, bool NT, int VPL>
__device__ __forceinline__ void gf8_span(const CodeArgs& a, const uint4* tq, const uint32_t* tt2,
                                         uint64_t soff, uint64_t vfirst, uint32_t n_in,
                                         uint32_t n_out, uint32_t mode) {
  const uint32_t lb = opaque_zero();
  uint64_t off[VPL];
#pragma unroll
  for (int q = 0; q < VPL; ++q) off[q] = soff + (vfirst + (uint64_t)q * kBlock) * 16u;
  uint4 acc[NO][VPL];
#pragma unroll
  for (int r = 0; r < NO; ++r)
#pragma unroll
    for (int q = 0; q < VPL; ++q) {
      acc[r][q] = make_uint4(0u, 0u, 0u, 0u);
      if (a.accumulate && (NOGUARD || (uint32_t)r < n_out)) acc[r][q] = ld16(a.out[r] + off[q]);
    }
  for (uint32_t i0 = 0; i0 < n_in; i0 += KC) {
    uint4 x[KC][VPL];
#pragma unroll
    for (int j = 0; j < KC; ++j)
      if (NOGUARD || i0 + j < n_in)
#pragma unroll
        for (int q = 0; q < VPL; ++q) x[j][q] = ld16<NT>(a.in[i0 + j] + off[q]);
#pragma unroll
    for (int j = 0; j < KC; ++j) {
      if (!(NOGUARD || i0 + j < n_in)) continue;
      Sel sel[VPL][4];
#pragma unroll
      for (int q = 0; q < VPL; ++q) {
        sel[q][0] = make_sel(x[j][q].x);
        sel[q][1] = make_sel(x[j][q].y);
        sel[q][2] = make_sel(x[j][q].z);
        sel[q][3] = make_sel(x[j][q].w);
      }
#pragma unroll
      for (int r = 0; r < NO; ++r) {
        if (!(NOGUARD || (uint32_t)r < n_out)) continue;
        const Gf8Tab t = read_tab(tq, tt2, lb + r * n_in + i0 + j);
#pragma unroll
        for (int q = 0; q < VPL; ++q) {
          acc[r][q].x = gf8_mac4(acc[r][q].x, t, sel[q][0]);
          acc[r][q].y = gf8_mac4(acc[r][q].y, t, sel[q][1]);
          acc[r][q].z = gf8_mac4(acc[r][q].z, t, sel[q][2]);
          acc[r][q].w = gf8_mac4(acc[r][q].w, t, sel[q][3]);
        }
      }
      // Pin the running sums after every input: without it the XOR chain is
      // reassociated into a tree whose k*p partial products spill.
#pragma unroll
      for (int r = 0; r < NO; ++r)
#pragma unroll
        for (int q = 0; q < VPL; ++q) pin(acc[r][q]);
    }
  }
  if (mode != kCheck) {
#pragma unroll
    for (int r = 0; r < NO; ++r)
      if (NOGUARD || (uint32_t)r < n_out)
#pragma unroll
        for (int q = 0; q < VPL; ++q) st16<NT>(a.out[r] + off[q], acc[r][q]);
  }
  if (mode != kStore) {
    bool diff = false;
#pragma unroll
    for (int r = 0; r < NO; ++r)
      if (NOGUARD || (uint32_t)r < n_out)
#pragma unroll
        for (int q = 0; q < VPL; ++q) diff |= ne4(acc[r][q], ld16<NT>(a.cmp[r] + off[q]));
    flag_mismatch(diff, a, soff);
  }
}

// GF(2^8) fused coding kernel.  NOGUARD: n_out == NO and KC divides n_in.
template <int KC, int NO, bool NOGUARD, bool NT, int VPL>
__device__ __forceinline__ void gf8_code_impl(const CodeArgs& a, uint32_t stripe0,
                                              uint32_t stripe_step) {
  // table (r, i) lives at index r * n_in + i
  __shared__ uint4 tq[kMaxIn * NO];
  __shared__ uint32_t tt2[kMaxIn * NO];

  const uint32_t n_in = a.n_in;
  const uint32_t n_out = NOGUARD ? NO : a.n_out;

  for (uint32_t t = threadIdx.x; t < n_out * n_in; t += kBlock) {
    const uint32_t r = t / n_in, i = t % n_in;
    write_tab(tq, tt2, t, make_gf8_tab(a.coef[r][i]));
  }
  __syncthreads();

  const uint64_t gstride = (uint64_t)gridDim.x * kBlock;
  const uint64_t gtid = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
  const uint32_t mode = a.mode;
  const uint64_t span = (uint64_t)kBlock * VPL;
  const uint64_t n_full = a.n_vec / span;

  // Stripes in flight = gridDim.y: every block of row y sweeps stripes
  // y, y + gridDim.y, ...  (gridDim.y == 1: the whole grid walks the stripes in
  // order, keeping few DRAM regions open at a time).
  for (uint32_t stripe = stripe0; stripe < a.n_stripes; stripe += stripe_step) {
  const uint64_t soff = (uint64_t)stripe * a.stripe_stride;

  for (uint64_t sp = blockIdx.x; sp < n_full; sp += gridDim.x)
    gf8_span<KC, NO, NOGUARD, NT, VPL>(a, tq, tt2, soff, sp * span + threadIdx.x, n_in, n_out,
                                       mode);
  // vectors after the last full span, one per lane
  for (uint64_t v = n_full * span + gtid; v < a.n_vec; v += gstride)
      gf8_span<KC, NO, NOGUARD, NT, 1>(a, tq, tt2, soff, v, n_in, n_out, mode);

  // Byte tail (len % 16), and the whole range when a pointer is not 16-B aligned.
  for (uint64_t b = a.n_vec * 16u + gtid; b < a.len; b += gstride) {
    const uint64_t off = soff + b;
    uint32_t acc[NO];
#pragma unroll
    for (int r = 0; r < NO; ++r)
      acc[r] = (a.accumulate && (NOGUARD || (uint32_t)r < n_out)) ? a.out[r][off] : 0u;
    const uint32_t lb = opaque_zero();
#pragma unroll 1
    for (uint32_t i = 0; i < n_in; ++i) {
      const Sel s = make_sel(a.in[i][off]);
#pragma unroll
      for (int r = 0; r < NO; ++r)
        if (NOGUARD || (uint32_t)r < n_out) acc[r] ^= gf8_mul4(read_tab(tq, tt2, lb + r * n_in + i), s);
    }
    bool diff = false;
#pragma unroll
    for (int r = 0; r < NO; ++r) {
      if (!(NOGUARD || (uint32_t)r < n_out)) continue;
      if (mode != kCheck) a.out[r][off] = (uint8_t)acc[r];
      if (mode != kStore) diff |= (uint8_t)acc[r] != a.cmp[r][off];
    }
    if (mode != kStore && diff) flag_mismatch(mismatch_word(a, soff));
  }
  }  // stripe loop
}

template <int KC, int NO, bool NOGUARD, bool NT, int VPL>
__global__ __launch_bounds__(kBlock, VPL == 1 ? (NO >= 16 ? 3 : 4) : 2) void gf8_code_kernel(
    const CodeArgs a) {
  gf8_code_impl<KC, NO, NOGUARD, NT, VPL>(a, blockIdx.y, gridDim.y);
}

// Per-stripe descriptors in HBM (written by recon_plan_kernel): row y of
// the grid codes stripe y with its own shard pointers and coefficient rows.
template <bool NT>
__global__ __launch_bounds__(kBlock, 3) void gf8_code_desc_kernel(const CodeArgs* __restrict__ descs) {
  // through the constant address space: scalar loads of the descriptor's fields
  // (written by the planner kernel before this one, never during it)
  using CPtr = const __attribute__((address_space(4))) CodeArgs*;
  const CodeArgs& a = *(const CodeArgs*)((CPtr)descs + blockIdx.y);
  if (a.n_out == 0) return;  // uniform: nothing missing in this stripe
  gf8_code_impl<8, kMaxOut, false, NT, 1>(a, 0, 1);
}

// ---------------------------------------------------------------------------
// Software-pipelined GF(2^8) kernel for exact shapes (n_in == K, n_out == NO,
// STORE mode, no accumulate): while a lane codes span s, the K loads of its
// next span s + gridDim.x are already in flight, so a wave never idles on HBM
// between spans and fewer waves (fewer open DRAM regions) keep the bus busy.
// Spans are numbered across stripes (stripe-major), so the pipeline also runs
// across stripe boundaries.  Partial spans and byte tails fall back to the
// plain span code after the pipelined sweep.
// The K loads of a span are issued from inline asm and waited for by hand:
// hipcc's own vmcnt accounting is conservative across the loop back-edge and
// drains the next span's loads before the current span is coded (measured:
// vmcnt(7)..vmcnt(0) inside the compute).  Invariant kept here: between a
// span's loads and its coding, the only younger vector-memory operations of the
// wave are the previous span's NO stores (older than the next loads) and, when
// `more`, the next span's K loads; so input j is complete once at most
// K - 1 - j (+ K when more) operations are outstanding.  Waiting with that
// count ignores the NO stores, which only makes the wait stricter.
template <int K>
__device__ __forceinline__ void load_k(u32x4 (&x)[K], const CodeArgs& a, uint64_t off) {
#pragma unroll
  for (int j = 0; j < K; ++j)
    asm volatile("global_load_dwordx4 %0, %1, off nt" : "=v"(x[j]) : "v"(a.in[j] + off) : "memory");
}

// s_waitcnt vmcnt(n) that also "produces" v, so v's consumers stay behind it.
// n is a compile-time constant after unrolling; the switch folds away.
__device__ __forceinline__ void wait_vm(int n, u32x4& v) {
  switch (n) {
    case 0: asm volatile("s_waitcnt vmcnt(0)" : "+v"(v) :: "memory"); break;
    case 1: asm volatile("s_waitcnt vmcnt(1)" : "+v"(v) :: "memory"); break;
    case 2: asm volatile("s_waitcnt vmcnt(2)" : "+v"(v) :: "memory"); break;
    case 3: asm volatile("s_waitcnt vmcnt(3)" : "+v"(v) :: "memory"); break;
    case 4: asm volatile("s_waitcnt vmcnt(4)" : "+v"(v) :: "memory"); break;
    case 5: asm volatile("s_waitcnt vmcnt(5)" : "+v"(v) :: "memory"); break;
    case 6: asm volatile("s_waitcnt vmcnt(6)" : "+v"(v) :: "memory"); break;
    case 7: asm volatile("s_waitcnt vmcnt(7)" : "+v"(v) :: "memory"); break;
    case 8: asm volatile("s_waitcnt vmcnt(8)" : "+v"(v) :: "memory"); break;
    case 9: asm volatile("s_waitcnt vmcnt(9)" : "+v"(v) :: "memory"); break;
    case 10: asm volatile("s_waitcnt vmcnt(10)" : "+v"(v) :: "memory"); break;
    case 11: asm volatile("s_waitcnt vmcnt(11)" : "+v"(v) :: "memory"); break;
    case 12: asm volatile("s_waitcnt vmcnt(12)" : "+v"(v) :: "memory"); break;
    case 13: asm volatile("s_waitcnt vmcnt(13)" : "+v"(v) :: "memory"); break;
    case 14: asm volatile("s_waitcnt vmcnt(14)" : "+v"(v) :: "memory"); break;
    case 15: asm volatile("s_waitcnt vmcnt(15)" : "+v"(v) :: "memory"); break;
    case 16: asm volatile("s_waitcnt vmcnt(16)" : "+v"(v) :: "memory"); break;
    case 17: asm volatile("s_waitcnt vmcnt(17)" : "+v"(v) :: "memory"); break;
    case 18: asm volatile("s_waitcnt vmcnt(18)" : "+v"(v) :: "memory"); break;
    case 19: asm volatile("s_waitcnt vmcnt(19)" : "+v"(v) :: "memory"); break;
    case 20: asm volatile("s_waitcnt vmcnt(20)" : "+v"(v) :: "memory"); break;
    case 21: asm volatile("s_waitcnt vmcnt(21)" : "+v"(v) :: "memory"); break;
    case 22: asm volatile("s_waitcnt vmcnt(22)" : "+v"(v) :: "memory"); break;
    case 23: asm volatile("s_waitcnt vmcnt(23)" : "+v"(v) :: "memory"); break;
    case 24: asm volatile("s_waitcnt vmcnt(24)" : "+v"(v) :: "memory"); break;
    case 25: asm volatile("s_waitcnt vmcnt(25)" : "+v"(v) :: "memory"); break;
    case 26: asm volatile("s_waitcnt vmcnt(26)" : "+v"(v) :: "memory"); break;
    case 27: asm volatile("s_waitcnt vmcnt(27)" : "+v"(v) :: "memory"); break;
    case 28: asm volatile("s_waitcnt vmcnt(28)" : "+v"(v) :: "memory"); break;
    case 29: asm volatile("s_waitcnt vmcnt(29)" : "+v"(v) :: "memory"); break;
    case 30: asm volatile("s_waitcnt vmcnt(30)" : "+v"(v) :: "memory"); break;
    case 31: asm volatile("s_waitcnt vmcnt(31)" : "+v"(v) :: "memory"); break;
    default: asm volatile("s_waitcnt vmcnt(0)" : "+v"(v) :: "memory"); break;
  }
}

template <int K, int NO, int NB>
__device__ __forceinline__ void code_k(u32x4 (&x)[K], const uint4* tq, const uint32_t* tt2,
                                       const CodeArgs& a, uint64_t off) {
  const uint32_t lb = opaque_zero();
  uint4 acc[NO];
#pragma unroll
  for (int r = 0; r < NO; ++r) acc[r] = make_uint4(0u, 0u, 0u, 0u);
#pragma unroll
  for (int j = 0; j < K; ++j) {
    wait_vm(NB + K - 1 - j, x[j]);
    const Sel sx = make_sel(x[j].x), sy = make_sel(x[j].y);
    const Sel sz = make_sel(x[j].z), sw = make_sel(x[j].w);
#pragma unroll
    for (int r = 0; r < NO; ++r) {
      const Gf8Tab t = read_tab(tq, tt2, lb + r * K + j);
      acc[r].x = gf8_mac4(acc[r].x, t, sx);
      acc[r].y = gf8_mac4(acc[r].y, t, sy);
      acc[r].z = gf8_mac4(acc[r].z, t, sz);
      acc[r].w = gf8_mac4(acc[r].w, t, sw);
    }
    // also orders input j's arithmetic before input j+1's wait (both volatile)
#pragma unroll
    for (int r = 0; r < NO; ++r) pin(acc[r]);
  }
#pragma unroll
  for (int r = 0; r < NO; ++r) st16<true>(a.out[r] + off, acc[r]);
}

template <int K, int NO>
__global__ __launch_bounds__(kBlock, 2) void gf8_pipe_kernel(const CodeArgs a) {
  __shared__ uint4 tq[K * NO];
  __shared__ uint32_t tt2[K * NO];
  for (uint32_t t = threadIdx.x; t < (uint32_t)(K * NO); t += kBlock)
    write_tab(tq, tt2, t, make_gf8_tab(a.coef[t / K][t % K]));
  __syncthreads();

  const uint64_t sps = a.n_vec / kBlock;  // full spans per stripe
  const uint64_t total = sps * a.n_stripes;
  uint64_t sp = blockIdx.x;
  if (sps && sp < total) {
    uint64_t stripe = sp / sps, local = sp % sps;
    uint64_t off = stripe * a.stripe_stride + (local * kBlock + threadIdx.x) * 16u;
    u32x4 xa[K], xb[K];
    load_k<K>(xa, a, off);
    for (;;) {  // two spans per trip: xa/xb swap roles without register copies
      uint64_t sp2 = sp + gridDim.x, off2 = 0;
      const bool more = sp2 < total;
      if (more) {
        local += gridDim.x;
        while (local >= sps) { local -= sps; ++stripe; }
        off2 = stripe * a.stripe_stride + (local * kBlock + threadIdx.x) * 16u;
        load_k<K>(xb, a, off2);
        code_k<K, NO, K>(xa, tq, tt2, a, off);
      } else {
        code_k<K, NO, 0>(xa, tq, tt2, a, off);
        break;
      }
      sp = sp2;
      off = off2;
      const uint64_t sp3 = sp + gridDim.x;
      if (sp3 < total) {
        local += gridDim.x;
        while (local >= sps) { local -= sps; ++stripe; }
        off2 = stripe * a.stripe_stride + (local * kBlock + threadIdx.x) * 16u;
        load_k<K>(xa, a, off2);
        code_k<K, NO, K>(xb, tq, tt2, a, off);
      } else {
        code_k<K, NO, 0>(xb, tq, tt2, a, off);
        break;
      }
      sp = sp3;
      off = off2;
    }
  }
  // leftovers: vectors after the last full span of every stripe, byte tails
  const uint64_t gstride = (uint64_t)gridDim.x * kBlock;
  const uint64_t gtid = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
  for (uint32_t stripe = 0; stripe < a.n_stripes; ++stripe) {
    const uint64_t soff = (uint64_t)stripe * a.stripe_stride;
    for (uint64_t v = sps * kBlock + gtid; v < a.n_vec; v += gstride)
      gf8_span<K, NO, true, true, 1>(a, tq, tt2, soff, v, K, NO, kStore);
    for (uint64_t b = a.n_vec * 16u + gtid; b < a.len; b += gstride) {
      const uint64_t off = soff + b;
      uint32_t acc[NO];
#pragma unroll
      for (int r = 0; r < NO; ++r) acc[r] = 0u;
      const uint32_t lb = opaque_zero();
#pragma unroll 1
      for (uint32_t i = 0; i < (uint32_t)K; ++i) {
        const Sel s = make_sel(a.in[i][off]);
#pragma unroll
        for (int r = 0; r < NO; ++r) acc[r] ^= gf8_mul4(read_tab(tq, tt2, lb + r * K + i), s);
      }
#pragma unroll
      for (int r = 0; r < NO; ++r) a.out[r][off] = (uint8_t)acc[r];
    }
  }
}

// ---------------------------------------------------------------------------
// GF(2^16) fused coding kernel.  Per coefficient: 4 GF(2^8) tables
// [HH, LH, HL, LL]: OH = HH*H ^ LH*L, OL = HL*H ^ LL*L, where H/L are the
// byte planes (coefficient-of-x / constant bytes) of 4 consecutive elements.
template <int KC, int NO, bool NOGUARD, bool NT, int VPL>
__device__ __forceinline__ void gf16_span(const CodeArgs& a, const uint4* tq, const uint32_t* tt2,
                                          uint64_t soff, uint64_t vfirst, uint32_t n_in,
                                          uint32_t n_out, uint32_t mode) {
  const uint32_t lb = opaque_zero();
  uint64_t off[VPL];
#pragma unroll
  for (int q = 0; q < VPL; ++q) off[q] = soff + (vfirst + (uint64_t)q * kBlock) * 16u;
  // [r][q][0..3] = OH(elements 0-3), OL(0-3), OH(4-7), OL(4-7)
  uint32_t o[NO][VPL][4];
#pragma unroll
  for (int r = 0; r < NO; ++r)
#pragma unroll
    for (int q = 0; q < VPL; ++q) {
      o[r][q][0] = o[r][q][1] = o[r][q][2] = o[r][q][3] = 0u;
      if (a.accumulate && (NOGUARD || (uint32_t)r < n_out))
        split_planes(ld16(a.out[r] + off[q]), o[r][q][0], o[r][q][1], o[r][q][2], o[r][q][3]);
    }
  for (uint32_t i0 = 0; i0 < n_in; i0 += KC) {
    uint4 x[KC][VPL];
#pragma unroll
    for (int j = 0; j < KC; ++j)
      if (NOGUARD || i0 + j < n_in)
#pragma unroll
        for (int q = 0; q < VPL; ++q) x[j][q] = ld16<NT>(a.in[i0 + j] + off[q]);
#pragma unroll
    for (int j = 0; j < KC; ++j) {
      if (!(NOGUARD || i0 + j < n_in)) continue;
      Sel sel[VPL][4];  // H0, L0, H1, L1 planes
#pragma unroll
      for (int q = 0; q < VPL; ++q) {
        uint32_t h0, l0, h1, l1;
        split_planes(x[j][q], h0, l0, h1, l1);
        sel[q][0] = make_sel(h0);
        sel[q][1] = make_sel(l0);
        sel[q][2] = make_sel(h1);
        sel[q][3] = make_sel(l1);
      }
#pragma unroll
      for (int r = 0; r < NO; ++r) {
        if (!(NOGUARD || (uint32_t)r < n_out)) continue;
        const uint32_t base = lb + (r * n_in + i0 + j) * 4;
        const Gf8Tab hh = read_tab(tq, tt2, base + 0);
        const Gf8Tab lh = read_tab(tq, tt2, base + 1);
#pragma unroll
        for (int q = 0; q < VPL; ++q) {
          o[r][q][0] = xor3(o[r][q][0], gf8_mul4(hh, sel[q][0]), gf8_mul4(lh, sel[q][1]));
          o[r][q][2] = xor3(o[r][q][2], gf8_mul4(hh, sel[q][2]), gf8_mul4(lh, sel[q][3]));
        }
        const Gf8Tab hl = read_tab(tq, tt2, base + 2);
        const Gf8Tab ll = read_tab(tq, tt2, base + 3);
#pragma unroll
        for (int q = 0; q < VPL; ++q) {
          o[r][q][1] = xor3(o[r][q][1], gf8_mul4(hl, sel[q][0]), gf8_mul4(ll, sel[q][1]));
          o[r][q][3] = xor3(o[r][q][3], gf8_mul4(hl, sel[q][2]), gf8_mul4(ll, sel[q][3]));
        }
      }
#pragma unroll
      for (int r = 0; r < NO; ++r)
#pragma unroll
        for (int q = 0; q < VPL; ++q)
#pragma unroll
          for (int w = 0; w < 4; ++w) pin(o[r][q][w]);
    }
  }
  bool diff = false;
#pragma unroll
  for (int r = 0; r < NO; ++r) {
    if (!(NOGUARD || (uint32_t)r < n_out)) continue;
#pragma unroll
    for (int q = 0; q < VPL; ++q) {
      const uint4 ov = merge_planes(o[r][q][0], o[r][q][1], o[r][q][2], o[r][q][3]);
      if (mode != kCheck) st16<NT>(a.out[r] + off[q], ov);
      if (mode != kStore) diff |= ne4(ov, ld16<NT>(a.cmp[r] + off[q]));
    }
  }
  if (mode != kStore) flag_mismatch(diff, a, soff);
}

template <int KC, int NO, bool NOGUARD, bool NT, int VPL>
__device__ __forceinline__ void gf16_code_impl(const CodeArgs& a, uint32_t stripe0,
                                               uint32_t stripe_step) {
  __shared__ uint4 tq[kMaxIn * NO * 4];
  __shared__ uint32_t tt2[kMaxIn * NO * 4];

  const uint32_t n_in = a.n_in;
  const uint32_t n_out = NOGUARD ? NO : a.n_out;

  for (uint32_t t = threadIdx.x; t < n_out * n_in; t += kBlock) {
    const uint32_t r = t / n_in, i = t % n_in;
    uint32_t sub[4];
    gf16_sub_coefs(a.coef[r][i], sub);
#pragma unroll
    for (int q = 0; q < 4; ++q) write_tab(tq, tt2, t * 4 + q, make_gf8_tab(sub[q]));
  }
  __syncthreads();

  const uint64_t gstride = (uint64_t)gridDim.x * kBlock;
  const uint64_t gtid = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
  const uint32_t mode = a.mode;
  const uint64_t span = (uint64_t)kBlock * VPL;
  const uint64_t n_full = a.n_vec / span;

  for (uint32_t stripe = stripe0; stripe < a.n_stripes; stripe += stripe_step) {
  const uint64_t soff = (uint64_t)stripe * a.stripe_stride;

  for (uint64_t sp = blockIdx.x; sp < n_full; sp += gridDim.x)
    gf16_span<KC, NO, NOGUARD, NT, VPL>(a, tq, tt2, soff, sp * span + threadIdx.x, n_in, n_out,
                                        mode);
  for (uint64_t v = n_full * span + gtid; v < a.n_vec; v += gstride)
      gf16_span<KC, NO, NOGUARD, NT, 1>(a, tq, tt2, soff, v, n_in, n_out, mode);

  // Element tail: 2 bytes per element, byte loads (any alignment).
  for (uint64_t e = a.n_vec * 8u + gtid; e * 2u < a.len; e += gstride) {
    const uint64_t off = soff + e * 2u;
    uint32_t oh[NO], ol[NO];
#pragma unroll
    for (int r = 0; r < NO; ++r) {
      oh[r] = ol[r] = 0u;
      if (a.accumulate && (NOGUARD || (uint32_t)r < n_out)) {
        oh[r] = a.out[r][off];
        ol[r] = a.out[r][off + 1];
      }
    }
    const uint32_t lb = opaque_zero();
#pragma unroll 1
    for (uint32_t i = 0; i < n_in; ++i) {
      const Sel sh = make_sel(a.in[i][off]), sl = make_sel(a.in[i][off + 1]);
#pragma unroll
      for (int r = 0; r < NO; ++r) {
        if (!(NOGUARD || (uint32_t)r < n_out)) continue;
        const uint32_t base = lb + (r * n_in + i) * 4;
        oh[r] = xor3(oh[r], gf8_mul4(read_tab(tq, tt2, base + 0), sh), gf8_mul4(read_tab(tq, tt2, base + 1), sl));
        ol[r] = xor3(ol[r], gf8_mul4(read_tab(tq, tt2, base + 2), sh), gf8_mul4(read_tab(tq, tt2, base + 3), sl));
      }
    }
    bool diff = false;
#pragma unroll
    for (int r = 0; r < NO; ++r) {
      if (!(NOGUARD || (uint32_t)r < n_out)) continue;
      if (mode != kCheck) {
        a.out[r][off] = (uint8_t)oh[r];
        a.out[r][off + 1] = (uint8_t)ol[r];
      }
      if (mode != kStore)
        diff |= ((uint8_t)oh[r] != a.cmp[r][off]) || ((uint8_t)ol[r] != a.cmp[r][off + 1]);
    }
    if (mode != kStore && diff) flag_mismatch(mismatch_word(a, soff));
  }
  }  // stripe loop
}

template <int KC, int NO, bool NOGUARD, bool NT, int VPL>
__global__ __launch_bounds__(kBlock, VPL == 1 ? 3 : 2) void gf16_code_kernel(const CodeArgs a) {
  gf16_code_impl<KC, NO, NOGUARD, NT, VPL>(a, blockIdx.y, gridDim.y);
}

// Per-stripe (or per-block) descriptors of recon_plan_kernel, GF(2^16): row y
// of the grid codes descriptor y (as gf8_code_desc_kernel).
template <bool NT>
__global__ __launch_bounds__(kBlock, 3) void gf16_code_desc_kernel(const CodeArgs* __restrict__ descs) {
  using CPtr = const __attribute__((address_space(4))) CodeArgs*;
  const CodeArgs& a = *(const CodeArgs*)((CPtr)descs + blockIdx.y);
  if (a.n_out == 0) return;  // uniform: nothing to rebuild in this block
  gf16_code_impl<4, kMaxOut, false, NT, 1>(a, 0, 1);
}

// ---------------------------------------------------------------------------
// Chunk-pipelined GF(2^16) kernel for exact shapes (n_in == KC*CPS, n_out ==
// NO, STORE mode, no accumulate).  The unit of the software pipeline is a
// chunk of KC inputs of one span: while chunk c is coded, chunk c+1's KC loads
// (the next chunk of the same span, or the first chunk of the next span) are
// in flight.  Accumulators live across the CPS chunks of a span and are stored
// after its last chunk.  vmcnt invariant as in gf8_pipe_kernel: the only
// vector-memory operations younger than chunk c's loads are stores of the
// previous span (ignored -> stricter wait) and chunk c+1's KC loads.
struct SpanCursor {
  uint64_t stripe, local, sps, stride;
  uint32_t step;
  __device__ uint64_t off() const { return stripe * stride + (local * kBlock + threadIdx.x) * 16u; }
  __device__ void next() {
    local += step;
    while (local >= sps) { local -= sps; ++stripe; }
  }
};

template <int KC>
__device__ __forceinline__ void load_chunk(u32x4 (&x)[KC], const CodeArgs& a, int i0, uint64_t off) {
#pragma unroll
  for (int j = 0; j < KC; ++j)
    asm volatile("global_load_dwordx4 %0, %1, off nt" : "=v"(x[j]) : "v"(a.in[i0 + j] + off) : "memory");
}

template <int KC, int NO, int NB>
__device__ __forceinline__ void gf16_code_chunk(u32x4 (&x)[KC], uint32_t (&o)[NO][4],
                                                const uint4* tq, const uint32_t* tt2, int K,
                                                int i0) {
  const uint32_t lb = opaque_zero();
#pragma unroll
  for (int j = 0; j < KC; ++j) {
    wait_vm(NB + KC - 1 - j, x[j]);
    uint32_t h0, l0, h1, l1;
    split_planes(make_uint4(x[j].x, x[j].y, x[j].z, x[j].w), h0, l0, h1, l1);
    const Sel sh0 = make_sel(h0), sl0 = make_sel(l0), sh1 = make_sel(h1), sl1 = make_sel(l1);
#pragma unroll
    for (int r = 0; r < NO; ++r) {
      const uint32_t base = lb + (r * K + i0 + j) * 4;
      const Gf8Tab hh = read_tab(tq, tt2, base + 0);
      const Gf8Tab lh = read_tab(tq, tt2, base + 1);
      o[r][0] = xor3(o[r][0], gf8_mul4(hh, sh0), gf8_mul4(lh, sl0));
      o[r][2] = xor3(o[r][2], gf8_mul4(hh, sh1), gf8_mul4(lh, sl1));
      const Gf8Tab hl = read_tab(tq, tt2, base + 2);
      const Gf8Tab ll = read_tab(tq, tt2, base + 3);
      o[r][1] = xor3(o[r][1], gf8_mul4(hl, sh0), gf8_mul4(ll, sl0));
      o[r][3] = xor3(o[r][3], gf8_mul4(hl, sh1), gf8_mul4(ll, sl1));
    }
#pragma unroll
    for (int r = 0; r < NO; ++r)
#pragma unroll
      for (int w = 0; w < 4; ++w) pin(o[r][w]);
  }
}

template <int NO>
__device__ __forceinline__ void gf16_store_span(uint32_t (&o)[NO][4], const CodeArgs& a,
                                                uint64_t off) {
#pragma unroll
  for (int r = 0; r < NO; ++r) {
    st16<true>(a.out[r] + off, merge_planes(o[r][0], o[r][1], o[r][2], o[r][3]));
    o[r][0] = o[r][1] = o[r][2] = o[r][3] = 0u;
  }
}

template <int KC, int CPS, int NO>
__global__ __launch_bounds__(kBlock, 2) void gf16_pipe_kernel(const CodeArgs a) {
  constexpr int K = KC * CPS;
  __shared__ uint4 tq[K * NO * 4];
  __shared__ uint32_t tt2[K * NO * 4];
  for (uint32_t t = threadIdx.x; t < (uint32_t)(K * NO); t += kBlock) {
    uint32_t sub[4];
    gf16_sub_coefs(a.coef[t / K][t % K], sub);
#pragma unroll
    for (int q = 0; q < 4; ++q) write_tab(tq, tt2, t * 4 + q, make_gf8_tab(sub[q]));
  }
  __syncthreads();

  const uint64_t sps = a.n_vec / kBlock;
  const uint64_t total = sps * a.n_stripes;
  if (sps && blockIdx.x < total) {
    const uint64_t my_spans = (total - blockIdx.x - 1) / gridDim.x + 1;
    const uint64_t n_chunks = my_spans * CPS;
    SpanCursor ld{blockIdx.x / sps, blockIdx.x % sps, sps, a.stripe_stride, gridDim.x};
    uint32_t o[NO][4];
#pragma unroll
    for (int r = 0; r < NO; ++r) o[r][0] = o[r][1] = o[r][2] = o[r][3] = 0u;
    u32x4 xa[KC], xb[KC];
    // loader state: chunk index within span and the span's offset
    int ld_q = 0;
    uint64_t ld_off = ld.off();
    auto advance = [&]() {
      if (++ld_q == CPS) {
        ld_q = 0;
        ld.next();
        ld_off = ld.off();
      }
    };
    load_chunk<KC>(xa, a, 0, ld_off);
    int cp_q = 0;
    uint64_t cp_off = ld_off;
    advance();
    for (uint64_t c = 0;; c += 2) {
      // ---- chunk c in xa, prefetch chunk c+1 into xb
      int nq = ld_q;
      uint64_t noff = ld_off;
      if (c + 1 < n_chunks) {
        load_chunk<KC>(xb, a, nq * KC, noff);
        advance();
        gf16_code_chunk<KC, NO, KC>(xa, o, tq, tt2, K, cp_q * KC);
      } else {
        gf16_code_chunk<KC, NO, 0>(xa, o, tq, tt2, K, cp_q * KC);
      }
      if (cp_q == CPS - 1) gf16_store_span<NO>(o, a, cp_off);
      if (c + 1 >= n_chunks) break;
      cp_q = nq;
      cp_off = noff;
      // ---- chunk c+1 in xb, prefetch chunk c+2 into xa
      nq = ld_q;
      noff = ld_off;
      if (c + 2 < n_chunks) {
        load_chunk<KC>(xa, a, nq * KC, noff);
        advance();
        gf16_code_chunk<KC, NO, KC>(xb, o, tq, tt2, K, cp_q * KC);
      } else {
        gf16_code_chunk<KC, NO, 0>(xb, o, tq, tt2, K, cp_q * KC);
      }
      if (cp_q == CPS - 1) gf16_store_span<NO>(o, a, cp_off);
      if (c + 2 >= n_chunks) break;
      cp_q = nq;
      cp_off = noff;
    }
  }
  // leftovers: vectors after the last full span of every stripe, element tails
  const uint64_t gstride = (uint64_t)gridDim.x * kBlock;
  const uint64_t gtid = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
  for (uint32_t stripe = 0; stripe < a.n_stripes; ++stripe) {
    const uint64_t soff = (uint64_t)stripe * a.stripe_stride;
    for (uint64_t v = sps * kBlock + gtid; v < a.n_vec; v += gstride)
      gf16_span<KC, NO, true, true, 1>(a, tq, tt2, soff, v, K, NO, kStore);
    for (uint64_t e = a.n_vec * 8u + gtid; e * 2u < a.len; e += gstride) {
      const uint64_t off = soff + e * 2u;
      uint32_t oh[NO], ol[NO];
#pragma unroll
      for (int r = 0; r < NO; ++r) oh[r] = ol[r] = 0u;
      const uint32_t lb = opaque_zero();
#pragma unroll 1
      for (uint32_t i = 0; i < (uint32_t)K; ++i) {
        const Sel sh = make_sel(a.in[i][off]), sl = make_sel(a.in[i][off + 1]);
#pragma unroll
        for (int r = 0; r < NO; ++r) {
          const uint32_t base = lb + (r * K + i) * 4;
          oh[r] = xor3(oh[r], gf8_mul4(read_tab(tq, tt2, base + 0), sh), gf8_mul4(read_tab(tq, tt2, base + 1), sl));
          ol[r] = xor3(ol[r], gf8_mul4(read_tab(tq, tt2, base + 2), sh), gf8_mul4(read_tab(tq, tt2, base + 3), sl));
        }
      }
#pragma unroll
      for (int r = 0; r < NO; ++r) {
        a.out[r][off] = (uint8_t)oh[r];
        a.out[r][off + 1] = (uint8_t)ol[r];
      }
    }
  }
}

// ---------------------------------------------------------------------------
// Dispatch: exact instantiations for the configurations the reference's
// README / benches / BASELINE configs use; capacity-bucketed generic kernels
// (8-input chunks, up to 2/4/8/16 outputs) for everything else.  Each in a
// plain and a non-temporal flavour.
using KernelFn = void (*)(const CodeArgs);

struct Variant {
  KernelFn fn[2];  // [nt]
  bool pipe;       // gf8_pipe_kernel: STORE mode only, no accumulate, gridDim.y == 1
};
struct Shape {
  int field;
  uint32_t ni, no;
  int n;        // variants compiled
  int def;      // default variant (fastest in tools/tune.py sweeps)
  Variant v[5];
};

#define V8(KC, NO, NG, VPL) \
  { {gf8_code_kernel<KC, NO, NG, false, VPL>, gf8_code_kernel<KC, NO, NG, true, VPL>}, false }
#define V16(KC, NO, NG, VPL) \
  { {gf16_code_kernel<KC, NO, NG, false, VPL>, gf16_code_kernel<KC, NO, NG, true, VPL>}, false }
#define VP8(K, NO) \
  { {gf8_pipe_kernel<K, NO>, gf8_pipe_kernel<K, NO>}, true }
#define VP16(KC, CPS, NO) \
  { {gf16_pipe_kernel<KC, CPS, NO>, gf16_pipe_kernel<KC, CPS, NO>}, true }
static const Shape kShapes[] = {
    {8, 10, 4, 4, 1, {V8(10, 4, true, 1), V8(10, 4, true, 2), V8(5, 4, true, 2), VP8(10, 4)}},
    {8, 10, 2, 3, 1, {V8(10, 2, true, 1), V8(10, 2, true, 2), VP8(10, 2)}},
    {8, 3, 2, 1, 0, {V8(3, 2, true, 1)}},
    {8, 5, 5, 1, 0, {V8(5, 5, true, 1)}},
    {8, 2, 2, 1, 0, {V8(2, 2, true, 1)}},
    {16, 20, 8, 5, 3,
     {V16(10, 8, true, 1), VP16(5, 4, 8), VP16(4, 5, 8), V16(10, 8, true, 2), VP16(10, 2, 8)}},
};
static const Variant kGf8Generic[4] = {V8(8, 2, false, 1), V8(8, 4, false, 1), V8(8, 8, false, 1),
                                       V8(8, 16, false, 1)};
static const Variant kGf16Generic[4] = {V16(4, 2, false, 1), V16(4, 4, false, 1),
                                        V16(4, 8, false, 1), V16(4, 16, false, 1)};
#undef V8
#undef V16
#undef VP8
#undef VP16

// variant < 0 or out of range: the shape's default.  A pipelined variant is
// only used where it applies (plain encode); otherwise the first plain one.
const Variant* pick(int field, const CodeArgs& a, int64_t variant) {
  for (const Shape& sh : kShapes)
    if (sh.field == field && sh.ni == a.n_in && sh.no == a.n_out) {
      int v = (variant > 0 && variant < sh.n) ? (int)variant : sh.def;
      if (variant == 0) v = 0;
      if (sh.v[v].pipe && (a.mode != kStore || a.accumulate)) v = 0;
      return &sh.v[v];
    }
  const Variant* g = field == 8 ? kGf8Generic : kGf16Generic;
  const uint32_t no = a.n_out;
  return &g[no <= 2 ? 0 : no <= 4 ? 1 : no <= 8 ? 2 : 3];
}

// Launch-shape options (rse_set_option).  Defaults come from in-process A/B
// sweeps on MI355X (tools/tune.py; DESIGN.md "Launch shape").
struct Options {
  int64_t nontemporal = 1;        // streaming hint on shard loads/stores
  int64_t grid_x = 0;             // blocks per stripe row (0 = auto)
  int64_t stripes_in_flight = 0;  // gridDim.y (0 = all stripes at once)
  int64_t variant = -1;           // kernel variant of a tuned shape (-1 = default)
  int64_t bitslice = 1;           // bit-sliced kernels where compiled (rse_bitslice.hip)
  int64_t host_chunk_kib = 4096;  // host pipeline chunk per shard (rse_encode_host*)
  int64_t host_h2d_streams = 2;   // host pipeline H2D streams (tools/host_e2e.py)
  int64_t jit = 1;                // run-time specialised bit-sliced kernels (rse_jit.cpp)
  int64_t jit_patterns = 1;       // ... also for repeated decode patterns
  int64_t jit_cse = 32;           // GF(2^16) specialised networks: temporaries per input
  int64_t wide_lds = 1;           // wide modules: slicing shared through LDS
  int64_t jit_disk_cache = 1;     // run-time specialised modules cached on disk
  int64_t recon_mix = 3;          // syndrome reconstruct mixing: 3/2 Horner (4 steps per word / 1), 1 doubling chains, 0 tables
  int64_t wide_split = 0;         // outputs per wave of wide modules (0: auto, rse_jit.cpp wide_waves)
  int64_t wide_balance = 1;       // wide modules: waves per workgroup rounded to 2, 4, 8
  int64_t wide_occupancy = 0;     // wide modules: waves per SIMD compiled for (0 = auto)
  int64_t host_copy_2d = 1;       // host pipeline: 2D copies for runs of a flat buffer's shards
  int64_t jit_exact = 1;          // run-time networks: exact-decomposition temporaries
  int64_t wide_depth = 1;         // wide modules: inputs in flight per wave (1..4)
  int64_t recon_depth = 1;        // syndrome reconstruct: inputs in flight per lane (1..4)
  int64_t recon_pairs = 8;        // syndrome reconstruct at 8 sigma rows on wave pairs (8: by field)
  int64_t wide_pairs = 1;         // wide GF(2^8) modules: networks over pairs of inputs
  int64_t sync_event = 0;         // verify calls wait on an event, not the stream (A/B)
  int64_t spin_wait = 1;          // one-launch verifies: poll the completion word (A/B)
  int64_t host_direct = 1;        // small one-stripe host calls: one staging buffer (A/B)
  int64_t sub_chunks = 1;         // 1 / 2 KiB shards on the bit-sliced kernels (A/B)
  int64_t subfield = 1;           // GF(2^16) codecs of <= 256 shards code in GF(2^8) (A/B)
  int64_t jit_max_patterns = 64;  // decode-pattern modules per process
  int64_t jit_max_pattern_blocks = 64;  // blocks of wide decode patterns per process
  int64_t recon_w4_min = 64;      // 4 KiB syndrome chunks from this many coefficients
  int64_t wide_half = 1;          // GF(2^8) paired wide modules on 2 KiB chunks (one plane group)
  int64_t dispatch = 1;           // *_now calls on the resident dispatcher (rse_dispatch.hip)
  int64_t dispatch_idle_us = 200;  // the resident kernel ends after this long without a call
  int64_t dispatch_max_bytes = 65536;  // shard bytes up to which a *_now call is dispatched
  int64_t wide_grid = 0;          // wide launches: -1 fixed workgroup counts, m > 0 m x resident, 0 auto
  int64_t dispatch_wgs = 8;       // workgroups of the resident dispatcher
  int64_t wide_block_inputs = 128;  // data inputs per wide module of a chain (0: 8 x 32 blocks)
  int64_t dispatch_lane_units = 1;  // dispatcher: (vector, output) units per lane per workgroup
  int64_t sub_depth = 4;  // narrow modules' 1 / 2 KiB-shard kernels: inputs in flight per wave
  int64_t tune_nosync = 0;  // RSE_TUNE_SPLITS builds: wide modules without barriers (timing)
  int64_t fft = 1;  // GF(2^8) k = p = 16 / 32 / 64 codecs on the additive-FFT kernels (rse_fft.hip)
  int64_t host_queues = 1;  // host pipeline: 1 the D2H stream at high priority, 0 plain (A/B)
  int64_t host_zc_out = 1;  // host pipeline: outputs stored in place in mapped pinned memory
};
thread_local int64_t g_bs_launches = 0;  // bit-sliced launches on this thread (RSE_OPT 6)
Options g_opt;
thread_local char g_last_kernel[128] = "";  // rse_last_kernel()

// ---------------------------------------------------------------------------
// splitmix64 fill (synthetic shards; same byte stream as oracle/oracle.py).
__device__ __forceinline__ uint64_t splitmix(uint64_t z) {
  z += 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

__global__ __launch_bounds__(kBlock) void fill_splitmix_kernel(uint8_t* dst, uint64_t nbytes,
                                                               uint64_t seed, uint64_t shard) {
  const uint64_t base = seed + (shard << 40);
  const uint64_t nwords = nbytes / 8u;
  const uint64_t gstride = (uint64_t)gridDim.x * kBlock;
  const bool aligned = (reinterpret_cast<uintptr_t>(dst) & 7u) == 0;
  for (uint64_t w = (uint64_t)blockIdx.x * kBlock + threadIdx.x; w < (nbytes + 7u) / 8u;
       w += gstride) {
    const uint64_t v = splitmix(base + w);
    if (aligned && w < nwords) {
      reinterpret_cast<uint64_t*>(dst)[w] = v;
    } else {
      for (int b = 0; b < 8 && w * 8u + b < nbytes; ++b) dst[w * 8u + b] = (uint8_t)(v >> (8 * b));
    }
  }
}

// ---------------------------------------------------------------------------
// Field arithmetic of the planner and inversion kernels: log/exp of GF(2^8)'s
// generator 2 modulo 0x11D (build.rs:13-43) in LDS, exp extended to kExLen
// entries so a sum of two logs plus 7 needs no reduction.  GF(2^16) =
// GF(2^8)[x]/(x^2 + 2x + 128) (galois_16.rs:9-14, 146-162):
//   (a1 x + a0)(b1 x + b0) = (a1 b0 + a0 b1 + 2 a1 b1) x + (a0 b0 + 128 a1 b1)
// and the inverse through the norm N = a0^2 + 2 a0 a1 + 128 a1^2 (in GF(2^8)):
//   (a1 x + a0)^-1 = (a1 / N) x + (a0 + 2 a1) / N
// -- the same unique inverse as the reference's extended Euclid
// (galois_16.rs:113-144; tests/test_oracle_golden.py checks all 65535).
constexpr int kExLen = 520;
constexpr uint32_t kTabBytes = 784;  // lg[256] + ex[kExLen], rounded to 16

// Every thread computes its entries on its own (2^l by square-and-multiply,
// 14 carry-less steps) instead of one thread walking 520 doublings: the
// planner runs one workgroup per stripe, so this is per stripe.  The caller
// synchronises before use.
__device__ __forceinline__ uint32_t gf8_mul_slow(uint32_t a, uint32_t b) {  // modulo 0x11D
  uint32_t r = 0;
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    r ^= ((b >> i) & 1u) ? a : 0u;
    a = (a << 1) ^ ((a & 0x80u) ? 0x11Du : 0u);
  }
  return r;
}
__device__ __forceinline__ void build_log_exp(uint8_t* lg, uint8_t* ex) {
  for (uint32_t l = threadIdx.x; l < (uint32_t)kExLen; l += blockDim.x) {
    uint32_t e = l % 255u, r = 1u, b = 2u;
    while (e) {  // r = 2^e
      if (e & 1u) r = gf8_mul_slow(r, b);
      b = gf8_mul_slow(b, b);
      e >>= 1;
    }
    ex[l] = (uint8_t)r;
    if (l < 255u) lg[r] = (uint8_t)l;
  }
  if (threadIdx.x == 0) lg[0] = 0;
}

struct PlanF8 {
  static constexpr int kField = 8;
  __device__ static uint32_t mul(const uint8_t* lg, const uint8_t* ex, uint32_t a, uint32_t b) {
    return (a && b) ? ex[lg[a] + lg[b]] : 0u;
  }
  __device__ static uint32_t inv(const uint8_t* lg, const uint8_t* ex, uint32_t a) {  // a != 0
    return ex[255 - lg[a]];
  }
  __device__ static uint32_t load(const uint8_t* m, size_t i) { return m[i]; }
  __device__ static void store(uint8_t* m, size_t i, uint32_t v) { m[i] = (uint8_t)v; }
};

struct PlanF16 {
  static constexpr int kField = 16;
  __device__ static uint32_t mul(const uint8_t* lg, const uint8_t* ex, uint32_t a, uint32_t b) {
    const uint32_t a1 = a >> 8, a0 = a & 0xFFu, b1 = b >> 8, b0 = b & 0xFFu;
    uint32_t hi = 0, lo = 0;
    if (a1 && b1) {
      const uint32_t l = lg[a1] + lg[b1];
      hi = ex[l + 1];  // 2 a1 b1
      lo = ex[l + 7];  // 128 a1 b1
    }
    if (a1 && b0) hi ^= ex[lg[a1] + lg[b0]];
    if (a0 && b1) hi ^= ex[lg[a0] + lg[b1]];
    if (a0 && b0) lo ^= ex[lg[a0] + lg[b0]];
    return (hi << 8) | lo;
  }
  __device__ static uint32_t inv(const uint8_t* lg, const uint8_t* ex, uint32_t a) {  // a != 0
    const uint32_t a1 = a >> 8, a0 = a & 0xFFu;
    uint32_t n = 0;
    if (a0) n ^= ex[2u * lg[a0]];
    if (a0 && a1) n ^= ex[lg[a0] + lg[a1] + 1];
    if (a1) n ^= ex[2u * lg[a1] + 7];
    const uint32_t li = 255u - lg[n];  // n != 0 for a != 0
    const uint32_t c = a0 ^ (a1 ? ex[lg[a1] + 1] : 0u);
    return ((a1 ? (uint32_t)ex[lg[a1] + li] : 0u) << 8) | (c ? ex[lg[c] + li] : 0u);
  }
  // [u8;2] elements {coefficient of x, constant} (galois_16.rs:49-51)
  __device__ static uint32_t load(const uint8_t* m, size_t i) {
    return ((uint32_t)m[2 * i] << 8) | m[2 * i + 1];
  }
  __device__ static void store(uint8_t* m, size_t i, uint32_t v) {
    m[2 * i] = (uint8_t)(v >> 8);
    m[2 * i + 1] = (uint8_t)v;
  }
};

// Gauss-Jordan on the n x 2n augmented matrix w (row stride 2n) by the whole
// workgroup (matrix.rs:195-261: the same unique inverse -- the pivot choice
// cannot change the result of an exact field).  False if singular (uniform).
template <class F>
__device__ bool gauss_jordan(uint16_t* w, uint32_t n, const uint8_t* lg, const uint8_t* ex,
                             int* s_piv) {
  const uint32_t tid = threadIdx.x, nt = blockDim.x, w2 = 2 * n;
  for (uint32_t col = 0; col < n; ++col) {
    if (tid == 0) {
      int piv = -1;
      for (uint32_t r = col; r < n; ++r)
        if (w[r * w2 + col]) {
          piv = (int)r;
          break;
        }
      *s_piv = piv;
    }
    __syncthreads();
    const int piv = *s_piv;
    if (piv < 0) return false;
    if ((uint32_t)piv != col) {
      for (uint32_t c = tid; c < w2; c += nt) {
        const uint16_t t0 = w[col * w2 + c];
        w[col * w2 + c] = w[piv * w2 + c];
        w[piv * w2 + c] = t0;
      }
      __syncthreads();
    }
    const uint32_t inv = F::inv(lg, ex, w[col * w2 + col]);
    __syncthreads();  // every thread has read the pivot before the row is scaled
    for (uint32_t c = tid; c < w2; c += nt)
      w[col * w2 + c] = (uint16_t)F::mul(lg, ex, inv, w[col * w2 + c]);
    __syncthreads();
    for (uint32_t t = tid; t < n * w2; t += nt) {  // eliminate column `col` elsewhere
      const uint32_t r = t / w2, c = t % w2;
      if (r == col || c == col) continue;
      const uint32_t f = w[r * w2 + col];
      if (f) w[t] ^= (uint16_t)F::mul(lg, ex, f, w[col * w2 + c]);
    }
    __syncthreads();
    for (uint32_t r = tid; r < n; r += nt)
      if (r != col) w[r * w2 + col] = 0;
    __syncthreads();
  }
  return true;
}

// Batched inversion, one workgroup per n x n matrix (row-major, the field's
// element bytes), [M | I] in LDS -- or, past kInvLds, in a global workspace
// of batch x n x 2n elements (gws).  singular[b] = 1 for a singular matrix
// (matrix.rs:11-13 Error::SingularMatrix), and out[b] is then left unwritten.
constexpr uint32_t kInvLds = 65536 - kTabBytes - 16;

template <class F>
__global__ __launch_bounds__(1024) void invert_kernel(const uint8_t* in, uint8_t* out,
                                                      uint32_t* singular, uint32_t n,
                                                      uint16_t* gws) {
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  uint8_t* lg = smem;
  uint8_t* ex = smem + 256;
  int* s_piv = reinterpret_cast<int*>(smem + kTabBytes);
  uint16_t* w = gws ? gws + (size_t)blockIdx.x * n * 2 * n
                    : reinterpret_cast<uint16_t*>(smem + kTabBytes + 16);
  const uint32_t tid = threadIdx.x, nt = blockDim.x, w2 = 2 * n;
  const uint8_t* m = in + (size_t)blockIdx.x * n * n * (F::kField / 8);
  build_log_exp(lg, ex);
  for (uint32_t t = tid; t < n * w2; t += nt) {
    const uint32_t r = t / w2, c = t % w2;
    w[t] = (uint16_t)(c < n ? F::load(m, (size_t)r * n + c) : ((c - n) == r ? 1u : 0u));
  }
  __syncthreads();
  if (!gauss_jordan<F>(w, n, lg, ex, s_piv)) {
    if (tid == 0) singular[blockIdx.x] = 1u;
    return;
  }
  uint8_t* o = out + (size_t)blockIdx.x * n * n * (F::kField / 8);
  for (uint32_t t = tid; t < n * n; t += nt) F::store(o, t, w[(t / n) * w2 + n + (t % n)]);
  if (tid == 0) singular[blockIdx.x] = 0u;
}

// ---------------------------------------------------------------------------
// Device reconstruct planner, one workgroup per stripe, either field, any codec
// whose batch fits the LDS budget (recon_plan_lds): the planning of
// core.rs:733-923 for the stripe's own erasure pattern, written as CodeArgs
// descriptors for the table kernels' descriptor variants.
//  * valid = the first k present shards in index order (core.rs:801-841): the
//    k - e present data shards, then R, the first e present parity rows;
//    S = the e missing data shards; outputs = missing data, then (unless
//    data_only) missing parity, ascending.
//  * Only the e x e matrix A = P[R][S] is inverted (Gauss-Jordan in LDS): the
//    k x k decode matrix of core.rs:711-722 restricted to what the outputs
//    need.  With W[o] = A^-1 row u for missing data S_u, and
//    W[o] = sum_u P[r][S_u] A^-1[u] for missing parity r, the composed row
//    over the valid inputs is
//        on parity input R_t:     W[o][t]
//        on present data d:       [r missing: P[r][d]] + sum_t W[o][t] P[R_t][d]
//    -- the unique linear map from the k valid shards to each output, so the
//    bytes equal the host planner's (plan_reconstruct) and the reference's.
//  * Descriptor (ib, ob) of a stripe codes outputs [16 ob, 16 ob + 16) from
//    inputs [32 ib, 32 ib + 32), accumulating for ib > 0; descs[(ib * n_grp +
//    stripe) * n_ob + ob].  A block with nothing to rebuild gets n_out = 0.
// Layout of the dynamic LDS: tables | ints | valid[k] | miss[T] | S[e_cap] |
// R[e_cap] | A[e_cap][2 e_cap] | W[nout_cap][e_cap] (uint16).
template <class F>
__global__ __launch_bounds__(256) void recon_plan_kernel(
    const uint16_t* __restrict__ P, const uint8_t* __restrict__ present, uint32_t k, uint32_t T,
    uint32_t data_only, uint32_t e_cap, uint8_t* base, uint64_t shard_bytes, uint64_t off,
    uint64_t len, uint64_t n_vec, uint32_t n_grp, uint32_t n_ib, uint32_t n_ob, CodeArgs* descs) {
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  uint8_t* lg = smem;
  uint8_t* ex = smem + 256;
  int* sc = reinterpret_cast<int*>(smem + kTabBytes);  // e, n_out, pivot, ok
  uint16_t* valid = reinterpret_cast<uint16_t*>(smem + kTabBytes + 16);
  uint16_t* miss = valid + k;
  uint16_t* S = miss + T;
  uint16_t* R = S + e_cap;
  uint16_t* A = R + e_cap;
  uint16_t* W = A + 2 * e_cap * e_cap;
  const uint32_t sl = blockIdx.x, tid = threadIdx.x, nt = blockDim.x;
  const uint8_t* pres = present + (size_t)sl * T;
  build_log_exp(lg, ex);
  if (tid == 0) {
    uint32_t nv = 0, ne = 0, nr = 0, nm = 0;
    for (uint32_t row = 0; row < T; ++row) {
      if (pres[row]) {
        if (nv < k) {
          valid[nv++] = (uint16_t)row;
          if (row >= k) R[nr++] = (uint16_t)(row - k);
        }
      } else if (row < k) {
        S[ne++] = (uint16_t)row;
        miss[nm++] = (uint16_t)row;
      } else if (!data_only) {
        miss[nm++] = (uint16_t)row;
      }
    }
    sc[0] = (int)ne;
    sc[1] = (int)nm;
    sc[3] = 1;
  }
  __syncthreads();
  const uint32_t e = (uint32_t)sc[0], nm = (uint32_t)sc[1];
  if (e) {  // [A | I], then A^-1 in the right half
    const uint32_t w2 = 2 * e;
    for (uint32_t t = tid; t < e * w2; t += nt) {
      const uint32_t r = t / w2, c = t % w2;
      A[t] = c < e ? P[(size_t)R[r] * k + S[c]] : (uint16_t)((c - e) == r ? 1 : 0);
    }
    __syncthreads();
    if (!gauss_jordan<F>(A, e, lg, ex, &sc[2]) && tid == 0) sc[3] = 0;  // impossible for MDS
    __syncthreads();
    for (uint32_t t = tid; t < nm * e; t += nt) {
      const uint32_t o = t / e, u = t % e, m = miss[o];
      uint32_t v = 0;
      if (m < k) {
        v = A[o * w2 + e + u];  // outputs o < e are S in order
      } else {
        for (uint32_t q = 0; q < e; ++q)
          v ^= F::mul(lg, ex, P[(size_t)(m - k) * k + S[q]], A[q * w2 + e + u]);
      }
      W[o * e + u] = (uint16_t)v;
    }
  }
  __syncthreads();
  const uint32_t n_out = sc[3] ? nm : 0u;  // singular: leave the stripe untouched
  uint8_t* sbase = base + (uint64_t)sl * T * shard_bytes + off;
  for (uint32_t b = tid; b < n_ib * n_ob; b += nt) {
    const uint32_t ib = b / n_ob, ob = b % n_ob;
    CodeArgs& d = descs[((size_t)ib * n_grp + sl) * n_ob + ob];
    const uint32_t ni = k - 32 * ib < 32u ? k - 32 * ib : 32u;
    const uint32_t no = 16 * ob < n_out ? (n_out - 16 * ob < 16u ? n_out - 16 * ob : 16u) : 0u;
    d.n_in = ni;
    d.n_out = no;
    d.n_stripes = 1;
    d.stripe_stride = 0;
    d.n_vec = n_vec;
    d.len = len;
    d.mismatch = nullptr;
    d.mode = kStore;
    d.accumulate = ib > 0 ? 1u : 0u;
    d.per_stripe = 0;
    d.done = nullptr;
    d.done_count = nullptr;
    for (uint32_t i = 0; i < ni; ++i) d.in[i] = sbase + (uint64_t)valid[32 * ib + i] * shard_bytes;
    for (uint32_t o = 0; o < no; ++o) {
      d.out[o] = sbase + (uint64_t)miss[16 * ob + o] * shard_bytes;
      d.cmp[o] = nullptr;
    }
  }
  for (uint32_t t = tid; t < n_out * k; t += nt) {
    const uint32_t o = t / k, i = t % k, v = valid[i], m = miss[o];
    uint32_t c;
    if (v >= k) {
      c = W[o * e + (i - (k - e))];
    } else {
      c = m >= k ? P[(size_t)(m - k) * k + v] : 0u;
      for (uint32_t q = 0; q < e; ++q) c ^= F::mul(lg, ex, W[o * e + q], P[(size_t)R[q] * k + v]);
    }
    descs[((size_t)(i / 32) * n_grp + sl) * n_ob + o / 16].coef[o % 16][i % 32] = (uint16_t)c;
  }
}

}  // namespace

hipError_t launch_code(int field, const CodeArgs& args, hipStream_t stream) {
  if (args.n_in == 0 || args.n_in > (uint32_t)kMaxIn || args.n_out == 0 ||
      args.n_out > (uint32_t)kMaxOut || args.n_stripes == 0)
    return hipErrorInvalidValue;
  if (g_opt.bitslice) {
    bool handled = false;
    uint64_t done = 0;
    hipError_t e = launch_bitslice(field, args, g_opt.nontemporal != 0, g_opt.grid_x, stream,
                                   &handled, &done);
    if (e != hipSuccess) return e;
    if (handled) {
      ++g_bs_launches;
      // the bit-sliced kernels code whole chunks; the rest goes to the table kernels
      if (done == args.len) return hipSuccess;
      CodeArgs r = args;
      for (uint32_t i = 0; i < r.n_in; ++i) r.in[i] += done;
      for (uint32_t o = 0; o < r.n_out; ++o) {
        if (r.out[o]) r.out[o] += done;  // null in kCheck mode
        if (r.cmp[o]) r.cmp[o] += done;
      }
      r.len -= done;
      r.n_vec -= done / 16u;
      char keep[sizeof g_last_kernel];  // the bit-sliced launch is the one to report
      __builtin_memcpy(keep, g_last_kernel, sizeof keep);
      e = launch_table(field, r, stream);
      __builtin_memcpy(g_last_kernel, keep, sizeof keep);
      return e;
    }
  }
  return launch_table(field, args, stream);
}

hipError_t launch_table(int field, const CodeArgs& args, hipStream_t stream) {
  const Variant* var = pick(field, args, g_opt.variant);
  KernelFn fn = var->fn[g_opt.nontemporal ? 1 : 0];
  note_kernel("table gf%d %u+%u %s nt%d", field, args.n_in, args.n_out,
              var->pipe ? "pipe" : "fused", (int)g_opt.nontemporal);
  uint64_t gy = g_opt.stripes_in_flight > 0 ? (uint64_t)g_opt.stripes_in_flight : args.n_stripes;
  if (gy > args.n_stripes) gy = args.n_stripes;
  if (gy > 65535) gy = 65535;
  if (var->pipe) gy = 1;
  const uint64_t units = args.n_vec ? args.n_vec : (args.len + 1u);
  const uint64_t want = (units + kBlock - 1) / kBlock;
  // ~2048 workgroups over the chip in total, never more per stripe row than
  // the row has vectors for (idle workgroups still build their LDS tables:
  // 16 per row at 1 KiB shards ran 13x slower than 1, tools/small_session.sh)
  uint64_t gx = g_opt.grid_x > 0 ? (uint64_t)g_opt.grid_x : (2048u + gy - 1) / gy;
  if (gx > want) gx = want;
  if (gx < 1) gx = 1;
  hipLaunchKernelGGL(fn, dim3((uint32_t)gx, (uint32_t)gy, 1), dim3(kBlock, 1, 1), 0, stream, args);
  return hipGetLastError();
}

size_t recon_plan_lds(uint32_t k, uint32_t T, uint32_t e_cap, uint32_t nout_cap) {
  return kTabBytes + 16 +
         2 * ((size_t)k + T + 2 * (size_t)e_cap + 2 * (size_t)e_cap * e_cap + (size_t)nout_cap * e_cap);
}

// One lane per stripe: the per-stripe counts of the host loop in
// rse_reconstruct_batch, reduced over the wave before one atomic each.  With
// at most kScanStageT flags per stripe the workgroup first copies its 256
// stripes' flags into LDS, consecutive bytes per lane (a lane reading its own
// stripe's flags from HBM is k + p dependent loads, 28 round trips at 20+8:
// 39 us for 65536 stripes, profiles/r04/s9/b4k_trace/), then scans from LDS.
constexpr uint32_t kScanStageT = 128;
__global__ __launch_bounds__(256) void batch_scan_kernel(const uint8_t* __restrict__ present,
                                                         uint64_t n, uint32_t k, uint32_t p,
                                                         uint32_t data_only, uint32_t* res) {
  __shared__ uint8_t fl[256 * kScanStageT];
  const uint32_t T = k + p;
  const uint64_t s0 = (uint64_t)blockIdx.x * blockDim.x, s = s0 + threadIdx.x;
  const bool staged = T <= kScanStageT;
  if (staged) {
    const uint64_t rows = n - s0 < 256 ? n - s0 : 256;
    const uint32_t nb = (uint32_t)(rows * T);
    const uint8_t* src = present + s0 * T;
#pragma unroll 8
    for (uint32_t i = threadIdx.x; i < nb; i += 256) fl[i] = src[i];
    __syncthreads();
  }
  uint32_t need = 0, ne = 0, nout = 0;
  unsigned long long err = ~0ull;
  if (s < n) {
    const uint8_t* pr = staged ? fl + threadIdx.x * T : present + s * T;
    for (uint32_t j = 0; j < k; ++j) ne += pr[j] ? 0u : 1u;
    uint32_t np = k - ne, nr = 0, nmp = 0;
    for (uint32_t r = 0; r < p; ++r) {
      const bool here = pr[k + r] != 0;
      np += here ? 1u : 0u;
      const bool syn = here && nr < ne;
      nr += syn ? 1u : 0u;
      if (!here && !data_only) ++nmp;
      if (syn || (!here && !data_only)) need = r + 1;
    }
    nout = ne + nmp;
    if (np < k) err = (unsigned long long)s * 2 + 1;
  }
  for (int m = 32; m > 0; m >>= 1) {
    need = max(need, (uint32_t)__shfl_xor((int)need, m));
    ne = max(ne, (uint32_t)__shfl_xor((int)ne, m));
    nout = max(nout, (uint32_t)__shfl_xor((int)nout, m));
    const unsigned long long o = __shfl_xor(err, m);
    err = o < err ? o : err;
  }
  // the workgroup's 4 waves through LDS, then one lane; an atomic only where
  // it would raise the word (the words agree across most workgroups, and
  // 4096 atomics on 4 addresses serialise: the scan took 40 us for 65536
  // stripes with them, profiles/r04/s10/b4k_trace/)
  __shared__ uint32_t wr[4][3];
  __shared__ unsigned long long we[4];
  const uint32_t wv = threadIdx.x >> 6;
  if ((threadIdx.x & 63u) == 0) {
    wr[wv][0] = need;
    wr[wv][1] = ne;
    wr[wv][2] = nout;
    we[wv] = err;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    for (uint32_t w = 1; w < blockDim.x / 64u; ++w) {
      need = max(need, wr[w][0]);
      ne = max(ne, wr[w][1]);
      nout = max(nout, wr[w][2]);
      err = we[w] < err ? we[w] : err;
    }
    const uint32_t v[3] = {need, ne, nout};
    for (int q = 0; q < 3; ++q)
      if (v[q] > __hip_atomic_load(&res[q], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT))
        atomicMax(&res[q], v[q]);
    if (err != ~0ull) atomicMin(reinterpret_cast<unsigned long long*>(res + 4), err);
  }
}

hipError_t launch_batch_scan(const uint8_t* d_present, uint64_t n_stripes, uint32_t k, uint32_t p,
                             uint32_t data_only, uint32_t* d_res, hipStream_t stream) {
  if (n_stripes == 0) return hipSuccess;
  hipLaunchKernelGGL(batch_scan_kernel, dim3((uint32_t)((n_stripes + 255) / 256)), dim3(256), 0,
                     stream, d_present, n_stripes, k, p, data_only, d_res);
  return hipGetLastError();
}

hipError_t launch_recon_plan(int field, const uint16_t* d_parity, const uint8_t* d_present,
                             uint32_t k, uint32_t T, uint32_t data_only, uint32_t e_cap,
                             uint32_t nout_cap, uint8_t* base, uint64_t shard_bytes, uint64_t off,
                             uint64_t len, uint32_t n_grp, CodeArgs* d_descs, hipStream_t stream) {
  const size_t lds = recon_plan_lds(k, T, e_cap, nout_cap);
  if (k == 0 || T <= k || nout_cap == 0 || n_grp == 0 || off + len > shard_bytes || len == 0 ||
      lds > kReconPlanLdsMax || (field != 8 && field != 16))
    return hipErrorInvalidValue;
  const bool al = (reinterpret_cast<uintptr_t>(base + off) % 16u) == 0 && shard_bytes % 16u == 0;
  const uint64_t n_vec = al ? len / 16u : 0;
  const uint32_t n_ib = (k + 31) / 32, n_ob = (nout_cap + 15) / 16;
  hipLaunchKernelGGL(field == 8 ? recon_plan_kernel<PlanF8> : recon_plan_kernel<PlanF16>,
                     dim3(n_grp), dim3(256), lds, stream, d_parity, d_present, k, T, data_only,
                     e_cap, base, shard_bytes, off, len, n_vec, n_grp, n_ib, n_ob, d_descs);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  const uint64_t rows = (uint64_t)n_grp * n_ob;  // descriptors per input block
  const uint64_t units = n_vec ? n_vec : (field == 8 ? len : len / 2) + 1;
  uint64_t gx = (2048u + rows - 1) / rows;
  const uint64_t want = (units + kBlock - 1) / kBlock;
  if (gx > want) gx = want;
  if (gx < 1) gx = 1;
  void (*fn)(const CodeArgs*) =
      field == 8 ? (g_opt.nontemporal ? gf8_code_desc_kernel<true> : gf8_code_desc_kernel<false>)
                 : (g_opt.nontemporal ? gf16_code_desc_kernel<true> : gf16_code_desc_kernel<false>);
  note_kernel("table-desc gf%d %u+%u", field, k, T - k);
  for (uint32_t ib = 0; ib < n_ib; ++ib)  // later input blocks accumulate: stream order
    for (uint64_t y0 = 0; y0 < rows; y0 += 65535u) {
      const uint32_t gy = (uint32_t)(rows - y0 < 65535u ? rows - y0 : 65535u);
      hipLaunchKernelGGL(fn, dim3((uint32_t)gx, gy, 1), dim3(kBlock, 1, 1), 0, stream,
                         d_descs + (size_t)ib * rows + y0);
      e = hipGetLastError();
      if (e != hipSuccess) return e;
    }
  return hipSuccess;
}

int set_option(int key, int64_t value) {
  switch (key) {
    case 1: g_opt.nontemporal = value ? 1 : 0; return 0;
    case 2: g_opt.grid_x = value < 0 ? 0 : value; return 0;
    case 3: g_opt.stripes_in_flight = value < 0 ? 0 : value; return 0;
    case 4: g_opt.variant = value; return 0;
    case 5: g_opt.bitslice = value ? 1 : 0; return 0;
    case 7: g_opt.host_chunk_kib = value < 64 ? 64 : value; return 0;
    case 8: g_opt.host_h2d_streams = value < 1 ? 1 : value > 4 ? 4 : value; return 0;
    case 9: g_opt.jit = value < 0 ? 0 : value > 2 ? 2 : value; return 0;
    case 11: g_opt.jit_patterns = value ? 1 : 0; return 0;
    case 13: g_opt.jit_cse = value < 0 ? 0 : value > 32 ? 32 : value; return 0;
    case 14: g_opt.wide_lds = value ? 1 : 0; return 0;
    case 15: g_opt.jit_disk_cache = value ? 1 : 0; return 0;
    case 17: g_opt.recon_mix = value < 0 ? 0 : value > 3 ? 3 : value; return 0;
    case 18: g_opt.wide_split = value <= 0 ? 0 : value < 2 ? 2 : value > 8 ? 8 : value; return 0;
    case 19: g_opt.wide_balance = value ? 1 : 0; return 0;
    case 20: g_opt.wide_occupancy = value < 0 ? 0 : value > 4 ? 4 : value == 1 ? 2 : value; return 0;
    case 21: g_opt.host_copy_2d = value ? 1 : 0; return 0;
    case 23: g_opt.jit_exact = value ? 1 : 0; return 0;
    case 26: g_opt.wide_depth = value < 1 ? 1 : value > 4 ? 4 : value; return 0;
    case 27: g_opt.recon_depth = value < 1 ? 1 : value > 4 ? 4 : value; return 0;
    case 28:
#ifndef RSE_TUNE_SPLITS
      // 4 / 5 select the timing splits, which write wrong bytes: tools/tune.py's
      // -DRSE_TUNE_SPLITS build only (rse_bitslice.hip RSE_SPLIT_FN)
      if (value == 4 || value == 5) return -2;
#endif
      g_opt.recon_pairs = value < 0 ? 0 : value > 8 ? 8 : value;
      return 0;
    case 29: g_opt.wide_pairs = value ? 1 : 0; return 0;
    case 30: g_opt.sync_event = value ? 1 : 0; return 0;
    case 31: g_opt.spin_wait = value ? 1 : 0; return 0;
    case 32: g_opt.host_direct = value ? 1 : 0; return 0;
    case 33: g_opt.sub_chunks = value ? 1 : 0; return 0;
    case 34: g_opt.subfield = value ? 1 : 0; return 0;
    case 35: g_opt.jit_max_patterns = value < 0 ? 0 : value; return 0;
    case 36: g_opt.jit_max_pattern_blocks = value < 0 ? 0 : value; return 0;
    case 37: g_opt.recon_w4_min = value < 0 ? 0 : value; return 0;
    case 38: g_opt.wide_half = value ? 1 : 0; return 0;
    case 39: g_opt.dispatch = value ? 1 : 0; return 0;
    case 40: g_opt.dispatch_idle_us = value < 10 ? 10 : value > 1000000 ? 1000000 : value; return 0;
    case 41: g_opt.dispatch_max_bytes = value < 0 ? 0 : value; return 0;
    case 44: g_opt.wide_grid = value < -1 ? -1 : value > 64 ? 64 : value; return 0;
    case 45: g_opt.dispatch_wgs = value < 1 ? 1 : value > 64 ? 64 : value; return 0;
    case 46: g_opt.wide_block_inputs = value < 0 ? 0 : value; return 0;
    case 49: g_opt.dispatch_lane_units = value < 1 ? 1 : value > 64 ? 64 : value; return 0;
    case 50: g_opt.sub_depth = value < 1 ? 1 : value > 4 ? 4 : value; return 0;
    case 51: g_opt.fft = value ? 1 : 0; return 0;
    case 52: g_opt.host_queues = value ? 1 : 0; return 0;
    case 53: g_opt.host_zc_out = value ? 1 : 0; return 0;
#ifdef RSE_TUNE_SPLITS
    case 47: g_opt.tune_nosync = value ? 1 : 0; return 0;  // rse_jit.cpp make_source
#endif
    default: return -1;
  }
}

void count_bitslice_launch() { ++g_bs_launches; }

void note_kernel(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  std::vsnprintf(g_last_kernel, sizeof g_last_kernel, fmt, ap);
  va_end(ap);
}
const char* last_kernel() { return g_last_kernel; }

int64_t get_option(int key) {
  switch (key) {
    case 1: return g_opt.nontemporal;
    case 2: return g_opt.grid_x;
    case 3: return g_opt.stripes_in_flight;
    case 4: return g_opt.variant;
    case 5: return g_opt.bitslice;
    case 6: return g_bs_launches;
    case 7: return g_opt.host_chunk_kib;
    case 8: return g_opt.host_h2d_streams;
    case 9: return g_opt.jit;
    case 10: return jit_modules_built();
    case 11: return g_opt.jit_patterns;
    case 13: return g_opt.jit_cse;
    case 14: return g_opt.wide_lds;
    case 15: return g_opt.jit_disk_cache;
    case 16: return jit_cache_hits();
    case 17: return g_opt.recon_mix;
    case 18: return g_opt.wide_split;
    case 19: return g_opt.wide_balance;
    case 20: return g_opt.wide_occupancy;
    case 21: return g_opt.host_copy_2d;
    case 23: return g_opt.jit_exact;
    case 26: return g_opt.wide_depth;
    case 27: return g_opt.recon_depth;
    case 28: return g_opt.recon_pairs;
    case 29: return g_opt.wide_pairs;
    case 30: return g_opt.sync_event;
    case 31: return g_opt.spin_wait;
    case 32: return g_opt.host_direct;
    case 33: return g_opt.sub_chunks;
    case 34: return g_opt.subfield;
    case 35: return g_opt.jit_max_patterns;
    case 36: return g_opt.jit_max_pattern_blocks;
    case 37: return g_opt.recon_w4_min;
    case 38: return g_opt.wide_half;
    case 39: return g_opt.dispatch;
    case 40: return g_opt.dispatch_idle_us;
    case 41: return g_opt.dispatch_max_bytes;
    case 44: return g_opt.wide_grid;
    case 45: return g_opt.dispatch_wgs;
    case 46: return g_opt.wide_block_inputs;
    case 49: return g_opt.dispatch_lane_units;
    case 50: return g_opt.sub_depth;
    case 51: return g_opt.fft;
    case 52: return g_opt.host_queues;
    case 53: return g_opt.host_zc_out;
#ifdef RSE_TUNE_SPLITS
    case 47: return g_opt.tune_nosync;
#endif
    default: return -1;
  }
}

hipError_t launch_fill_splitmix(void* dst, uint64_t nbytes, uint64_t seed, uint64_t shard_id,
                                hipStream_t stream) {
  if (nbytes == 0) return hipSuccess;
  uint64_t blocks = ((nbytes + 7) / 8 + kBlock - 1) / kBlock;
  if (blocks > 8192) blocks = 8192;
  hipLaunchKernelGGL(fill_splitmix_kernel, dim3((uint32_t)blocks), dim3(kBlock), 0, stream,
                     static_cast<uint8_t*>(dst), nbytes, seed, shard_id);
  return hipGetLastError();
}

hipError_t launch_invert(int field, const uint8_t* in, uint8_t* out, uint32_t* singular,
                         uint32_t n, uint32_t batch, uint16_t* gws, hipStream_t stream) {
  if (n == 0 || batch == 0 || (field != 8 && field != 16) || (field == 8 && n > 255))
    return hipErrorInvalidValue;
  const size_t w = (size_t)n * 2 * n * 2;
  if (!gws && w > kInvLds) return hipErrorInvalidValue;
  const size_t lds = kTabBytes + 16 + (gws ? 0 : w);
  auto fn = field == 8 ? invert_kernel<PlanF8> : invert_kernel<PlanF16>;
  hipLaunchKernelGGL(fn, dim3(batch), dim3(1024), lds, stream, in, out, singular, n, gws);
  return hipGetLastError();
}

size_t invert_lds_max_bytes() { return kInvLds; }

}  // namespace rse
