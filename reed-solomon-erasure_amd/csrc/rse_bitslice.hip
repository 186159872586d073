// rse_bitslice.hip -- bit-sliced encode/verify/reconstruct kernels for the
// codecs whose parity matrix is compiled into the library (GF(2^8) 10+4 and
// 10+2, GF(2^16) 20+8: the configurations BASELINE.json names), plus the
// dispatch that also serves codecs specialised at run time (rse_jit.cpp).
//
// Why: the table kernels in rse_kernels.hip spend 3 v_perm_b32 per GF(2^8)
// constant multiply and dword (4 GF(2^8) multiplies per GF(2^16) coefficient),
// which makes GF(2^16) VALU-bound far below HBM speed.  With the data
// bit-sliced (rse_bitslice_core.hpp) a multiply-accumulate is an XOR network
// fixed by the coefficient.  The encoding matrix of ReedSolomon::new (core.rs:
// 430-436, V * (V_top)^-1) depends only on (k, p), so for the configurations
// instantiated here its parity rows, and the bit matrices of every coefficient,
// are evaluated by constexpr code and the XOR network is straight-line code with
// no tables and no memory other than the shards.  The host checks that a
// launch's coefficients equal the compiled ones before dispatching here
// (anything else takes the table kernels), so a matrix mismatch can only cost
// speed, never correctness.
#include <atomic>
#include "rse_bitslice_core.hpp"

namespace rse {
namespace {

// bitslice_kernel variant (tools/tune.py sweeps): GF(2^8) 5 (two inputs in
// flight per lane: 10+4 x 16 MiB 6014-6072 GB/s against 5961-5994 for 1, the
// scheduling barrier, in three processes on two boxes, profiles/r03/s12, s13;
// 10+2 x 1 MiB the same within noise); GF(2^16), VALU-heavier, 0 (the
// scheduler's own interleaving)
constexpr int kBsDefaultVariant8 = 5, kBsDefaultVariant16 = 0;

// ------------------------------------------------------- compiled codecs
// The code structs of the compiled codecs -- their parity rows (core.rs:430-436,
// V * (V[0..K])^-1) and the XOR networks of those rows -- generated at build time
// by rse_gen_tables.cpp with the generator the run-time specialisation uses
// (rse_netgen.hpp): Bs8_10_4, Bs8_10_2, Bs16_20_8, and *Plain twins without
// shared subexpressions (kernel variant 9, for A/B).
#include "rse_bs_tables.inc"

template <class C, bool NT, bool SB, bool XC, bool XM = false, bool WT = false, bool W4 = false,
          bool CE = false, uint32_t SUB = 0>
__global__ __launch_bounds__(kBsBlock, C::p > 4 ? 2 : 3) void bitslice_kernel(
    const CodeArgs a, uint64_t chunks_per_stripe) {
  bitslice_body<C, NT, SB, XC, XM, WT, W4, false, CE, SUB>(a, chunks_per_stripe);
  if constexpr (CE) signal_done(a);
}

template <class C, int D>
__global__ __launch_bounds__(kBsBlock, C::p > 4 ? 2 : 3) void bitslice_deep_kernel(
    const CodeArgs a, uint64_t chunks_per_stripe) {
  bitslice_body_deep<C, true, D>(a, chunks_per_stripe);
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
    mac_input<C, I, false>(acc, pl, make_int_seq<C::p * 16>{});
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
    if (a.per_stripe && diff) {
      flag_mismatch(a.mismatch + (blockIdx.x + c * gridDim.x) / chunks_per_stripe);
      diff = false;
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // no DMA outlives the wave
  if (mode != kStore && diff) flag_mismatch(a.mismatch);
}

template <class C, bool NT, int NS, int MIX>
__global__ __launch_bounds__(kBsBlock, NS > 4 ? 2 : 3) void bitslice_recon_kernel(
    const BsReconArgs a, uint64_t chunks_per_stripe) {
  bitslice_recon_body<C, NT, NS, MIX>(a, chunks_per_stripe);
}

template <class C, bool NT, int NS>
__global__ __launch_bounds__(kBsBlock, NS > 4 ? 2 : 3) void bitslice_recon_desc_kernel(
    const BsReconArgs* descs, uint64_t chunks_per_stripe, uint64_t n_stripes) {
  bitslice_recon_desc_body<C, NT, NS>(descs, chunks_per_stripe, n_stripes);
}

template <class C, int NS>
__global__ __launch_bounds__(kBsBlock, NS > 4 ? 2 : 3) void bitslice_recon_desc_w4_kernel(
    const BsReconArgs* descs, uint64_t cps4, uint64_t n_stripes, uint64_t base) {
  bitslice_recon_desc_body_w4<C, true, NS>(descs, cps4, n_stripes, base);
}

template <class C, int NS>
__global__ __launch_bounds__(kBsBlock, NS > 4 ? 2 : 3) void bitslice_recon_w4_kernel(
    const BsReconArgs a, uint64_t cps4, uint64_t base) {
  bitslice_recon_body_w4<C, true, NS>(a, cps4, base);
}

// The same with D inputs in flight per lane (RSE_OPT_RECON_DEPTH; Horner mixing).
template <class C, int NS, int D>
__global__ __launch_bounds__(kBsBlock, NS > 4 ? 2 : 3) void bitslice_recon_deep_kernel(
    const BsReconArgs a, uint64_t chunks_per_stripe) {
  bitslice_recon_body_deep<C, true, NS, D>(a, chunks_per_stripe);
}

template <class C, int NS, int D>
__global__ __launch_bounds__(kBsBlock, NS > 4 ? 2 : 3) void bitslice_recon_desc_deep_kernel(
    const BsReconArgs* descs, uint64_t chunks_per_stripe, uint64_t n_stripes) {
  bitslice_recon_desc_body_deep<C, true, NS, D>(descs, chunks_per_stripe, n_stripes);
}

// 8 sigma rows on wave pairs (RSE_OPT_RECON_PAIRS; Horner mixing, 3 waves/SIMD),
// P pairs per workgroup.
// PF: the next unit's first input loaded during the mixing (A/B, option 28 = 3).
// DBG: 4 two own inputs in flight per wave (the default); A/B variants
// (RSE_OPT_RECON_PAIRS 4-6): 1 / 2 skip the Horner steps / the data networks
// (tune-only timing splits, wrong bytes), 3 the compact mixing.
template <class C, int P, bool PF = false, int DBG = 0>
__global__ __launch_bounds__(128 * P, 3) void bitslice_recon_pair_kernel(
    const BsReconArgs a, uint64_t chunks_per_stripe) {
  bitslice_recon_pair_body<C, true, P, PF, DBG>(a, chunks_per_stripe);
}

template <class C, int P, bool PF = false, int DBG = 0>
__global__ __launch_bounds__(128 * P, 3) void bitslice_recon_desc_pair_kernel(
    const BsReconArgs* descs, uint64_t chunks_per_stripe, uint64_t n_stripes) {
  bitslice_recon_desc_pair_body<C, true, P, PF, DBG>(descs, chunks_per_stripe, n_stripes);
}

// ------------------------------------------------- batched reconstruct planner
// One lane per stripe of rse_reconstruct_batch: the syndrome plan of
// rse_codec.cpp bitslice_reconstruct on the device.  The valid/invalid
// partition of core.rs:801-841 gives S (missing data), R (the first |S|
// present parity rows -- the parity rows of the reference's `valid` set) and
// M (missing parity, unless data_only); A = P[R][S] is inverted by
// Gauss-Jordan (the unique inverse: any k rows of the systematic MDS matrix
// are independent, so A is invertible) and the stripe's BsReconArgs written.
struct GfDev {
  const uint8_t* lg;
  const uint8_t* ex;
  int field;
  __device__ uint32_t m8(uint32_t a, uint32_t b) const {
    return (a && b) ? ex[lg[a] + lg[b]] : 0u;
  }
  __device__ uint32_t mul(uint32_t a, uint32_t b) const {  // galois_16.rs:146-162
    if (field == 8) return m8(a, b);
    const uint32_t a1 = a >> 8, a0 = a & 0xFFu, b1 = b >> 8, b0 = b & 0xFFu;
    const uint32_t hh = m8(a1, b1);
    const uint32_t x = m8(a1, b0) ^ m8(a0, b1) ^ m8(2u, hh);
    const uint32_t c = m8(a0, b0) ^ m8(128u, hh);
    return (x << 8) | c;
  }
  __device__ uint32_t inv(uint32_t a) const {  // a != 0
    if (field == 8) return ex[255 - lg[a]];
    // through the norm N = a0^2 + 2 a0 a1 + 128 a1^2 in GF(2^8), as
    // rse_kernels.hip PlanF16: (a1 x + a0)^-1 = (a1 x + a0 + 2 a1) / N (the
    // unique inverse; 8 subfield products instead of a^(2^16-2)'s 30)
    const uint32_t a1 = a >> 8, a0 = a & 0xFFu;
    const uint32_t n = m8(a0, a0) ^ m8(2u, m8(a0, a1)) ^ m8(128u, m8(a1, a1));
    const uint32_t ni = ex[255 - lg[n]];  // n != 0 for a != 0
    return (m8(a1, ni) << 8) | m8(a0 ^ m8(2u, a1), ni);
  }
};

constexpr int kPlanBlock = 64;
constexpr uint32_t kPlanLanes = 8;  // lanes that plan one stripe together
constexpr uint32_t kPlanStripes = kPlanBlock / kPlanLanes;  // stripes per workgroup

// The i-th set bit of m (i < popcount(m)).
__device__ __forceinline__ uint32_t nth_bit(uint32_t m, uint32_t i) {
  for (; i; --i) m &= m - 1u;
  return (uint32_t)__builtin_ctz(m);
}

// kPlanLanes lanes per stripe (a group), kPlanStripes stripes per 64-lane
// workgroup.  Every lane of a group derives the stripe's index sets from its
// flags (bit masks: S missing data, R syndrome rows, M missing parity); the
// group then shares the work: the columns of the [A | I] Gauss-Jordan
// (A = P[R][S], in LDS, one e_cap x 2 e_cap block per stripe), the outputs'
// Horner masks, and the descriptor's pointer arrays.  Lanes of a group are
// lanes of one wave, so LDS reads and writes of the group happen in program
// order: a row's factor is read by every lane before the lane owning that
// column clears it.  Round 3's planner (one lane per stripe, its workspace in
// scratch memory) took 223-236 us for 65536 stripes, the first round-4 one
// (one lane per stripe, LDS) 86-93 us.  Only the fields the Horner syndrome
// kernels read are written (data / par / out pointers, out_sigma, the masks,
// n_out, hm); the GF(2^8) log / exp tables come from `tabs` (host-built).
// Orders the group's LDS accesses explicitly between the Gauss-Jordan phases
// (fill, swap, scale, each row's elimination): the lanes of a group read
// columns other lanes write, so the order must not rest on the compiler
// keeping runtime-indexed LDS accesses in program order.
__device__ __forceinline__ void group_lds_order() {
  __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
  __builtin_amdgcn_wave_barrier();
}

__global__ __launch_bounds__(kPlanBlock) void bs_recon_plan_kernel(
    int field, const uint16_t* __restrict__ rows, const uint8_t* __restrict__ tabs,
    const uint8_t* __restrict__ present, uint32_t k, uint32_t p, uint32_t data_only, uint8_t* base,
    uint64_t shard_bytes, uint32_t n_stripes, uint32_t e_cap, BsReconArgs* descs) {
  __shared__ uint32_t tl[(256 + 512) / 4];
  extern __shared__ uint16_t gj[];
  for (uint32_t i = threadIdx.x; i < (256 + 512) / 4; i += kPlanBlock)
    tl[i] = reinterpret_cast<const uint32_t*>(tabs)[i];
  __syncthreads();
  const uint32_t grp = threadIdx.x / kPlanLanes, gl = threadIdx.x % kPlanLanes;
  const uint32_t s = blockIdx.x * kPlanStripes + grp;
  if (s >= n_stripes) return;
  const uint8_t* lg = reinterpret_cast<const uint8_t*>(tl);
  const GfDev gf{lg, lg + 256, field};
  const uint32_t total = k + p, E2 = 2 * e_cap;
  uint16_t* gm = gj + grp * e_cap * E2;
  auto G = [&](uint32_t t, uint32_t x) -> uint16_t& { return gm[t * E2 + x]; };
  const uint8_t* pr = present + (uint64_t)s * total;
  uint8_t* sb = base + (uint64_t)s * total * shard_bytes;
  BsReconArgs& d = descs[s];
  uint32_t pmask = 0, smask = 0, rmask = 0, mmask = 0, nr = 0;
  for (uint32_t j = 0; j < k; ++j) {
    if (pr[j]) pmask |= 1u << j;
    else smask |= 1u << j;
  }
  for (uint32_t j = gl; j < k; j += kPlanLanes)
    d.data[j] = ((pmask >> j) & 1u) ? sb + (uint64_t)j * shard_bytes : nullptr;
  const uint32_t ne = (uint32_t)__builtin_popcount(smask);
  for (uint32_t r = 0; r < p; ++r) {
    if (pr[k + r]) {
      if (nr < ne) {
        rmask |= 1u << r;
        ++nr;
      }
    } else if (!data_only) {
      mmask |= 1u << r;
    }
  }
  const uint32_t nm = (uint32_t)__builtin_popcount(mmask), n_out = ne + nm;
  const bool ok = nr == ne && ne <= e_cap && n_out > 0 && n_out <= (uint32_t)kMaxOut;
  if (gl == 0) {
    d.stripe_stride = 0;
    d.n_stripes = 1;
    d.present = pmask;
    d.sigma = d.synd = 0;
    d.n_out = 0;  // nothing to do unless completed below
  }
  if (!ok) return;
  // [A | I], A = P[R][S]: the group fills it element by element
  for (uint32_t i = gl; i < ne * 2 * ne; i += kPlanLanes) {
    const uint32_t t = i / (2 * ne), x = i % (2 * ne);
    G(t, x) = x < ne ? rows[nth_bit(rmask, t) * k + nth_bit(smask, x)] : (x - ne == t ? 1 : 0);
  }
  group_lds_order();
  // Gauss-Jordan: lane gl owns columns x = gl, gl + kPlanLanes, ... of row
  // operations; the pivot row is found by every lane (same reads, same answer)
  for (uint32_t col = 0; col < ne; ++col) {
    uint32_t piv = col;
    while (piv < ne && G(piv, col) == 0) ++piv;
    if (piv == ne) return;  // singular: impossible for this code; stripe left at n_out = 0
    if (piv != col) {
      for (uint32_t x = gl; x < 2 * ne; x += kPlanLanes) {
        const uint16_t t0 = G(col, x);
        G(col, x) = G(piv, x);
        G(piv, x) = t0;
      }
      group_lds_order();
    }
    const uint32_t sc = gf.inv(G(col, col));
    group_lds_order();  // every lane has the pivot before its owner scales it
    for (uint32_t x = col + gl; x < 2 * ne; x += kPlanLanes) G(col, x) = (uint16_t)gf.mul(sc, G(col, x));
    group_lds_order();
    for (uint32_t r = 0; r < ne; ++r) {
      const uint32_t f = G(r, col);  // read by every lane before any lane writes row r
      group_lds_order();
      if (r == col || !f) continue;
      for (uint32_t x = col + gl; x < 2 * ne; x += kPlanLanes)
        G(r, x) ^= (uint16_t)gf.mul(f, G(col, x));
    }
    group_lds_order();
  }
  // outputs, lane gl the outputs o = gl, gl + kPlanLanes, ...: missing data
  // S_u = sum_t Ainv[u][t] s_t; missing parity r = sigma_r ^ sum_t (P[r][S]
  // Ainv)[t] s_t.  Weight (o, t) sets the Horner mask bits of syndrome row R_t
  // (rse_kernels.hpp set_horner_masks).
  const int nb = field == 8 ? 8 : 16;
  for (uint32_t o = gl; o < n_out; o += kPlanLanes) {
    const bool dat = o < ne;
    const uint32_t r = dat ? 0u : nth_bit(mmask, o - ne);
    d.out[o] = sb + (uint64_t)(dat ? nth_bit(smask, o) : k + r) * shard_bytes;
    d.out_sigma[o] = dat ? -1 : (int32_t)r;
    uint32_t hm[4] = {0u, 0u, 0u, 0u};
    for (uint32_t t = 0, rr = rmask; t < ne; ++t, rr &= rr - 1u) {
      uint32_t v = 0;
      if (dat) {
        v = G(o, ne + t);
      } else {
        for (uint32_t u = 0, ss = smask; u < ne; ++u, ss &= ss - 1u)
          v ^= gf.mul(rows[r * k + (uint32_t)__builtin_ctz(ss)], G(u, ne + t));
      }
      const uint32_t co = horner_coords(field, v), rt = (uint32_t)__builtin_ctz(rr);
      for (int j = 0; j < nb; ++j)
        if ((co >> (nb - 1 - j)) & 1u) hm[j >> 2] |= 1u << (8 * (j & 3) + rt);
    }
    for (int q = 0; q < 4; ++q) d.hm[o][q] = hm[q];
  }
  for (uint32_t t = gl; t < ne; t += kPlanLanes) {
    const uint32_t r = nth_bit(rmask, t);
    d.par[r] = sb + (uint64_t)(k + r) * shard_bytes;
  }
  if (gl == 0) {
    d.synd = rmask;
    d.sigma = rmask | mmask;
    d.n_out = n_out;
  }
}

using BsRecFn = void (*)(const BsReconArgs, uint64_t);
using BsDescFn = void (*)(const BsReconArgs*, uint64_t, uint64_t);
using BsDesc4Fn = void (*)(const BsReconArgs*, uint64_t, uint64_t, uint64_t);
using BsRec4Fn = void (*)(const BsReconArgs, uint64_t, uint64_t);

using BsFn = void (*)(const CodeArgs, uint64_t);
struct BsShape {
  int field;
  uint32_t k, p;
  const uint16_t* m;  // P x K parity rows compiled into the kernel
  BsFn fn[10][2];     // [variant][nt]: 0 plain, 1 +sched barrier, 2 +cross-chunk
                      // prefetch, 3/4 LDS-DMA input ring of 3/2 slots, 5/6 two/three
                      // inputs in flight in VGPRs, 7 = 1 in XCD-aware order, 8 = 1 with
                      // write-through (sc1) stores ([8][0] sc1, [8][1] sc1 nt), 9 = 1
                      // without shared subexpressions (GF(2^16); = 1 for GF(2^8))
  BsFn w4;            // 4 KiB chunks, one per wave (variant 1's scheme, nt)
  BsFn sub[2];        // the same over 1 / 2 KiB shards, 4 / 2 stripes per chunk (SUB)
  BsFn chk;           // the default variant for the check modes (verify): the
                      // stored parity loaded before un-slicing (store_outputs CE)
  BsRecFn rec[4][4];  // [RSE_OPT_RECON_MIX: kReconMix*][sigma rows NS = 1, 2, 4, 8]
                      // (nullptr above p); non-temporal
  BsDescFn rec_desc[4];  // the same over per-stripe argument blocks (reconstruct_batch)
  BsDesc4Fn rec_desc4[4];      // the same over 4 KiB chunks, one per wave (Horner)
  BsRec4Fn rec4[4];            // rec's Horner mode over 4 KiB chunks, one per wave
  BsRecFn rec_deep[2][4];      // Horner mixing, [depth 2 / 3 inputs in flight][NS]
  BsDescFn rec_desc_deep[2][4];
  BsRecFn rec_pair[7];         // NS = 8 on wave pairs (nullptr below 8 rows), by pair_slot:
  BsDescFn rec_desc_pair[7];   // [0] one pair per workgroup, two own inputs in flight per
                               // wave, [1] two pairs, [2] one pair with the next unit
                               // prefetched, [3] / [4] no Horner steps / no data networks
                               // (timing splits, wrong bytes), [5] compact mixing, [6] [0]
                               // with one input in flight (round 3's kernel)
};

template <class C, int NS, int MIX>
constexpr BsRecFn rec_fn() {
  if constexpr (NS <= C::p) return bitslice_recon_kernel<C, true, NS, MIX>;
  else return nullptr;
}
template <class C, int NS>
constexpr BsDescFn rec_desc_fn() {
  if constexpr (NS <= C::p) return bitslice_recon_desc_kernel<C, true, NS>;
  else return nullptr;
}
template <class C, int NS>
constexpr BsDesc4Fn rec_desc4_fn() {
  if constexpr (NS <= C::p) return bitslice_recon_desc_w4_kernel<C, NS>;
  else return nullptr;
}
template <class C, int NS>
constexpr BsRec4Fn rec4_fn() {
  if constexpr (NS <= C::p) return bitslice_recon_w4_kernel<C, NS>;
  else return nullptr;
}
template <class C, int NS, int D>
constexpr BsRecFn rec_deep_fn() {
  if constexpr (NS <= C::p) return bitslice_recon_deep_kernel<C, NS, D>;
  else return nullptr;
}
template <class C, int P, bool PF = false, int DBG = 0>
constexpr BsRecFn rec_pair_fn() {
  if constexpr (C::p >= 8) return bitslice_recon_pair_kernel<C, P, PF, DBG>;
  else return nullptr;
}
template <class C, int P, bool PF = false, int DBG = 0>
constexpr BsDescFn rec_desc_pair_fn() {
  if constexpr (C::p >= 8) return bitslice_recon_desc_pair_kernel<C, P, PF, DBG>;
  else return nullptr;
}
template <class C, int NS, int D>
constexpr BsDescFn rec_desc_deep_fn() {
  if constexpr (NS <= C::p) return bitslice_recon_desc_deep_kernel<C, NS, D>;
  else return nullptr;
}
// The timing splits (pair_slot 3 / 4: no Horner steps / no data networks) write
// wrong bytes by design; they exist only in tools/tune.py's own build
// (-DRSE_TUNE_SPLITS).  The release library has nullptr there, and
// rse_set_option refuses RSE_OPT_RECON_PAIRS 4 / 5 (rse_kernels.hip).
#ifdef RSE_TUNE_SPLITS
#define RSE_SPLIT_FN(...) __VA_ARGS__
#else
#define RSE_SPLIT_FN(...) nullptr
#endif
#define BS(C, CP, FIELD)                                                          \
  {FIELD, C::k, C::p, &C::rows[0][0],                                             \
   {{bitslice_kernel<C, false, false, false>, bitslice_kernel<C, true, false, false>}, \
    {nullptr, bitslice_kernel<C, true, true, false>},                              \
    {nullptr, bitslice_kernel<C, true, true, true>},                               \
    {nullptr, bitslice_dma_kernel<C, 3>},                                          \
    {nullptr, bitslice_dma_kernel<C, 2>},                                          \
    {nullptr, bitslice_deep_kernel<C, 2>},                                         \
    {nullptr, bitslice_deep_kernel<C, 3>},                                         \
    {nullptr, bitslice_kernel<C, true, true, false, true>},                        \
    {bitslice_kernel<C, false, true, false, false, true>,                          \
     bitslice_kernel<C, true, true, false, false, true>},                          \
    {nullptr, bitslice_kernel<CP, true, true, false>}},                            \
   bitslice_kernel<C, true, true, false, false, false, true>,                      \
   {bitslice_kernel<C, true, true, false, false, false, true, false, 1024u>,       \
    bitslice_kernel<C, true, true, false, false, false, true, false, 2048u>},      \
   bitslice_kernel<C, true, C::NP == 8, false, false, false, false, true>,         \
   {{rec_fn<C, 1, 0>(), rec_fn<C, 2, 0>(), rec_fn<C, 4, 0>(), rec_fn<C, 8, 0>()},  \
    {rec_fn<C, 1, 1>(), rec_fn<C, 2, 1>(), rec_fn<C, 4, 1>(), rec_fn<C, 8, 1>()},  \
    {rec_fn<C, 1, 2>(), rec_fn<C, 2, 2>(), rec_fn<C, 4, 2>(), rec_fn<C, 8, 2>()},  \
    {rec_fn<C, 1, 3>(), rec_fn<C, 2, 3>(), rec_fn<C, 4, 3>(), rec_fn<C, 8, 3>()}}, \
   {rec_desc_fn<C, 1>(), rec_desc_fn<C, 2>(), rec_desc_fn<C, 4>(), rec_desc_fn<C, 8>()},   \
   {rec_desc4_fn<C, 1>(), rec_desc4_fn<C, 2>(), rec_desc4_fn<C, 4>(), rec_desc4_fn<C, 8>()}, \
   {rec4_fn<C, 1>(), rec4_fn<C, 2>(), rec4_fn<C, 4>(), rec4_fn<C, 8>()},                 \
   {{rec_deep_fn<C, 1, 2>(), rec_deep_fn<C, 2, 2>(), rec_deep_fn<C, 4, 2>(),           \
     rec_deep_fn<C, 8, 2>()},                                                          \
    {rec_deep_fn<C, 1, 3>(), rec_deep_fn<C, 2, 3>(), rec_deep_fn<C, 4, 3>(),           \
     rec_deep_fn<C, 8, 3>()}},                                                         \
   {{rec_desc_deep_fn<C, 1, 2>(), rec_desc_deep_fn<C, 2, 2>(), rec_desc_deep_fn<C, 4, 2>(), \
     rec_desc_deep_fn<C, 8, 2>()},                                                     \
    {rec_desc_deep_fn<C, 1, 3>(), rec_desc_deep_fn<C, 2, 3>(), rec_desc_deep_fn<C, 4, 3>(), \
     rec_desc_deep_fn<C, 8, 3>()}},                                                    \
   {rec_pair_fn<C, 1, false, 4>(), rec_pair_fn<C, 2>(), rec_pair_fn<C, 1, true>(),  \
    RSE_SPLIT_FN(rec_pair_fn<C, 1, false, 1>()), RSE_SPLIT_FN(rec_pair_fn<C, 1, false, 2>()), \
    rec_pair_fn<C, 1, false, 3>(), rec_pair_fn<C, 1>()},                            \
   {rec_desc_pair_fn<C, 1, false, 4>(), rec_desc_pair_fn<C, 2>(),                   \
    rec_desc_pair_fn<C, 1, true>(), nullptr, nullptr,                               \
    rec_desc_pair_fn<C, 1, false, 3>(), rec_desc_pair_fn<C, 1>()}}
static const BsShape kBsShapes[] = {
    BS(Bs8_10_4, Bs8_10_4, 8),        // BASELINE headline: galois_8 10+4
    BS(Bs8_10_2, Bs8_10_2, 8),        // benches/bandwidth.rs 10+2
    BS(Bs8_20_8, Bs8_20_8Plain, 8),   // BASELINE configs[4]: galois_16 20+8 (subfield)
    BS(Bs16_20_8, Bs16_20_8Plain, 16),  // the same in GF(2^16) (RSE_OPT_SUBFIELD 0)
};
#undef BS
#undef RSE_SPLIT_FN

}  // namespace

thread_local bool t_done_armed = false;

// Compute units of the current device (cached per device).
uint32_t device_cus() {
  static std::atomic<uint32_t> cus[64];  // zero-initialised (static storage)
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return 256;
  uint32_t c = cus[dev].load(std::memory_order_relaxed);
  if (!c) {
    int n = 0;
    c = hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess && n > 0
            ? (uint32_t)n
            : 256u;
    cus[dev].store(c, std::memory_order_relaxed);
  }
  return c;
}

hipError_t launch_bitslice(int field, const CodeArgs& a, bool nt, int64_t grid,
                           hipStream_t stream, bool* handled, uint64_t* done) {
  *handled = false;
  *done = 0;
  constexpr uint64_t kV16 = kBsChunk / 16, kV4 = 4096 / 16;  // vectors per chunk
  // shards of exactly 1 or 2 KiB: 4 or 2 stripes per 4 KiB chunk (SUB)
  const bool subm = (a.len == 1024u || a.len == 2048u) && a.n_vec * 16u == a.len &&
                    get_option(33) != 0;
  // accumulate: store mode on a wide codec's block kernels (kJitBlock) only
  if ((a.n_vec < kV4 && !subm) || (a.accumulate && a.mode != kStore)) return hipSuccess;
  // the kernels for these coefficients: compiled in, or specialised at run time
  BsFn f16 = nullptr, f4 = nullptr, fs = nullptr;
  hipFunction_t j16 = nullptr, j4 = nullptr, js = nullptr;
  bool compiled = false;
  int vopt_used = -1;
  bool chk = false;  // f16 is the compiled check kernel (it reads a.done)
  for (const BsShape& sh : kBsShapes) {
    if (a.accumulate) break;
    if (sh.field != field || sh.k != a.n_in || sh.p != a.n_out) continue;
    bool same = true;  // other rows of this shape (a decode pattern) may be specialised
    for (uint32_t o = 0; o < sh.p && same; ++o)
      for (uint32_t i = 0; i < sh.k && same; ++i) same = a.coef[o][i] == sh.m[o * sh.k + i];
    if (!same) break;
    // RSE_OPT_KERNEL_VARIANT picks a bit-sliced variant too (-1: default)
    const int64_t vopt = get_option(4);
    int v = (vopt >= 0 && vopt < 10) ? (int)vopt
                                     : (field == 16 ? kBsDefaultVariant16 : kBsDefaultVariant8);
    f16 = sh.fn[v][nt ? 1 : 0];
    if (!f16) f16 = sh.fn[v][1];
    if (a.mode != kStore && vopt < 0 && nt) {
      f16 = sh.chk;
      chk = true;
    }
    vopt_used = v;
    f4 = sh.w4;
    fs = sh.sub[a.len == 2048u];
    compiled = true;
    break;
  }
  if (!compiled) {  // run-time specialised (rse_jit.cpp): the default scheme, nt
    JitFns jf;
    hipError_t e = hipSuccess;
    if (!jit_find(field, a.n_in, a.n_out, &a.coef[0][0], kMaxIn, 0, &jf, &e, a.accumulate != 0))
      return e;
    j16 = a.accumulate ? jf.enc_acc : jf.enc;
    j4 = a.accumulate ? jf.enc4_acc : jf.enc4;
    js = a.accumulate ? nullptr : jf.sub[a.len == 2048u];
    if (!j16) return hipSuccess;
    if (a.mode != kStore && !a.accumulate && nt && jf.chk && get_option(4) < 0) {
      j16 = jf.chk;  // the check kernel, which can signal the call's completion
      chk = true;
    }
  }
  // tools/tune.py sweeps: GF(2^8) 4096 workgroups (16384 at <= 2 outputs: 10+2
  // x 1 MiB +0.8-1.1 % in two processes, profiles/r03/s12, s13), GF(2^16)
  // (2 waves/SIMD) 8192
  const uint64_t g0 = grid > 0 ? (uint64_t)grid
                               : (field == 16 ? 8192u : a.n_out <= 2 ? 16384u : 4096u);
  // A launch of one to two rounds of the resident workgroups (one 10+4 x 16
  // MiB stripe: 1024 chunks against 768) runs as one round of resident
  // workgroups, grid-striding over the rest, instead of a full round plus a
  // late third of one.  Per call through the C ABI (tools/capi_latency.cpp,
  // two boxes, profiles/r03/s5/, s6/): verify 52.3-52.9 -> 48.5-49.5 us,
  // encode 43.6-43.8 -> 40.9-41.2 us (half the chunks per workgroup, 512,
  // was 48.6-51.8 for verify).
  const uint64_t resident = (uint64_t)device_cus() * (a.n_out > 4 ? 2u : 3u);
  auto clamp = [&](uint64_t steps) {
    uint64_t gx = g0 < steps ? g0 : steps;
    if (grid <= 0 && steps > resident && steps <= 2 * resident) gx = resident;
    return gx > 0x7fffffffu ? (uint64_t)0x7fffffffu : gx;
  };
  auto launch = [&](BsFn f, hipFunction_t j, const CodeArgs& args, uint64_t cps, uint64_t steps) {
    const uint64_t gx = clamp(steps);
    if (f) {
      hipLaunchKernelGGL(f, dim3((uint32_t)gx), dim3(kBsBlock), 0, stream, args, cps);
      return hipGetLastError();
    }
    uint64_t cps_arg = cps;
    void* argv[] = {const_cast<CodeArgs*>(&args), &cps_arg};
    return hipModuleLaunchKernel(j, (uint32_t)gx, 1, 1, kBsBlock, 1, 1, 0, stream, argv, nullptr);
  };
  if (subm) {
    // one launch codes every byte: 4096 / len stripes per chunk, a chunk per
    // wave; never the whole call's completion signal (not a check kernel)
    if (!fs && !js) return hipSuccess;
    const uint64_t spc = 4096u / a.len, chunks = (a.n_stripes + spc - 1) / spc;
    if (compiled)
      note_kernel("bitslice gf%d %u+%u v%d nt1 sub%u", field, a.n_in, a.n_out, vopt_used,
                  a.len / 1024u);
    else
      note_kernel("bitslice-jit gf%d %u+%u sub%u", field, a.n_in, a.n_out, a.len / 1024u);
    CodeArgs c = a;
    c.done = c.done_count = nullptr;
    const hipError_t e = launch(fs, js, c, 0, (chunks + 3) / 4);
    if (e != hipSuccess) return e;
    *done = a.len;
    *handled = true;
    return hipSuccess;
  }
  // whole 16 KiB chunks, then whole 4 KiB chunks of the rest (one per wave)
  const uint64_t cps16 = a.n_vec / kV16, cps4 = (a.n_vec - cps16 * kV16) / kV4;
  if (compiled)
    note_kernel("bitslice gf%d %u+%u v%d nt%d%s", field, a.n_in, a.n_out,
                (int)(vopt_used), nt ? 1 : 0, cps16 ? "" : " w4");
  else
    note_kernel("bitslice-jit gf%d %u+%u%s%s", field, a.n_in, a.n_out, a.accumulate ? " acc" : "",
                cps16 ? "" : " w4");
  if (cps16) {
    // a verify's completion word (run_check): armed only when this launch is
    // the whole job, else cleared so that the kernel does not signal early.
    // Only the plain check (kCheck) arms it: its stores are the verdict words
    // alone, which the host reads itself.  verify_with_buffer (kCheckStore)
    // writes parity into the caller's buffer, which other streams, devices or
    // mapped-memory readers may read once the call returns, so it waits for
    // the kernel's end-of-kernel release instead.
    const bool arm = a.done && chk && a.mode == kCheck && a.n_vec == cps16 * kV16 &&
                     a.len == a.n_vec * 16u;
    hipError_t e;
    if (a.done && !arm) {
      CodeArgs c = a;
      c.done = c.done_count = nullptr;
      e = launch(f16, j16, c, cps16, cps16 * a.n_stripes);
    } else {
      e = launch(f16, j16, a, cps16, cps16 * a.n_stripes);
    }
    if (e != hipSuccess) return e;
    t_done_armed = arm;
    *done = cps16 * kBsChunk;
  }
  if (cps4 && (f4 || j4)) {
    CodeArgs b = a;
    for (uint32_t i = 0; i < b.n_in; ++i) b.in[i] += *done;
    for (uint32_t o = 0; o < b.n_out; ++o) {
      if (b.out[o]) b.out[o] += *done;
      if (b.cmp[o]) b.cmp[o] += *done;
    }
    b.n_vec -= *done / 16;
    b.len -= *done;
    const hipError_t e = launch(f4, j4, b, cps4, (cps4 * a.n_stripes + 3) / 4);
    if (e != hipSuccess) return e;
    *done += cps4 * 4096;
  }
  *handled = *done > 0;
  return hipSuccess;
}

// RSE_OPT_RECON_PAIRS: 0 off, 1 one pair per workgroup (its barriers sync
// the pair only: 4.26 TB/s at 8 lost against 4.18 for two pairs per
// workgroup, profiles/r03/s3/r8.log), 2 two pairs; returns pairs per
// workgroup (0: off).  3-6: one pair per workgroup, A/B variants (pair_slot).
// 8 (the default): by field -- GF(2^8) two pairs per workgroup (20+8 x 4 MiB
// at 8 lost, 256 stripes: 4.96 TB/s against 4.73 for the depth-2 pair and
// 4.79 for round 3's, profiles/r04/s8/r8ab.log), GF(2^16) the depth-2 pair.
int64_t pair_option(int field) {
  const int64_t o = get_option(28);
  return o == 8 ? (field == 8 ? 2 : 1) : o;
}
int pair_groups(int field) {
  const int64_t o = pair_option(field);
  return o == 0 ? 0 : o == 2 ? 2 : 1;
}
// RSE_OPT_RECON_DEPTH (inputs in flight per lane in the syndrome kernels).  The
// deep kernels mix by Horner's rule, so a depth above 1 applies only when the
// mixing mode is a Horner mode (RSE_OPT_RECON_MIX >= kReconMixHorner), on the
// shared-pattern and the per-stripe (batch) paths alike; it then selects the
// deep Horner kernel in place of the mode's own.
int recon_depth(int mix) {
  return mix >= kReconMixHorner ? (int)get_option(27) : 1;
}

// index into BsShape::rec_pair / rec_desc_pair: option 28 = 3 the prefetching
// variant, 4 / 5 the timing splits (no Horner steps / no data networks; wrong
// bytes, tools/tune.py only), 6 the compact mixing, 7 one input in flight.
// (Two own inputs in flight per wave, the default since round 4: GF(2^16) 20+8
// x 4 MiB at 8 lost 4.37 against 4.25 TB/s at 128 stripes, 4.45 against 4.38
// at 256, reconstruct_batch 8 erasures 2.77 against 2.73; profiles/r04/s4/.)
int pair_slot(int field) {
  const int64_t o = pair_option(field);
  return o >= 3 && o <= 7 ? (int)o - 1 : pair_groups(field) - 1;
}

// The 4 KiB syndrome chunks against the table kernels over the same bytes
// (tools/tune.py --op reconstruct --patterns 0 --bitslice 1,0, 16384 stripes,
// profiles/r04/s14/): GF(2^8) 10+4 x 8 KiB, 2 lost, 5.24 against 5.57 TB/s;
// 6+3 x 12 KiB, 3 lost, 5.96 both; GF(2^16) 20+8 (subfield) x 4 KiB, 4 lost,
// 5.24 against 4.68.  The table kernels' work grows with the coefficients
// (k x outputs); the syndrome kernels' much less: used from
// RSE_OPT_RECON_W4_MIN coefficients (default 64), and always for GF(2^16)
// proper, whose table kernels are 2 x 2 blocks of GF(2^8) ones.
bool recon4_pays(int field, uint32_t k, uint32_t n_out) {
  return field == 16 || (int64_t)k * n_out >= get_option(37);
}

hipError_t launch_bitslice_recon(int field, uint32_t k, uint32_t p, const uint16_t* parity_rows,
                                 const BsReconArgs& a, uint64_t n_vec, hipStream_t stream,
                                 uint64_t* done) {
  *done = 0;
  if (!get_option(5) || n_vec < 4096u / 16 || a.n_out == 0 || a.n_out > (uint32_t)kMaxOut ||
      (a.present == 0 && a.synd == 0))
    return hipSuccess;
  // whole 16 KiB chunks, then whole 4 KiB chunks of the rest (one per wave)
  const uint64_t cps = n_vec / (kBsChunk / 16);
  const uint64_t cps4 = (n_vec * 16u - cps * kBsChunk) / 4096u, base4 = cps * kBsChunk;
  const uint64_t total = cps * a.n_stripes;
  const int64_t grid = get_option(2);
  // tools/tune.py --op reconstruct --patterns 0 sweeps: GF(2^8) 10+4 x 16 MiB at
  // 32768 workgroups against 8192, 2 lost 5.83 against 5.72 TB/s, 4 lost 5.53
  // against 5.27 (profiles/r03/s17/); GF(2^16) 8192
  uint64_t gx = grid > 0 ? (uint64_t)grid : (field == 8 ? 32768u : 8192u);
  if (gx > total) gx = total;
  if (gx > 0x7fffffffu) gx = 0x7fffffffu;
  auto grid4 = [&]() {  // the 4 KiB chunks: four per workgroup step
    uint64_t g4 = grid > 0 ? (uint64_t)grid : 8192u;
    const uint64_t steps = (cps4 * a.n_stripes + 3) / 4;
    if (g4 > steps) g4 = steps;
    return g4 > 0x7fffffffu ? (uint64_t)0x7fffffffu : g4;
  };
  // rows needed: sigma (R and missing parity); NS = smallest compiled cover
  const uint32_t need = 32u - (uint32_t)__builtin_clz(a.sigma | 1u);
  for (const BsShape& sh : kBsShapes) {
    if (sh.field != field || sh.k != k || sh.p != p) continue;
    for (uint32_t i = 0; i < k * p; ++i)
      if (parity_rows[i] != sh.m[i]) return hipSuccess;
    int slot = -1;
    for (int q = 0; q < 4 && slot < 0; ++q)
      if (sh.rec[0][q] && (1u << q) >= need) slot = q;
    if (slot < 0) return hipSuccess;
    const int mix = (int)get_option(17);
    const int depth = recon_depth(mix);
    static const char* const kMixName[4] = {"mix-tables", "mix-chain", "mix-horner", "mix-horner4"};
    if (cps) {
      // 8 sigma rows: wave pairs (RSE_OPT_RECON_PAIRS; Horner mixing), 8 KiB units
      const int np = pair_groups(field);
      if (slot == 3 && np && sh.rec_pair[pair_slot(field)] && mix >= kReconMixHorner &&
          depth == 1) {
        note_kernel("bitslice-recon gf%d %u+%u ns8 pairs%d s%d", field, k, p, np,
                    pair_slot(field));
        // (tools/tune.py, two pairs per workgroup: 32768 workgroups 4.24 TB/s, 8192
        // 4.16, 4096 4.10 at 8 lost; one pair: twice the workgroups)
        uint64_t gp = grid > 0 ? (uint64_t)grid : 32768u * (2 / np);
        const uint64_t units = total * (4 / np);
        if (gp > units) gp = units;
        if (gp > 0x7fffffffu) gp = 0x7fffffffu;
        hipLaunchKernelGGL(sh.rec_pair[pair_slot(field)], dim3((uint32_t)gp), dim3(128 * np), 0,
                           stream, a, cps);
      } else {
        note_kernel("bitslice-recon gf%d %u+%u ns%d %s d%d", field, k, p, 1 << slot,
                    kMixName[mix], depth > 3 ? 3 : depth);
        BsRecFn fn = depth > 1 ? sh.rec_deep[depth > 2 ? 1 : 0][slot] : sh.rec[mix][slot];
        hipLaunchKernelGGL(fn, dim3((uint32_t)gx), dim3(kBsBlock), 0, stream, a, cps);
      }
      const hipError_t e = hipGetLastError();
      if (e != hipSuccess) return e;
      count_bitslice_launch();
      *done = base4;
    }
    if (cps4 && sh.rec4[slot] && recon4_pays(field, k, a.n_out)) {
      if (!cps) note_kernel("bitslice-recon gf%d %u+%u ns%d w4", field, k, p, 1 << slot);
      hipLaunchKernelGGL(sh.rec4[slot], dim3((uint32_t)grid4()), dim3(kBsBlock), 0, stream, a,
                         cps4, base4);
      const hipError_t e = hipGetLastError();
      if (e != hipSuccess) return e;
      if (!cps) count_bitslice_launch();
      *done = base4 + cps4 * 4096u;
    }
    return hipSuccess;
  }
  JitFns jf;
  hipError_t e = hipSuccess;
  if (!jit_find(field, k, p, parity_rows, k, 1, &jf, &e)) return e;
  int slot = -1;
  for (int q = 0; q < jf.n_rec && slot < 0; ++q)
    if ((uint32_t)jf.rec_ns[q] >= need) slot = q;
  if (slot < 0) return hipSuccess;
  if (cps) {
    uint64_t cps_arg = cps;
    note_kernel("bitslice-jit-recon gf%d %u+%u ns%d", field, k, p, jf.rec_ns[slot]);
    void* args[] = {const_cast<BsReconArgs*>(&a), &cps_arg};
    e = hipModuleLaunchKernel(jf.rec[slot], (uint32_t)gx, 1, 1, kBsBlock, 1, 1, 0, stream, args,
                              nullptr);
    if (e != hipSuccess) return e;
    count_bitslice_launch();
    *done = base4;
  }
  if (cps4 && jf.rec4[slot] && recon4_pays(field, k, a.n_out)) {
    if (!cps) note_kernel("bitslice-jit-recon gf%d %u+%u ns%d w4", field, k, p, jf.rec_ns[slot]);
    uint64_t c4 = cps4, b4 = base4;
    void* args[] = {const_cast<BsReconArgs*>(&a), &c4, &b4};
    e = hipModuleLaunchKernel(jf.rec4[slot], (uint32_t)grid4(), 1, 1, kBsBlock, 1, 1, 0, stream,
                              args, nullptr);
    if (e != hipSuccess) return e;
    if (!cps) count_bitslice_launch();
    *done = base4 + cps4 * 4096u;
  }
  return hipSuccess;
}

hipError_t launch_bitslice_recon_batch(int field, uint32_t k, uint32_t p,
                                       const uint16_t* parity_rows, const uint16_t* d_rows,
                                       const uint8_t* d_tabs, const uint8_t* d_present,
                                       uint32_t data_only, uint8_t* base, uint64_t shard_bytes,
                                       uint32_t n_stripes, uint32_t need, uint32_t e_cap,
                                       BsReconArgs* d_descs, hipStream_t stream, uint64_t* done) {
  *done = 0;
  if (!get_option(5) || shard_bytes < 4096 || k == 0 || k > (uint32_t)kMaxIn ||
      p > (uint32_t)kMaxOut || need == 0 || n_stripes == 0 || e_cap > (uint32_t)kMaxOut)
    return hipSuccess;  // (e_cap 0: only parity lost -- rebuilt from the sigma rows)
  BsDescFn sfn = nullptr;
  BsDesc4Fn sfn4 = nullptr;
  hipFunction_t jfn = nullptr, jfn4 = nullptr;
  bool compiled = false, pairs = false;
  for (const BsShape& sh : kBsShapes) {
    if (sh.field != field || sh.k != k || sh.p != p) continue;
    compiled = true;
    for (uint32_t i = 0; i < k * p; ++i)
      if (parity_rows[i] != sh.m[i]) return hipSuccess;
    const int depth = recon_depth((int)get_option(17));
    for (int q = 0; q < 4 && !sfn; ++q)
      if (sh.rec_desc[q] && (1u << q) >= need) {
        sfn = depth > 1 ? sh.rec_desc_deep[depth > 2 ? 1 : 0][q] : sh.rec_desc[q];
        sfn4 = sh.rec_desc4[q];
        if (q == 3 && pair_groups(field) && sh.rec_desc_pair[pair_slot(field)] && depth == 1) {
          sfn = sh.rec_desc_pair[pair_slot(field)];  // 8 sigma rows on wave pairs
          pairs = true;
        }
        if (pairs)
          note_kernel("bitslice-recon-batch gf%d %u+%u ns8 pairs%d", field, k, p, pair_groups(field));
        else
          note_kernel("bitslice-recon-batch gf%d %u+%u ns%d d%d", field, k, p, 1 << q,
                      depth > 3 ? 3 : depth < 1 ? 1 : depth);
      }
    if (!sfn) return hipSuccess;
  }
  if (!compiled) {
    JitFns jf;
    hipError_t e = hipSuccess;
    if (!jit_find(field, k, p, parity_rows, k, 1, &jf, &e)) return e;
    for (int q = 0; q < jf.n_rec && !jfn; ++q)
      if ((uint32_t)jf.rec_ns[q] >= need) {
        jfn = jf.rec_desc[q];
        jfn4 = jf.rec_desc4[q];
      }
    if (!jfn) return hipSuccess;
  }
  // the planner's Gauss-Jordan workspace: e_cap x 2 e_cap halfwords per stripe
  const size_t gj_lds = (size_t)e_cap * 2u * e_cap * kPlanStripes * sizeof(uint16_t);
  hipLaunchKernelGGL(bs_recon_plan_kernel, dim3((n_stripes + kPlanStripes - 1) / kPlanStripes),
                     dim3(kPlanBlock), gj_lds, stream, field, d_rows, d_tabs, d_present, k, p,
                     data_only, base, shard_bytes, n_stripes, e_cap, d_descs);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  const int64_t grid = get_option(2);
  auto grid_for = [&](uint64_t steps) {
    uint64_t gx = grid > 0 ? (uint64_t)grid : pairs ? 32768u * (2 / pair_groups(field)) : 8192u;
    if (gx > steps) gx = steps;
    return gx > 0x7fffffffu ? (uint64_t)0x7fffffffu : gx;
  };
  // whole 16 KiB chunks, then whole 4 KiB chunks of the rest (one per wave)
  uint64_t cps = shard_bytes / kBsChunk, ns = n_stripes;
  uint64_t cps4 = (shard_bytes - cps * kBsChunk) / 4096u, base4 = cps * kBsChunk;
  if (cps) {
    const int np = pairs ? pair_groups(field) : 2;
    const uint64_t gx = grid_for(cps * ns * (pairs ? 4 / np : 1));
    if (sfn) {
      hipLaunchKernelGGL(sfn, dim3((uint32_t)gx), dim3(pairs ? 128 * np : kBsBlock), 0, stream,
                         (const BsReconArgs*)d_descs, cps, ns);
      e = hipGetLastError();
    } else {
      const BsReconArgs* dp = d_descs;
      void* args[] = {&dp, &cps, &ns};
      e = hipModuleLaunchKernel(jfn, (uint32_t)gx, 1, 1, kBsBlock, 1, 1, 0, stream, args, nullptr);
    }
    if (e != hipSuccess) return e;
    *done = base4;
    count_bitslice_launch();
  }
  if (cps4 && (sfn4 || jfn4)) {
    const uint64_t gx = grid_for((cps4 * ns + 3) / 4);
    if (sfn4) {
      hipLaunchKernelGGL(sfn4, dim3((uint32_t)gx), dim3(kBsBlock), 0, stream,
                         (const BsReconArgs*)d_descs, cps4, ns, base4);
      e = hipGetLastError();
    } else {
      const BsReconArgs* dp = d_descs;
      void* args[] = {&dp, &cps4, &ns, &base4};
      e = hipModuleLaunchKernel(jfn4, (uint32_t)gx, 1, 1, kBsBlock, 1, 1, 0, stream, args, nullptr);
    }
    if (e != hipSuccess) return e;
    *done = base4 + cps4 * 4096u;
    if (!cps) count_bitslice_launch();
  }
  return hipSuccess;
}

int bitslice_compiled(int field, uint32_t k, uint32_t p) {
  for (const BsShape& sh : kBsShapes)
    if (sh.field == field && sh.k == k && sh.p == p) return 1;
  return 0;
}

uint64_t bitslice_chunk_bytes() { return kBsChunk; }

}  // namespace rse
