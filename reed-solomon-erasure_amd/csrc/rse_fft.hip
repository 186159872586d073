// rse_fft.hip -- GF(2^8) codecs with k = p = 2^m data and parity shards
// (the reference bench's 16+16, 32+32 and 64+64, benches/bandwidth.rs:88-190)
// coded with an additive FFT instead of k x p coefficient networks.
//
// Why it gives the reference's bytes.  ReedSolomon::new builds the systematic
// matrix M = V . V_top^-1 with V[r][c] = nth(r)^c and nth(r) = r
// (matrix.rs:263-276, core.rs:430-436, galois_8.rs:37-39).  So with P the
// unique polynomial of degree < k with P(i) = data_i for i < k, parity row j is
// P(k + j): M's rows are the evaluations of the interpolating polynomial.  For
// k = 2^m the points {0 .. k-1} are the F2-span U of {1, 2, .. 2^(m-1)} and
// {k .. 2k-1} = k ^ U is a coset of it.  The additive FFT of Lin, Chung and Han
// (novel polynomial basis X_j = prod over set bits i of j of s^_i, with
// s_i(x) = prod over a in span(1..2^(i-1)) of (x - a) and s^_i = s_i / s_i(2^i))
// evaluates a polynomial of degree < 2^m given in that basis on any coset
// beta ^ U in m 2^(m-1) butterflies
//     a ^= s^_i(beta ^ j) . b;   b ^= a
// (level i, block offset j), and its inverse interpolates.  Encode is the
// inverse transform on U (the data values -> P in the novel basis) followed
// by the forward transform on k ^ U (-> the parity values).  Rebuilding every
// data shard from the parity shards is the same map: Q(x) = P(x ^ k) has
// degree < k too and swaps the two cosets (i <-> k ^ i = k + i for i < k), so
// the k x k parity block is its own inverse and one kernel serves encode,
// verify and the rebuild (tests/test_fft_math.py checks the involution on the
// oracle's matrices).  The polynomial is unique, so the bytes are the
// reference's exactly (tests/test_fft_math.py checks the transform against the
// oracle's encode and reconstruct; tests/test_gpu_fft.py the kernels).
//
// Cost.  (k/2) log2 k butterflies per transform, each one constant multiply
// (an 8 x 8 bit matrix: a v_bitop3 XOR network over the bit-sliced planes)
// plus 8 XORs: 64+64 takes 384 multiplies per byte column against 4096 for
// the coefficient networks of the wide modules (rse_bitslice_core.hpp), and
// the zero twiddles of the transform on U (the first block of every level) are
// free.
//
// Kernel.  A workgroup of k/8 waves codes one 2 KiB column of every shard at a
// time (lane l: bytes 16 l and 1024 + 16 l, one 8-plane group, as
// wide_body_half; 1 KiB shards: two stripes per column).  Element e (a shard)
// lives in the registers of one wave as 8 planes:
//   phase A: wave h holds elements 8h .. 8h+7 (its own loads) and runs the
//            inverse transform's levels 0-2 (twiddles per wave);
//   phase B: through LDS, wave w holds the groups of elements with the same
//            low three bits (8 / (k/8) groups of k/8) and runs the levels >= 3
//            of the inverse transform, then of the forward one (twiddles equal
//            for every wave: they depend only on the bits >= 3);
//   phase C: back through LDS, wave h holds elements 8h .. 8h+7 again and runs
//            the forward transform's levels 2-0, then un-slices and stores (or
//            compares) its 8 outputs.
// Every wave writes its phase-B results into the LDS slots it read them from,
// and its phase-A results into the slots it read in phase C, so a column
// needs two workgroup barriers.  The next column's loads are issued before
// phase A.  LDS: k x 2 KiB (64+64: 128 KiB, one workgroup per CU).
#include <hip/hip_runtime.h>

#include <cstring>
#include <mutex>
#include <vector>

#include "rse_bitslice_core.hpp"
#include "rse_field.hpp"
#include "rse_fft.hpp"

namespace rse {
namespace {

// ------------------------------------------------------ field, at compile time
constexpr uint32_t f8_inv(uint32_t a) {
  for (uint32_t x = 1; x < 256; ++x)
    if (hb_mul8(a, x) == 1u) return x;
  return 0;
}
// s_i(x): the subspace polynomial of span(1, 2, .. 2^(i-1)) at x
constexpr uint32_t fft_vanish(int i, uint32_t x) {
  uint32_t r = 1;
  for (uint32_t a = 0; a < (1u << i); ++a) r = hb_mul8(r, x ^ a);
  return r;
}
// s^_i(x) = s_i(x) / s_i(2^i): the butterfly twiddle of level i at shift x
constexpr uint32_t fft_skew(int i, uint32_t x) {
  return hb_mul8(fft_vanish(i, x), f8_inv(fft_vanish(i, 1u << i)));
}
// Row q of the 8 x 8 bit matrix of multiplication by c: bit j set when bit q
// of c . 2^j is (the planes of b that plane q of c . b XORs).
constexpr uint64_t fft_row(uint32_t c, int q) {
  uint64_t m = 0;
  for (int j = 0; j < 8; ++j)
    if ((hb_mul8(c, 1u << j) >> q) & 1u) m |= 1ull << j;
  return m;
}

template <uint32_t C, int... Q>
__device__ __forceinline__ void fft_mul_add(uint32_t (&a)[8], const uint32_t (&b)[8],
                                            int_seq<int, Q...>) {
  ((a[Q] = xacc<fft_row(C, Q)>(a[Q], b)), ...);
}
// forward butterfly: a ^= C b; b ^= a.  Inverse: b ^= a; a ^= C b.
template <uint32_t C, bool INV>
__device__ __forceinline__ void fft_bfly(uint32_t (&a)[8], uint32_t (&b)[8]) {
  if constexpr (INV) {
#pragma unroll
    for (int q = 0; q < 8; ++q) b[q] ^= a[q];
    fft_mul_add<C>(a, b, make_int_seq<8>{});
  } else {
    fft_mul_add<C>(a, b, make_int_seq<8>{});
#pragma unroll
    for (int q = 0; q < 8; ++q) b[q] ^= a[q];
  }
}

// Which element register r of a wave holds, and back, by phase.
//  A / C: wave H holds elements 8H + r.
template <int H>
struct MapAC {
  static constexpr int elem(int r) { return 8 * H + r; }
  static constexpr int reg(int e) { return e - 8 * H; }
};
//  B: the wave's groups of G = K / 8 elements with the same low three bits,
//  register gi * G + t = element g + 8 t.  Only bits >= 3 matter to the
//  levels of phase B, so the first wave's map serves every wave.
template <int K>
struct MapB {
  static constexpr int G = K / 8;
  static constexpr int elem(int r) { return (r / G) + 8 * (r % G); }
  static constexpr int reg(int e) { return (e & 7) * G + (e >> 3); }
};

// One level I of a transform at shift BETA over the 8 registers: every
// register whose element has bit I clear is butterflied with its partner.
template <class M, uint32_t BETA, int I, bool INV, int R = 0>
__device__ __forceinline__ void fft_level(uint32_t (&x)[8][8]) {
  if constexpr (R < 8) {
    constexpr int e = M::elem(R);
    if constexpr (((e >> I) & 1) == 0) {
      constexpr int r2 = M::reg(e + (1 << I));
      constexpr uint32_t c = fft_skew(I, BETA ^ (uint32_t)(e & ~((2 << I) - 1)));
      fft_bfly<c, INV>(x[R], x[r2]);
    }
    fft_level<M, BETA, I, INV, R + 1>(x);
  }
}

// Phase A of wave H: the inverse transform at B0, levels 0-2.
template <int H, uint32_t B0>
__device__ __forceinline__ void fft_phase_a(uint32_t (&x)[8][8]) {
  fft_level<MapAC<H>, B0, 0, true>(x);
  fft_level<MapAC<H>, B0, 1, true>(x);
  fft_level<MapAC<H>, B0, 2, true>(x);
}
// Phase C of wave H: the forward transform at B1, levels 2-0.
template <int H, uint32_t B1>
__device__ __forceinline__ void fft_phase_c(uint32_t (&x)[8][8]) {
  fft_level<MapAC<H>, B1, 2, false>(x);
  fft_level<MapAC<H>, B1, 1, false>(x);
  fft_level<MapAC<H>, B1, 0, false>(x);
}
// Phase B: the inverse transform's levels 3 .. m-1 at B0, then the forward
// transform's levels m-1 .. 3 at B1.
template <int K, uint32_t B0, uint32_t B1, int I>
__device__ __forceinline__ void fft_phase_b_inv(uint32_t (&x)[8][8]) {
  if constexpr ((1 << I) < K) {
    fft_level<MapB<K>, B0, I, true>(x);
    fft_phase_b_inv<K, B0, B1, I + 1>(x);
  }
}
template <int K, uint32_t B1, int I>
__device__ __forceinline__ void fft_phase_b_fwd(uint32_t (&x)[8][8]) {
  if constexpr (I >= 3) {
    fft_level<MapB<K>, B1, I, false>(x);
    fft_phase_b_fwd<K, B1, I - 1>(x);
  }
}
constexpr int fft_log2(int k) { return k <= 1 ? 0 : 1 + fft_log2(k / 2); }

// The wave-dependent phases, dispatched on the (uniform) wave index.
template <int K, uint32_t B0, int H = 0>
__device__ __forceinline__ void fft_a(int w, uint32_t (&x)[8][8]) {
  if constexpr (H < K / 8) {
    if (w == H) fft_phase_a<H, B0>(x);
    else fft_a<K, B0, H + 1>(w, x);
  }
}
template <int K, uint32_t B1, int H = 0>
__device__ __forceinline__ void fft_c(int w, uint32_t (&x)[8][8]) {
  if constexpr (H < K / 8) {
    if (w == H) fft_phase_c<H, B1>(x);
    else fft_c<K, B1, H + 1>(w, x);
  }
}

// LDS: element e's 8 planes, as two quads of planes per lane.
template <int K>
using FftPlanes = uint4[K][2][64];

__device__ __forceinline__ void fft_put(uint4 (&slot)[2][64], const uint32_t (&x)[8], uint32_t lane) {
  slot[0][lane] = make_uint4(x[0], x[1], x[2], x[3]);
  slot[1][lane] = make_uint4(x[4], x[5], x[6], x[7]);
}
__device__ __forceinline__ void fft_get(const uint4 (&slot)[2][64], uint32_t (&x)[8], uint32_t lane) {
  const uint4 a = slot[0][lane], b = slot[1][lane];
  x[0] = a.x;
  x[1] = a.y;
  x[2] = a.z;
  x[3] = a.w;
  x[4] = b.x;
  x[5] = b.y;
  x[6] = b.z;
  x[7] = b.w;
}

// The kernel: K = k = p, B0 / B1 the cosets of the inputs / outputs (0 / K:
// the parity rows, which are also their inverse), SUB 1024 for 1 KiB shards
// (two stripes per 2 KiB column), else 0 (whole 2 KiB columns).
template <int K, uint32_t B0, uint32_t B1, uint32_t SUB>
__global__ __launch_bounds__(K * 8) void fft_kernel(const FftArgs a) {
  static_assert(K == 16 || K == 32 || K == 64, "k = p = 16, 32 or 64");
  __shared__ FftPlanes<K> st;
  constexpr int G = K / 8;         // phase B: elements per group
  constexpr int GPW = 8 / G;       // ... groups per wave
  constexpr uint32_t S = SUB ? SUB / 2u : 1024u;            // a lane's two vectors, S apart
  constexpr uint32_t SPC = 2048u / (SUB ? SUB : 2048u), LPS = 64u / SPC;  // stripes / column, lanes / stripe
  const int w = (int)__builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint32_t lane = threadIdx.x & 63u;
  const uint32_t lane_off = (SUB ? lane % LPS : lane) * 16u;
  const uint64_t cols = a.cols_per_stripe;
  const uint64_t total = SUB ? (a.n_stripes + SPC - 1) / SPC : cols * a.n_stripes;
  const uint32_t mode = a.mode;
  auto col_off = [&](uint64_t c) {
    if constexpr (SUB) {
      uint64_t stripe = c * SPC + lane / LPS;
      if (stripe >= a.n_stripes) stripe = a.n_stripes - 1;  // loaded, never stored
      return stripe * a.stripe_stride + lane_off;
    }
    const uint64_t stripe = c / cols;
    return stripe * a.stripe_stride + (c - stripe * cols) * 2048u + lane_off;
  };
  const uint8_t* const* in = a.in + 8 * w;
  u32x4 buf[8][2];
  if (blockIdx.x < total) {
    const uint64_t off0 = col_off(blockIdx.x);
#pragma unroll
    for (int t = 0; t < 8; ++t) load2<S>(buf[t], in[t] + off0);
  }
  bool diff = false;
  for (uint64_t c = blockIdx.x; c < total; c += gridDim.x) {
    const uint64_t off = col_off(c);
    const uint64_t next = c + gridDim.x;
    uint32_t x[8][8];
#pragma unroll
    for (int t = 0; t < 8; ++t) slice8(buf[t], x[t]);
    if (next < total) {  // the next column's inputs in flight through the transform
      const uint64_t noff = col_off(next);
#pragma unroll
      for (int t = 0; t < 8; ++t) load2<S>(buf[t], in[t] + noff);
    }
    // phase A, then its results into the slots this wave read in phase C
    fft_a<K, B0>(w, x);
#pragma unroll
    for (int t = 0; t < 8; ++t) fft_put(st[8 * w + t], x[t], lane);
    __syncthreads();
    // phase B on this wave's groups (the same slots written back)
#pragma unroll
    for (int r = 0; r < 8; ++r) fft_get(st[(w * GPW + r / G) + 8 * (r % G)], x[r], lane);
    fft_phase_b_inv<K, B0, B1, 3>(x);
    fft_phase_b_fwd<K, B1, fft_log2(K) - 1>(x);
#pragma unroll
    for (int r = 0; r < 8; ++r) fft_put(st[(w * GPW + r / G) + 8 * (r % G)], x[r], lane);
    __syncthreads();
    // phase C on this wave's own elements, then its 8 outputs
#pragma unroll
    for (int t = 0; t < 8; ++t) fft_get(st[8 * w + t], x[t], lane);
    fft_c<K, B1>(w, x);
    const bool ok = SUB == 0 || c * SPC + lane / LPS < a.n_stripes;
    bool d = false;
#pragma unroll
    for (int t = 0; t < 8; ++t) {
      u32x4 v[2];
      unslice8(x[t], v);
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const uint64_t o16 = off + j * S;
        if (mode != kCheck && ok) stv<true>(a.out[8 * w + t] + o16, v[j]);
        if (mode != kStore) {
          const u32x4 q = ldv<true>(a.cmp[8 * w + t] + o16);
          d |= ok & ((q.x != v[j].x) | (q.y != v[j].y) | (q.z != v[j].z) | (q.w != v[j].w));
        }
      }
    }
    if (a.per_stripe) {
      if (d) flag_mismatch(a.mismatch + (SUB ? c * SPC + lane / LPS : c / cols));
    } else {
      diff |= d;
    }
  }
  if (mode != kStore && diff) flag_mismatch(a.mismatch);
}

// ------------------------------------------------------------------- host
// The rows the kernels replace: the K+K codec's parity rows (encode, verify;
// their own inverse, so also every data shard rebuilt from the parity shards
// in parity order: reconstruct with shards 0 .. K-1 missing, core.rs:801-923).
struct FftRows {
  std::vector<uint16_t> par[3];  // K = 16, 32, 64
};
const FftRows& fft_rows() {
  static const FftRows r = [] {
    FftRows f;
    for (int q = 0; q < 3; ++q) {
      const size_t K = 16u << q;
      const Matrix<Gf8Field> v = Matrix<Gf8Field>::vandermonde(2 * K, K);
      Matrix<Gf8Field> top(K, K), inv;
      for (size_t i = 0; i < K; ++i)
        for (size_t j = 0; j < K; ++j) top.at(i, j) = v.at(i, j);
      top.invert(inv);
      const Matrix<Gf8Field> m = v.multiply(inv);  // core.rs:430-436
      f.par[q].assign(m.d.begin() + K * K, m.d.begin() + 2 * K * K);
    }
    return f;
  }();
  return r;
}

template <int K>
const void* fft_fn(uint32_t sub) {
  return sub ? reinterpret_cast<const void*>(&fft_kernel<K, 0u, K, 1024u>)
             : reinterpret_cast<const void*>(&fft_kernel<K, 0u, K, 0u>);
}

}  // namespace

bool fft_applies(int field, uint32_t k, uint32_t p, const uint16_t* rows) {
  if (field != 8 || k != p || (k != 16 && k != 32 && k != 64) || !get_option(51)) return false;
  const int q = k == 16 ? 0 : k == 32 ? 1 : 2;
  return std::memcmp(rows, fft_rows().par[q].data(), (size_t)k * k * sizeof(uint16_t)) == 0;
}

hipError_t launch_fft(int field, uint32_t k, uint32_t p, const uint16_t* rows,
                      const uint8_t* const* in, uint8_t* const* out, const uint8_t* const* cmp,
                      uint64_t len, uint64_t stripe_stride, uint32_t n_stripes, uint32_t mode,
                      uint32_t* mismatch, bool per_stripe, hipStream_t stream, uint64_t* done) {
  *done = 0;
  if (!fft_applies(field, k, p, rows) || n_stripes == 0) return hipSuccess;
  // 1 KiB shards: two stripes per 2 KiB column; otherwise whole 2 KiB columns
  const uint32_t sub = len == 1024u && get_option(33) != 0 ? 1024u : 0u;
  const uint64_t cols = len / 2048u;
  if (!sub && cols == 0) return hipSuccess;
  FftArgs a;
  std::memset(&a, 0, sizeof a);
  a.stripe_stride = stripe_stride;
  a.cols_per_stripe = cols;
  a.mismatch = mismatch;
  a.n_stripes = n_stripes;
  a.mode = mode;
  a.per_stripe = per_stripe ? 1u : 0u;
  for (uint32_t i = 0; i < k; ++i) {
    a.in[i] = in[i];
    a.out[i] = out ? out[i] : nullptr;
    a.cmp[i] = cmp ? cmp[i] : nullptr;
  }
  const void* fn = nullptr;
  switch (k) {
    case 16: fn = fft_fn<16>(sub); break;
    case 32: fn = fft_fn<32>(sub); break;
    case 64: fn = fft_fn<64>(sub); break;
    default: return hipSuccess;
  }
  const uint64_t total = sub ? ((uint64_t)n_stripes + 1) / 2 : cols * n_stripes;
  // resident workgroups (LDS: k x 2 KiB each), a few rounds of them
  int dev = 0, n_cu = 0, per = 0;
  hipError_t e = hipGetDevice(&dev);
  if (e == hipSuccess) e = hipDeviceGetAttribute(&n_cu, hipDeviceAttributeMultiprocessorCount, dev);
  if (e == hipSuccess) e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, fn, k * 8, 0);
  if (e != hipSuccess) return e;
  const int64_t grid_opt = get_option(2);
  uint64_t gx = grid_opt > 0 ? (uint64_t)grid_opt : (uint64_t)std::max(per, 1) * (uint64_t)n_cu;
  if (gx > total) gx = total;
  if (gx > 0x7fffffffu) gx = 0x7fffffffu;
  void* args[] = {&a};
  e = hipLaunchKernel(fn, dim3((uint32_t)gx), dim3(k * 8), args, 0, stream);
  if (e != hipSuccess) return e;
  note_kernel("fft gf8 %u+%u %s%s", k, p, mode == kStore ? "code" : "check", sub ? " sub1" : "");
  count_bitslice_launch();
  *done = sub ? len : cols * 2048u;
  return hipSuccess;
}

}  // namespace rse
