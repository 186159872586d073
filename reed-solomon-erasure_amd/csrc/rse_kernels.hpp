// rse_kernels.hpp -- internal launch interface between the host codec
// (rse_codec.cpp) and the CDNA4 kernels (rse_kernels.hip, rse_bitslice.hip,
// and the run-time specialised modules of rse_jit.cpp).
//
// One fused kernel family replaces the reference's whole code_some_slices
// (core.rs:481-509): every input shard byte is read once from HBM, every output
// byte is written once, and the k x p' coefficient products are XOR-accumulated
// in VGPRs.  The same launch also serves check_some_slices_with_buffer
// (core.rs:511-532) through the CHECK modes, so verify never round-trips parity
// through HBM twice.
//
// The argument blocks below are also compiled by hiprtc (RSE_JIT defined): that
// part must stay free of host-only headers and declarations.
#pragma once

#ifndef RSE_JIT
#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>
#endif

namespace rse {

// Shards per launch carried in the kernel-argument segment (no device-side
// descriptor, hence no lifetime hazard across streams).  Bigger codecs are split
// by the host into input/output chunks (see rse_codec.cpp: launch_code).
constexpr int kMaxIn = 32;
constexpr int kMaxOut = 16;

enum CodeMode : uint32_t {
  kStore = 0,       // out[r]  = sum_i coef[r][i] * in[i]            (encode)
  kCheck = 1,       // mismatch |= (sum_i coef[r][i] * in[i]) != cmp[r]   (verify)
  kCheckStore = 2,  // both: buffer written and compared (verify_with_buffer)
};

struct CodeArgs {
  const uint8_t* in[kMaxIn];
  uint8_t* out[kMaxOut];
  const uint8_t* cmp[kMaxOut];
  uint64_t stripe_stride;  // bytes between stripe s and s+1 for EVERY pointer
  uint32_t n_stripes;      // stripes handled by this launch (>= 1)
  uint64_t n_vec;          // 16-byte vectors handled by the vector body
  uint64_t len;            // bytes per shard
  uint32_t* mismatch;      // device word, CHECK modes only
  uint32_t n_in, n_out;
  uint32_t mode;
  uint32_t accumulate;     // 1: out[r] ^= ... (ShardByShard / chunked inputs)
  uint32_t per_stripe;     // CHECK modes: 1 = mismatch[stripe] per stripe (verify_flat),
                           // 0 = one mismatch word for the launch
  uint32_t* done;          // check kernels: completion word (rse_device.hpp signal_done)
  uint32_t* done_count;    //   and its workgroup count; null: not armed
  // GF(2^8): coef[r][i] & 0xff.  GF(2^16): (coef_of_x << 8) | constant.
  uint16_t coef[kMaxOut][kMaxIn];
};

// Bit-sliced syndrome reconstruct for codecs with bit-sliced kernels
// (rse_bitslice.hip, rse_jit.cpp).  With P the codec's parity rows, S the e
// missing data shards and R e present parity rows:
//   sigma_r = sum over present data d of P[r][d] * shard_d   (XOR networks)
//   syndrome s_r = sigma_r ^ parity_r for r in R
//   output o = (out_sigma[o] >= 0 ? sigma_{out_sigma[o]} : 0)
//              ^ sum over r in R of w[o][r] * s_r
// (missing data: w = rows of (P[R][S])^-1; missing parity r: out_sigma = r,
// w = P[r][S] (P[R][S])^-1).  One pass over k surviving shards.
struct BsReconArgs {
  const uint8_t* data[kMaxIn];    // data shard d (read when present)
  const uint8_t* par[kMaxOut];    // parity shard r (read when a syndrome row)
  uint8_t* out[kMaxOut];          // output o
  uint64_t stripe_stride;
  uint32_t n_stripes;
  uint32_t present;               // bit d: data shard d present
  uint32_t sigma;                 // bit r: sigma_r is needed
  uint32_t synd;                  // bit r: parity row r is a syndrome row (R)
  uint32_t n_out;
  int32_t out_sigma[kMaxOut];     // sigma row XORed into output o, -1 for none
  uint16_t w[kMaxOut][kMaxOut];   // [o][r], zero unless r is in R
  // Horner masks of w (set_horner_masks, rows r < 8): byte j of hm[o] (byte
  // j % 4 of word j / 4) has bit r set iff coordinate NB - 1 - j of w[o][r]
  // in the Horner basis is 1 (NB = 8 / 16 coordinates for GF(2^8) / GF(2^16)).
  uint32_t hm[kMaxOut][4];
};

// ---- Horner mixing basis ----------------------------------------------------
// The run-time e x e mixing of the syndrome reconstruct multiplies sliced
// syndromes by run-time constants with Horner's rule over the coordinates c_i
// of a constant c in a polynomial basis {1, z, .., z^(NB-1)}:
//   c * s = (..((c_{NB-1} s) z + c_{NB-2} s) z + ..) z + c_0 s,
// so that multiplying the accumulator by z is a rotation of its planes plus
// 3 XORs of the top plane (the taps of z's minimal polynomial).
//  GF(2^8):  z = 2, the generator of build.rs (x^8 = x^4 + x^3 + x^2 + 1):
//            the standard basis, no conversion.
//  GF(2^16): z = 0x4815, a root of z^16 + z^6 + z^2 + z + 1 (an irreducible
//            pentanomial): sliced syndromes are converted into z-coordinates
//            (to_b) and the mixed outputs back (from_b), 16 x 16 bit matrices.
constexpr uint32_t kHornerTaps8 = (1u << 4) | (1u << 3) | (1u << 2);
constexpr uint32_t kHornerZ16 = 0x4815u;
constexpr uint32_t kHornerTaps16 = (1u << 6) | (1u << 2) | (1u << 1);

constexpr uint32_t hb_mul8(uint32_t a, uint32_t b) {  // GF(2^8) modulo 0x11D (build.rs:11)
  uint32_t r = 0;
  for (int i = 0; i < 8; ++i) {
    if ((b >> i) & 1u) r ^= a;
    a <<= 1;
    if (a & 0x100u) a ^= 0x11Du;
  }
  return r;
}
constexpr uint32_t hb_mul16(uint32_t a, uint32_t b) {  // galois_16.rs:146-162
  const uint32_t a1 = a >> 8, a0 = a & 0xFFu, b1 = b >> 8, b0 = b & 0xFFu;
  const uint32_t hh = hb_mul8(a1, b1);
  const uint32_t x = hb_mul8(a1, b0) ^ hb_mul8(a0, b1) ^ hb_mul8(2u, hh);
  return (x << 8) | (hb_mul8(a0, b0) ^ hb_mul8(128u, hh));
}

struct HornerBasis16 {
  uint16_t to_b[16];    // coordinate i of element e: parity(e & to_b[i])
  uint16_t from_b[16];  // bit j of an element: parity(coordinates & from_b[j])
  bool ok;              // z^16 = z^6 + z^2 + z + 1 and the powers are a basis
};
constexpr HornerBasis16 make_horner_basis16() {
  HornerBasis16 h{};
  uint32_t zp[17] = {};
  zp[0] = 1;
  for (int i = 0; i < 16; ++i) zp[i + 1] = hb_mul16(zp[i], kHornerZ16);
  uint32_t rel = zp[16] ^ 1u;
  for (int i = 1; i < 16; ++i)
    if ((kHornerTaps16 >> i) & 1u) rel ^= zp[i];
  for (int j = 0; j < 16; ++j)
    for (int i = 0; i < 16; ++i)
      if ((zp[i] >> j) & 1u) h.from_b[j] |= (uint16_t)(1u << i);
  // to_b = from_b^-1: Gauss-Jordan on [from_b | I] (bit 16 + j of row j)
  uint32_t m[16] = {};
  for (int j = 0; j < 16; ++j) m[j] = h.from_b[j] | (1u << (16 + j));
  bool full = true;
  for (int col = 0; col < 16; ++col) {
    int piv = col;
    while (piv < 16 && !((m[piv] >> col) & 1u)) ++piv;
    if (piv == 16) {
      full = false;
      break;
    }
    const uint32_t t = m[piv];
    m[piv] = m[col];
    m[col] = t;
    for (int r = 0; r < 16; ++r)
      if (r != col && ((m[r] >> col) & 1u)) m[r] ^= m[col];
  }
  for (int i = 0; i < 16; ++i) h.to_b[i] = (uint16_t)(m[i] >> 16);
  h.ok = full && rel == 0;
  return h;
}
constexpr HornerBasis16 kHornerBasis16 = make_horner_basis16();
static_assert(kHornerBasis16.ok, "z must be a root of the pentanomial and generate GF(2^16)");

// Coordinates of c in the Horner basis of the field.
__host__ __device__ inline uint32_t horner_coords(int field, uint32_t c) {
  if (field == 8) return c & 0xFFu;
  constexpr HornerBasis16 hb = make_horner_basis16();
  uint32_t r = 0;
  for (int i = 0; i < 16; ++i) r |= (uint32_t)__builtin_parity(c & hb.to_b[i]) << i;
  return r;
}

// BsReconArgs::hm from w, synd and n_out (after those are final).
__host__ __device__ inline void set_horner_masks(BsReconArgs& a, int field) {
  const int nb = field == 8 ? 8 : 16;
  for (int o = 0; o < kMaxOut; ++o)
    for (int q = 0; q < 4; ++q) a.hm[o][q] = 0;
  for (uint32_t o = 0; o < a.n_out && o < (uint32_t)kMaxOut; ++o)
    for (int r = 0; r < 8; ++r) {
      if (!((a.synd >> r) & 1u)) continue;
      const uint32_t co = horner_coords(field, a.w[o][r]);
      for (int j = 0; j < nb; ++j)
        if ((co >> (nb - 1 - j)) & 1u) a.hm[o][j >> 2] |= 1u << (8 * (j & 3) + r);
    }
}

// Header of a wide codec's argument block (rse_jit.cpp kJitWide).  The block
// is the header followed by the k input, p output and p compare pointers
// (WideArgs<k, p> in the module's source; the host packs the same bytes).
struct WideHdr {
  uint64_t stripe_stride;      // bytes between stripe s and s+1 for every pointer
  uint64_t chunks_per_stripe;  // whole 4 KiB chunks per shard coded by the launch
  uint32_t* mismatch;          // CHECK modes
  uint32_t n_stripes;
  uint32_t mode;               // CodeMode
  uint32_t per_stripe;         // CHECK modes: mismatch[stripe] instead of mismatch[0]
  uint32_t pad;
};

#ifndef RSE_JIT
// Launch the fused coding kernel over args.n_stripes stripes on `stream`.
// field is 8 or 16.  Returns a hipError_t.
hipError_t launch_code(int field, const CodeArgs& args, hipStream_t stream);

// Device-resident batched reconstruct planner (rse_kernels.hip
// recon_plan_kernel), either field, any codec: per stripe of a group of n_grp
// flat stripes (`base`: the group's first stripe; d_present: its n_grp x T
// flags), the partition, the e x e syndrome inverse and the composed rows are
// computed on the device and written as CodeArgs descriptors -- ceil(k / 32)
// input blocks x ceil(nout_cap / 16) output blocks per stripe -- then the
// table kernels code bytes [off, off + len) of every shard from them.
// d_parity: the p x k parity rows (uint16 elements).  e_cap / nout_cap: the
// most missing data shards / outputs of any stripe in the group.  Needs
// recon_plan_lds(...) <= kReconPlanLdsMax.
constexpr size_t kReconPlanLdsMax = 65536;
size_t recon_plan_lds(uint32_t k, uint32_t T, uint32_t e_cap, uint32_t nout_cap);
// rse_reconstruct_batch's validation of many stripes on the device
// (core.rs:747-772 per stripe): d_res[0..2] = max over stripes of `need` (the
// highest sigma row + 1), e (missing data) and outputs; d_res[4..5] = the
// 64-bit (first stripe with too few shards present) * 2 + 1, ~0 if none.
// d_res (8-byte aligned) must hold zeros in words 0..2 and all ones in 4..5.
hipError_t launch_batch_scan(const uint8_t* d_present, uint64_t n_stripes, uint32_t k, uint32_t p,
                             uint32_t data_only, uint32_t* d_res, hipStream_t stream);
hipError_t launch_recon_plan(int field, const uint16_t* d_parity, const uint8_t* d_present,
                             uint32_t k, uint32_t T, uint32_t data_only, uint32_t e_cap,
                             uint32_t nout_cap, uint8_t* base, uint64_t shard_bytes, uint64_t off,
                             uint64_t len, uint32_t n_grp, CodeArgs* d_descs, hipStream_t stream);

// Table kernels only (launch_code minus the bit-sliced dispatch).
hipError_t launch_table(int field, const CodeArgs& args, hipStream_t stream);

// Set by launch_bitslice when it launched a check kernel with CodeArgs::done
// armed (the launch is the whole job: the kernel signals its completion).
extern thread_local bool t_done_armed;

// Bit-sliced kernels (rse_bitslice.hip) for codecs whose parity rows are
// compiled in or were specialised at run time (rse_jit.cpp): the whole 16 KiB
// chunks of every shard, then the whole 4 KiB chunks of the rest.  Sets
// *handled when it launched and *done to the bytes of every shard coded (the
// caller codes the rest).
hipError_t launch_bitslice(int field, const CodeArgs& a, bool nt, int64_t grid,
                           hipStream_t stream, bool* handled, uint64_t* done);
uint64_t bitslice_chunk_bytes();
// 1 if (field, k, p) has bit-sliced kernels compiled into the library.
int bitslice_compiled(int field, uint32_t k, uint32_t p);

// parity_rows: the codec's p x k parity rows (row-major); must equal the
// compiled (or run-time specialised) ones for anything to be launched.  n_vec:
// 16-byte vectors per shard.  *done: the bytes of every shard coded, from 0
// (whole 16 KiB chunks, then whole 4 KiB chunks of the rest; 0: nothing
// launched, the caller codes the shards).
hipError_t launch_bitslice_recon(int field, uint32_t k, uint32_t p, const uint16_t* parity_rows,
                                 const BsReconArgs& a, uint64_t n_vec, hipStream_t stream,
                                 uint64_t* done);

// rse_reconstruct_batch on the bit-sliced kernels: a device planner writes one
// BsReconArgs per stripe (its own erasure pattern: partition, e x e syndrome
// inverse, mixing rows), then the syndrome kernels code the whole 16 KiB
// chunks of every stripe from them, and the whole 4 KiB chunks of the rest
// (one per wave).  d_rows: the p x k parity rows on the device (parity_rows:
// the same on the host, to select the kernels); d_tabs: the GF(2^8) log and
// exp tables on the device (kPlanTabBytes, plan_tables); need: sigma rows any
// stripe uses (max row + 1); e_cap: missing data shards any stripe has.
// *done = bytes of every shard coded (0: nothing queued).
constexpr size_t kPlanTabBytes = 256 + 512;
hipError_t launch_bitslice_recon_batch(int field, uint32_t k, uint32_t p,
                                       const uint16_t* parity_rows, const uint16_t* d_rows,
                                       const uint8_t* d_tabs, const uint8_t* d_present,
                                       uint32_t data_only, uint8_t* base, uint64_t shard_bytes,
                                       uint32_t n_stripes, uint32_t need, uint32_t e_cap,
                                       BsReconArgs* d_descs, hipStream_t stream, uint64_t* done);
// The planner's tables: log[256] then exp[512] of GF(2^8), generator 2
// modulo 0x11D (build.rs:13-43), exp doubled so exp[log a + log b] needs no
// reduction; log[0] = 0 and exp[510..511] = 0 are never read for nonzero a, b.
inline void plan_tables(uint8_t* t) {  // kPlanTabBytes bytes
  uint8_t* lg = t;
  uint8_t* ex = t + 256;
  uint32_t b = 1;
  for (uint32_t l = 0; l < 255; ++l) {
    lg[b] = (uint8_t)l;
    ex[l] = ex[l + 255] = (uint8_t)b;
    b <<= 1;
    if (b & 0x100u) b ^= 0x11Du;
  }
  lg[0] = 0;
  ex[510] = ex[511] = 0;
}

// ---- run-time specialisation (rse_jit.cpp) ----------------------------------
// Bit-sliced kernels for codecs not compiled into the library: the XOR networks
// of the codec's parity rows are generated as source and compiled for gfx950
// with hiprtc (host CPU only; no device work), then loaded per device on first
// use.  Results never depend on which kernel runs.
constexpr uint32_t kJitMaxOut = 8;  // p' <= 8: 16 x p' accumulator VGPRs
// What a registered set of rows is:
//  kJitCodec   a codec's parity rows, built with the syndrome reconstruct
//              kernels too;
//  kJitPattern a decode pattern (the composed rows of a reconstruct,
//              core.rs:697-731), encode kernel only, capped in number and
//              queue length;
//  kJitBlock   one <= 8 x <= 32 block of a wide codec's parity rows (k > 32
//              or p > 8) over its first 32 inputs: encode kernels
//              (jit_register_blocks);
//  kJitBlockAcc a block over later inputs: accumulate-mode encode kernels
//              only (each kernel is seconds of hiprtc for 32 x 8 blocks).
//  kJitWide    a wide codec's (or wide decode pattern's) whole rows in ONE
//              module: each wave of a workgroup codes its share of <= 8
//              outputs over all k inputs of the same 4 KiB chunk, so every
//              input is read from HBM once and every output written once
//              (rse_bitslice_core.hpp wide_body).
enum JitKind { kJitCodec = 0, kJitPattern = 1, kJitBlock = 2, kJitBlockAcc = 3, kJitWide = 4 };
// Wide modules: p <= 64 (8 waves of 8 outputs), and k + 2p pointers in the
// kernel-argument block.
constexpr uint32_t kWideMaxPtrs = 480;
bool wide_eligible(uint32_t k, uint32_t p);
// Outputs per wave of a wide module (RSE_OPT_WIDE_SPLIT, default 8): below 8,
// codecs with more parity rows than that take wide modules too (A/B: splitting
// a codec's outputs over 2 waves halves the accumulator VGPRs).
uint32_t wide_per_wave();
int jit_register_wide(int field, uint32_t k, uint32_t p, const uint16_t* rows, bool pattern);
int jit_wide_status(int field, uint32_t k, uint32_t p, const uint16_t* rows, bool wait);
// Codes the whole 4 KiB chunks of every shard (of n_stripes stripes) with the
// wide module of these rows if it is built (RSE_OPT_JIT 2: waits for it);
// *done = bytes per shard coded, 0 if it did not launch.
hipError_t launch_wide(int field, uint32_t k, uint32_t p, const uint16_t* rows,
                       const uint8_t* const* in, uint8_t* const* out, const uint8_t* const* cmp,
                       uint64_t len, uint64_t stripe_stride, uint32_t n_stripes, uint32_t mode,
                       uint32_t* mismatch, bool per_stripe, hipStream_t stream, uint64_t* done);
// Registers p x k rows (row-major) and queues their build on the background
// thread.  Returns 1 if registered (now or before), 0 if not eligible or
// refused.
int jit_register(int field, uint32_t k, uint32_t p, const uint16_t* rows, JitKind kind);
// Registers every kJitBlock block of a wide codec's p x k parity rows -- all of
// them or, past the block cap, none.  Blocks: rows [o0, o0 + 8) x inputs
// [i0, i0 + 32), the chunking of run_job (rse_codec.cpp).
// pattern: the rows are a wide decode pattern's (a separate, smaller budget:
// patterns never take the codecs' blocks, and never queue without bound).
int jit_register_blocks(int field, uint32_t k, uint32_t p, const uint16_t* rows, bool pattern);
// jit_status over all of a wide codec's blocks (the least ready one).
int jit_blocks_status(int field, uint32_t k, uint32_t p, const uint16_t* rows, bool wait);
// 2 ready, 1 building, 0 not registered, -1 build failed; wait != 0 blocks
// until the build has finished.
int jit_status(int field, uint32_t k, uint32_t p, const uint16_t* rows, bool wait);
struct JitFns {
  hipFunction_t enc = nullptr;  // bitslice encode/verify (CodeArgs, chunks per stripe)
  hipFunction_t enc4 = nullptr; // ... over 4 KiB chunks, one per wave
  hipFunction_t enc_acc = nullptr, enc4_acc = nullptr;  // accumulate mode (kJitBlockAcc)
  hipFunction_t chk = nullptr;  // the check modes' kernel, with the completion word
  hipFunction_t sub[2] = {};    // ... over 1 / 2 KiB shards, 4 / 2 stripes per 4 KiB chunk
  int n_rec = 0;
  int rec_ns[5] = {};           // sigma rows of rec[i], ascending
  hipFunction_t rec[5] = {};    // bitslice reconstruct (BsReconArgs, chunks per stripe)
  hipFunction_t rec_desc[5] = {};  // ... over per-stripe BsReconArgs (descs, cps, n_stripes)
  hipFunction_t rec_desc4[5] = {}; // ... over 4 KiB chunks, one per wave (descs, cps4, n, base)
  hipFunction_t rec4[5] = {};      // rec over 4 KiB chunks, one per wave (args, cps4, base)
  hipFunction_t wide = nullptr;    // kJitWide: rse_jit_wide (WideArgs)
  hipFunction_t wide_sub[2] = {};  // ... over 1 / 2 KiB shards (rse_jit_wide_s1 / _s2)
};
// Kernels of `stage` (0: encode/verify, 1: reconstruct) for a launch whose
// coefficients rows[o * stride + i] equal a registered codec's parity rows,
// loaded on the current device.  Returns false (and *err = hipSuccess) if there
// are none (yet: RSE_OPT_JIT 1 does not wait for a compile in flight, 2 does);
// *err is set on a module-load failure.  acc: the accumulate-mode kernels of a
// kJitBlockAcc entry (stage 0) instead.
bool jit_find(int field, uint32_t k, uint32_t p, const uint16_t* rows, size_t stride, int stage,
              JitFns* out, hipError_t* err, bool acc = false);
int64_t jit_modules_built();  // RSE_OPT_JIT_MODULES (compiled in this process)
int64_t jit_cache_hits();     // RSE_OPT_JIT_CACHE_HITS (loaded from the disk cache)

// Launch-shape options (keys as RSE_OPT_* in include/rse_hip.h).
int set_option(int key, int64_t value);
int64_t get_option(int key);
void count_bitslice_launch();  // RSE_OPT_BITSLICE_LAUNCHES
// Identity of the last coding kernel launched on this thread ("bitslice gf8
// 10+4 v5 nt1", "table gf16 20+8 fused nt1", ...): rse_last_kernel().
void note_kernel(const char* fmt, ...);
const char* last_kernel();

// Fill nbytes of device memory with the splitmix64 byte stream of
// (seed, shard_id) -- identical to oracle/oracle.py: splitmix_bytes.
hipError_t launch_fill_splitmix(void* dst, uint64_t nbytes, uint64_t seed,
                                uint64_t shard_id, hipStream_t stream);

// Device Gauss-Jordan inversion of n x n matrices over GF(2^8) or GF(2^16)
// (batched: one workgroup per matrix).  in/out: batch x n x n elements of the
// field's bytes (GF(2^16): [u8;2] {coefficient of x, constant}); singular[b]
// receives 1 for a singular matrix.  The augmented matrix lives in LDS when
// its n x 2n uint16 entries fit invert_lds_max_bytes(), else in gws (batch x
// n x 2n uint16, device memory; nullptr: LDS only).
hipError_t launch_invert(int field, const uint8_t* in, uint8_t* out, uint32_t* singular,
                         uint32_t n, uint32_t batch, uint16_t* gws, hipStream_t stream);
size_t invert_lds_max_bytes();
#endif  // RSE_JIT

}  // namespace rse
