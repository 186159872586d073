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
};

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

// Device-resident batched reconstruct (GF(2^8), k <= kMaxIn, p <= kMaxOut):
// per stripe, plan (partition, inverse, composed rows) into d_descs[stripe]
// on the device, then code every stripe from its descriptor.  `base` holds
// n_stripes flat stripes of `total` shards of shard_bytes each; d_present is
// n_stripes x total flags; d_matrix the (total x k) encoding matrix.
// Only bytes [off, off + len) of every shard are coded (the bit-sliced batch
// path codes the whole chunks before).
hipError_t launch_recon_batch(const uint8_t* d_matrix, const uint8_t* d_present, uint32_t k,
                              uint32_t total, uint32_t data_only, uint8_t* base,
                              uint64_t shard_bytes, uint64_t off, uint64_t len,
                              uint32_t n_stripes, CodeArgs* d_descs, hipStream_t stream);

// Table kernels only (launch_code minus the bit-sliced dispatch).
hipError_t launch_table(int field, const CodeArgs& args, hipStream_t stream);

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
// compiled (or run-time specialised) ones for *handled to be set.  n_vec:
// 16-byte vectors per shard.
hipError_t launch_bitslice_recon(int field, uint32_t k, uint32_t p, const uint16_t* parity_rows,
                                 const BsReconArgs& a, uint64_t n_vec, hipStream_t stream,
                                 bool* handled);

// rse_reconstruct_batch on the bit-sliced kernels: a device planner writes one
// BsReconArgs per stripe (its own erasure pattern: partition, e x e syndrome
// inverse, mixing rows), then the syndrome kernel codes the whole 16 KiB
// chunks of every stripe from them.  d_rows: the p x k parity rows on the
// device (parity_rows: the same on the host, to select the kernels); need:
// sigma rows any stripe uses (max row + 1).  *handled unset = nothing queued.
hipError_t launch_bitslice_recon_batch(int field, uint32_t k, uint32_t p,
                                       const uint16_t* parity_rows, const uint16_t* d_rows,
                                       const uint8_t* d_present, uint32_t data_only,
                                       uint8_t* base, uint64_t shard_bytes, uint32_t n_stripes,
                                       uint32_t need, BsReconArgs* d_descs, hipStream_t stream,
                                       bool* handled);

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
  int n_rec = 0;
  int rec_ns[5] = {};           // sigma rows of rec[i], ascending
  hipFunction_t rec[5] = {};    // bitslice reconstruct (BsReconArgs, chunks per stripe)
  hipFunction_t rec_desc[5] = {};  // ... over per-stripe BsReconArgs (descs, cps, n_stripes)
  hipFunction_t wide = nullptr;    // kJitWide: rse_jit_wide (WideArgs)
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
// 10+4 v1 nt1", "table gf16 20+8 fused nt1", ...): rse_last_kernel().
void note_kernel(const char* fmt, ...);
const char* last_kernel();

// Fill nbytes of device memory with the splitmix64 byte stream of
// (seed, shard_id) -- identical to oracle/oracle.py: splitmix_bytes.
hipError_t launch_fill_splitmix(void* dst, uint64_t nbytes, uint64_t seed,
                                uint64_t shard_id, hipStream_t stream);

// Device Gauss-Jordan inversion of n x n matrices over GF(2^8) (batched: one
// workgroup per matrix).  in/out are device pointers to batch*n*n bytes;
// singular[b] receives 1 for a singular matrix.
hipError_t launch_gf8_invert(const uint8_t* in, uint8_t* out, uint32_t* singular,
                             uint32_t n, uint32_t batch, hipStream_t stream);
#endif  // RSE_JIT

}  // namespace rse
