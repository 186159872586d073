/*
 * rse_hip.h -- C ABI of the MI355X-native Reed-Solomon erasure-coding library
 * (librse_hip.so).  Drop-in for the hot path of rust-rse/reed-solomon-erasure
 * v6.0.0: the codec API of core.rs (ReedSolomon<F>::new / encode / encode_sep /
 * encode_single / encode_single_sep / verify / verify_with_buffer / reconstruct /
 * reconstruct_data) over the galois_8 and galois_16 fields, plus the fused
 * shard x matrix kernel that replaces code_some_slices (core.rs:481-509) and the
 * native FFI kernel reedsolomon_gal_mul(_xor) (simd_c/reedsolomon.h:30-42).
 *
 * Conventions (mirroring the reference; see INTEGRATION.md for the Rust binding):
 *  - Shards are DEVICE pointers (HBM) unless the function name ends in _host;
 *    the Field/FFI slice hooks (rse_gal_mul*, rse_gf8/gf16_mul_slice) take
 *    host or device memory.
 *  - Lengths are in field ELEMENTS, like Rust slice lengths: bytes for GF(2^8),
 *    2-byte [u8;2] elements ({coefficient of x, constant}, galois_16.rs:49-51)
 *    for GF(2^16).
 *  - Return value: RSE_OK (0), one of the 13 reference errors (errors.rs:4-18,
 *    numbered as wasm/src/lib.rs:11-24), or an RSE_ERR_* library status >= 100.
 *  - On any error nothing is written (core.rs:673-676).
 *  - Work is enqueued on `stream` (a hipStream_t; NULL = the legacy default
 *    stream) and runs asynchronously, except verify*, whose boolean result
 *    requires waiting before returning: for the stream's work up to and
 *    including the check, or (RSE_OPT_SPIN_WAIT, one compiled check-kernel
 *    launch) for the check kernel's completion word, stored after every one of
 *    its memory accesses has completed.  Either way the shards may be reused
 *    once the call returns.  Each call runs on
 *    the device that owns `stream` (NULL: the current device); the caller's
 *    current device is restored on return.
 *  - A codec is immutable after rse_codec_new except for its mutex-guarded
 *    decode-matrix LRU cache (capacity 254, core.rs:24), so concurrent calls on
 *    different streams are allowed (core.rs:349).
 *  - The caller owns all shard memory; the library never frees caller buffers.
 */
#ifndef RSE_HIP_H
#define RSE_HIP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- status codes ---------------------------------------------------- */
#define RSE_OK 0
/* errors.rs:4-18, in declaration order */
#define RSE_TOO_FEW_SHARDS 1
#define RSE_TOO_MANY_SHARDS 2
#define RSE_TOO_FEW_DATA_SHARDS 3
#define RSE_TOO_MANY_DATA_SHARDS 4
#define RSE_TOO_FEW_PARITY_SHARDS 5
#define RSE_TOO_MANY_PARITY_SHARDS 6
#define RSE_TOO_FEW_BUFFER_SHARDS 7
#define RSE_TOO_MANY_BUFFER_SHARDS 8
#define RSE_INCORRECT_SHARD_SIZE 9
#define RSE_TOO_FEW_SHARDS_PRESENT 10
#define RSE_EMPTY_SHARD 11
#define RSE_INVALID_SHARD_FLAGS 12
#define RSE_INVALID_INDEX 13
/* library statuses (no reference counterpart: the reference panics or cannot fail) */
#define RSE_ERR_INVALID_ARGUMENT 100 /* NULL pointer, unknown field, bad size */
#define RSE_ERR_DEVICE 101           /* HIP runtime error; see rse_last_device_error */
#define RSE_ERR_NO_MEMORY 102
#define RSE_ERR_SINGULAR_MATRIX 103  /* matrix.rs:11-13 Error::SingularMatrix */

#define RSE_FIELD_GF8 8   /* galois_8::Field,  ORDER 256   */
#define RSE_FIELD_GF16 16 /* galois_16::Field, ORDER 65536 */

typedef struct rse_codec rse_codec;
typedef void *rse_stream_t; /* hipStream_t */

/* Human-readable message; reference errors use errors.rs:20-38 verbatim. */
const char *rse_strerror(int status);
/* hipError_t of the last RSE_ERR_DEVICE on this thread (0 if none). */
int rse_last_device_error(void);
/* Library version string. */
const char *rse_version(void);
/* Identity of the last coding kernel this thread launched, e.g. "bitslice gf8
 * 10+4 v5 nt1" (compiled-in bit-sliced), "bitslice-jit gf16 12+8" (specialised
 * at run time), "table gf8 50+20 fused nt1"; "" before the first launch.
 * Diagnostics: profiles are attributed to the kernel that actually ran. */
const char *rse_last_kernel(void);

/* ---- codec: core.rs:343-923 ------------------------------------------ */
/* ReedSolomon::new (core.rs:445-467): TooFewDataShards / TooFewParityShards /
 * TooManyShards (data + parity > ORDER).  Builds the systematic matrix
 * V * (V[0..k])^-1 (core.rs:430-436) on the host; touches no device. */
int rse_codec_new(int field, size_t data_shards, size_t parity_shards, rse_codec **out);
void rse_codec_free(rse_codec *codec);
int rse_codec_field(const rse_codec *codec);
size_t rse_codec_data_shard_count(const rse_codec *codec);   /* core.rs:469 */
size_t rse_codec_parity_shard_count(const rse_codec *codec); /* core.rs:473 */
size_t rse_codec_total_shard_count(const rse_codec *codec);  /* core.rs:477 */
/* Copy the (k+p) x k encoding matrix, row-major, elem bytes per element. */
int rse_codec_matrix(const rse_codec *codec, uint8_t *out, size_t out_bytes);
/* Which kernels code this codec's whole 16 KiB and 4 KiB chunks (no reference counterpart;
 * results are identical either way).  Codecs other than the compiled-in ones get
 * bit-sliced kernels specialised at run time: the first call that codes at least
 * 4 KiB per shard (or this call with wait != 0) starts a hiprtc compile of the
 * codec's parity rows on a background thread (host CPU only) -- one module for
 * p <= 8 and k <= 32, one per 8 x 32 block of the rows otherwise.  wait != 0
 * blocks until every build has finished. */
#define RSE_KERNELS_TABLE 0             /* table kernels (rse_kernels.hip) */
#define RSE_KERNELS_COMPILED 1          /* bit-sliced, compiled into the library */
#define RSE_KERNELS_SPECIALISED 2       /* bit-sliced, specialised at run time, ready */
#define RSE_KERNELS_SPECIALISING 3      /* compile in flight (wait == 0) */
#define RSE_KERNELS_SPECIALISE_FAILED 4 /* compile failed: table kernels */
#define RSE_KERNELS_FFT 5               /* additive-FFT kernels, compiled into the library
                                           (GF(2^8) k = p = 16, 32, 64; RSE_OPT_FFT) */
int rse_codec_kernel_kind(const rse_codec *codec, int wait);

/* encode (core.rs:597-611): shards[0..k] data, shards[k..k+p] parity (overwritten). */
int rse_encode(const rse_codec *codec, void *const *shards, const size_t *lens,
               size_t n_shards, rse_stream_t stream);
/* encode_sep (core.rs:617-632) */
int rse_encode_sep(const rse_codec *codec, const void *const *data, const size_t *data_lens,
                   size_t n_data, void *const *parity, const size_t *parity_lens,
                   size_t n_parity, rse_stream_t stream);
/* encode_single (core.rs:545-562): i_data == 0 overwrites parity, later indices
 * accumulate (core.rs:503-507).  Used by ShardByShard (core.rs:101-231). */
int rse_encode_single(const rse_codec *codec, size_t i_data, void *const *shards,
                      const size_t *lens, size_t n_shards, rse_stream_t stream);
/* encode_single_sep (core.rs:576-592) */
int rse_encode_single_sep(const rse_codec *codec, size_t i_data, const void *single,
                          size_t single_len, void *const *parity, const size_t *parity_lens,
                          size_t n_parity, rse_stream_t stream);
/* verify (core.rs:637-651): *ok = 1 iff the parity matches.  Reads k+p shards
 * once, writes nothing.  Waits for the check (see above). */
int rse_verify(const rse_codec *codec, const void *const *shards, const size_t *lens,
               size_t n_shards, int *ok, rse_stream_t stream);
/* verify_with_buffer (core.rs:654-669): on RSE_OK the buffer holds the correct
 * parity whether or not verification passed (core.rs:328-331). */
int rse_verify_with_buffer(const rse_codec *codec, const void *const *shards,
                           const size_t *lens, size_t n_shards, void *const *buffer,
                           const size_t *buffer_lens, size_t n_buffer, int *ok,
                           rse_stream_t stream);
/* reconstruct / reconstruct_data (core.rs:680-695, 733-923) with the
 * ReconstructShard semantics of (T, bool) (lib.rs:168-200): present[i] != 0
 * marks shard i present; a missing shard's buffer must still have the common
 * length (else IncorrectShardSize) and is overwritten.  In data-only mode
 * missing parity buffers are neither checked nor touched (core.rs:805-806). */
int rse_reconstruct(const rse_codec *codec, void *const *shards, const size_t *lens,
                    const uint8_t *present, size_t n_shards, rse_stream_t stream);
int rse_reconstruct_data(const rse_codec *codec, void *const *shards, const size_t *lens,
                         const uint8_t *present, size_t n_shards, rse_stream_t stream);

/* ---- flat contiguous stripes (wasm/src/lib.rs:45-73 ABI, many stripes) --- */
/* `stripes` holds n_stripes consecutive stripes; each stripe is k+p shards of
 * shard_len elements laid end to end (the wasm encode() layout).  One launch. */
int rse_encode_flat(const rse_codec *codec, void *stripes, size_t shard_len,
                    size_t n_stripes, rse_stream_t stream);
/* verify (core.rs:637-651) of every stripe in one pass: ok[s] = 1 iff stripe
 * s's parity matches.  Reads each shard once, writes nothing.  Synchronises
 * `stream`.  (No reference counterpart: the crate verifies one stripe per
 * call; this is the batched form of the same check for scrubbing.) */
int rse_verify_flat(const rse_codec *codec, const void *stripes, size_t shard_len,
                    size_t n_stripes, uint8_t *ok, rse_stream_t stream);
/* Same layout; every stripe has the same erasure pattern `present[k+p]`
 * (wasm reconstruct(): reconstruct_data semantics). */
int rse_reconstruct_data_flat(const rse_codec *codec, void *stripes, size_t shard_len,
                              size_t n_stripes, const uint8_t *present, rse_stream_t stream);
/* Same layout; EVERY stripe has its own erasure pattern: present is
 * n_stripes x (k+p) flags, row s for stripe s.  reconstruct (data_only = 0,
 * core.rs:680) or reconstruct_data (data_only = 1, core.rs:690) of each stripe,
 * with the per-stripe planning of core.rs:733-923 (valid/invalid partition,
 * decode-matrix inversion, composed parity rows) done by a HIP kernel: two
 * launches for the whole batch.  Errors (TooFewShardsPresent / EmptyShard for
 * the first offending stripe) are detected before any stripe is modified.
 * Whole 16 KiB chunks of codecs with bit-sliced kernels (compiled in or run-time
 * specialised, either field) are planned per stripe on the device (e x e
 * syndrome inverse) and coded by the bit-sliced syndrome kernel; the rest of
 * every shard, and other GF(2^8) codecs with k <= 32 and p <= 16, use the
 * device planner with k x k inverses and the table kernels; anything else
 * falls back to the host planner stripe by stripe (same results).  `present`
 * may be host memory or device memory of the stripes' device (flags a GPU
 * scrub produced: they are then read in place, never copied, and the
 * shared-pattern detection -- a host pass -- is skipped).  Returns after the
 * work is queued and the host inputs have been consumed. */
int rse_reconstruct_batch(const rse_codec *codec, void *stripes, size_t shard_len,
                          size_t n_stripes, const uint8_t *present, int data_only,
                          rse_stream_t stream);

/* ---- low level: the fused kernel itself ------------------------------ */
/* outputs[r] (+)= sum_i rows[r*n_in + i] * inputs[i] over len elements.
 * rows is HOST memory, n_out x n_in elements (GF(2^16): [u8;2] each).
 * accumulate = 0 reproduces code_some_slices (core.rs:481-490, first input
 * overwrites); accumulate = 1 XORs into the outputs (mul_slice_add). */
int rse_code_shards(int field, const uint8_t *rows, size_t n_out, size_t n_in,
                    const void *const *inputs, void *const *outputs, size_t len,
                    int accumulate, rse_stream_t stream);
/* rse_code_shards on HOST inputs and outputs (the host pipeline above): the
 * one hook that puts the reference's code_some_slices (core.rs:481-490) on
 * the GPU unchanged -- encode, verify and reconstruct all funnel into it
 * (core.rs:522, 629, 861, 918).  Synchronous. */
int rse_code_shards_host(int field, const uint8_t *rows, size_t n_out, size_t n_in,
                         const void *const *inputs, void *const *outputs, size_t len,
                         int accumulate, rse_stream_t stream);
/* The Field/FFI slice hooks below take in/out WHEREVER THEY LIVE, as the
 * reference's callers do (they pass host slices): the library asks the runtime
 * (hipPointerGetAttributes) where each buffer is.
 *  - in and out both device memory of one device (hipMalloc, managed): the
 *    kernel, asynchronous on `stream`;
 *  - either in host memory (pageable, pinned or registered): the host
 *    pipeline -- H2D, kernel, D2H -- synchronous: out holds the result on
 *    return.  Pinned memory overlaps the copies; pageable memory works.
 * galois_8 mul_slice / mul_slice_xor (galois_8.rs:291-327): out = c*in (or
 * out ^= c*in) over GF(2^8). */
int rse_gf8_mul_slice(uint8_t c, const void *in, void *out, size_t len, int xor_into,
                      rse_stream_t stream);
/* The reference FFI kernel itself, same signature and contract:
 * reedsolomon_gal_mul / reedsolomon_gal_mul_xor (simd_c/reedsolomon.h:30-42,
 * bound at galois_8.rs:267-283).  low/high are the coefficient's 16-entry
 * nibble tables (MUL_TABLE_LOW/HIGH[c], build.rs:75-94; host memory); in/out
 * host or device memory as above.  Returns when out holds the result, as the
 * CPU kernel does, having waited only for its own work (a library stream, not
 * the whole device).  Returns the bytes processed: len (no scalar tail for
 * the caller to finish, galois_8.rs:301-304), or 0 on a device failure with
 * nothing written (rse_last_device_error says why).  On host slices a 0 lets
 * the reference's tail loop do the whole slice on the CPU, which is correct;
 * a caller passing DEVICE slices must treat 0 (for len > 0) as an error and
 * never run a host tail on them. */
size_t rse_gal_mul(const uint8_t *low, const uint8_t *high, const uint8_t *in, uint8_t *out,
                   size_t len);
size_t rse_gal_mul_xor(const uint8_t *low, const uint8_t *high, const uint8_t *in, uint8_t *out,
                       size_t len);
/* galois_16's Field::mul_slice / mul_slice_add (the trait defaults,
 * lib.rs:99-118), host or device memory as above: c is one [u8;2] element
 * {coefficient of x, constant}; len counts elements.  add_into = 0:
 * out = c*in, 1: out += c*in. */
int rse_gf16_mul_slice(const uint8_t *c, const void *in, void *out, size_t len, int add_into,
                       rse_stream_t stream);

/* ---- device matrix inversion (matrix.rs:195-261 semantics) ----------- */
/* Invert `batch` n x n matrices (device memory, row-major), one workgroup per
 * matrix (Gauss-Jordan; the augmented matrix in LDS up to n = 127, else in a
 * stream-ordered device workspace).  singular[b] = 1 for a singular matrix
 * (matrix.rs:11-13 Error::SingularMatrix; its out[b] is left unwritten), else
 * 0.  Asynchronous on `stream`.
 * GF(2^8): one byte per element, n <= 255 (the field's largest codec). */
int rse_gf8_invert_batch(const void *d_in, void *d_out, uint32_t *d_singular, size_t n,
                         size_t batch, rse_stream_t stream);
/* GF(2^16): [u8;2] elements {coefficient of x, constant} (galois_16.rs:49-51),
 * n <= 4096.  The decode matrices of galois_16 codecs (core.rs:697-731). */
int rse_gf16_invert_batch(const void *d_in, void *d_out, uint32_t *d_singular, size_t n,
                          size_t batch, rse_stream_t stream);

/* ---- host-memory (end-to-end) path ----------------------------------- */
/* The reference API's own form: shards are caller slices in HOST memory
 * (core.rs:597-695).  Each call pipelines chunks of every shard through the
 * device -- H2D of the shards the operation reads, the kernels, D2H of the
 * shards it writes, on separate streams over a ring of device buffers -- and
 * returns when the results are in host memory (synchronous).  Only what the
 * operation needs crosses PCIe: reconstruct uploads the k valid shards of
 * core.rs:801-841 and downloads only the rebuilt ones.  Pinned host memory
 * gives overlapped DMA; pageable memory works but serialises the copies.
 * Same validation, error precedence and results as the device entries. */
/* encode (core.rs:597-611) */
int rse_encode_host(const rse_codec *codec, void *const *shards, const size_t *lens,
                    size_t n_shards, rse_stream_t stream);
/* encode_sep (core.rs:617-632), encode_single (core.rs:545-562) and
 * encode_single_sep (core.rs:576-592; ShardByShard's calls) on host shards. */
int rse_encode_sep_host(const rse_codec *codec, const void *const *data, const size_t *data_lens,
                        size_t n_data, void *const *parity, const size_t *parity_lens,
                        size_t n_parity, rse_stream_t stream);
int rse_encode_single_host(const rse_codec *codec, size_t i_data, void *const *shards,
                           const size_t *lens, size_t n_shards, rse_stream_t stream);
int rse_encode_single_sep_host(const rse_codec *codec, size_t i_data, const void *single,
                               size_t single_len, void *const *parity, const size_t *parity_lens,
                               size_t n_parity, rse_stream_t stream);
/* Flat host stripes (rse_encode_flat layout, HOST memory): the same pipeline
 * over every chunk of every stripe, so PCIe stays busy across stripes. */
int rse_encode_host_flat(const rse_codec *codec, void *stripes, size_t shard_len,
                         size_t n_stripes, rse_stream_t stream);
/* verify (core.rs:637-651) / verify_with_buffer (core.rs:654-669; the host
 * buffer receives the correct parity on RSE_OK) */
int rse_verify_host(const rse_codec *codec, const void *const *shards, const size_t *lens,
                    size_t n_shards, int *ok, rse_stream_t stream);
int rse_verify_with_buffer_host(const rse_codec *codec, const void *const *shards,
                                const size_t *lens, size_t n_shards, void *const *buffer,
                                const size_t *buffer_lens, size_t n_buffer, int *ok,
                                rse_stream_t stream);
/* rse_verify_flat over flat HOST stripes: ok[s] per stripe. */
int rse_verify_host_flat(const rse_codec *codec, const void *stripes, size_t shard_len,
                         size_t n_stripes, uint8_t *ok, rse_stream_t stream);
/* reconstruct / reconstruct_data (core.rs:680-695) with (T, bool) semantics,
 * as rse_reconstruct / rse_reconstruct_data. */
int rse_reconstruct_host(const rse_codec *codec, void *const *shards, const size_t *lens,
                         const uint8_t *present, size_t n_shards, rse_stream_t stream);
int rse_reconstruct_data_host(const rse_codec *codec, void *const *shards, const size_t *lens,
                              const uint8_t *present, size_t n_shards, rse_stream_t stream);
/* rse_reconstruct_batch over flat HOST stripes: every stripe its own erasure
 * pattern (present: n_stripes x (k+p)); stripes with nothing missing move no
 * bytes.  Errors are detected before any stripe is touched. */
int rse_reconstruct_host_batch(const rse_codec *codec, void *stripes, size_t shard_len,
                               size_t n_stripes, const uint8_t *present, int data_only,
                               rse_stream_t stream);

/* ---- synchronous calls (the reference's own contract) ----------------- */
/* encode / verify / reconstruct / reconstruct_data of ONE stripe of device
 * shards that return when the result is in device memory, like the
 * reference's ReedSolomon methods (core.rs:597-611, 637-651, 680-695): same
 * validation, errors and bytes as rse_encode / rse_verify / rse_reconstruct /
 * rse_reconstruct_data.  No stream: the call is not ordered after work the
 * caller queued -- the caller has finished writing the shards it passes (for
 * example by synchronising its stream).  Small stripes (GF(2^8) codecs and
 * GF(2^16) codecs of at most 256 shards, 16-byte aligned shards, at most
 * RSE_OPT_DISPATCH_MAX_BYTES per shard, k x outputs <= 1024) go to a resident
 * workgroup that polls pinned host memory for requests (RSE_OPT_DISPATCH): no
 * kernel launch, no stream synchronisation -- a round trip of a few
 * microseconds.  It ends by itself after RSE_OPT_DISPATCH_IDLE_US without a
 * call, so it never holds the device for longer (a hipDeviceSynchronize may
 * wait that long).  Anything else runs the usual kernels on a library stream
 * and waits for them.  Thread-safe; calls to one device are served one at a
 * time. */
int rse_encode_now(const rse_codec *codec, void *const *shards, const size_t *lens, size_t n);
int rse_verify_now(const rse_codec *codec, const void *const *shards, const size_t *lens,
                   size_t n, int *ok);
int rse_reconstruct_now(const rse_codec *codec, void *const *shards, const size_t *lens,
                        const uint8_t *present, size_t n);
int rse_reconstruct_data_now(const rse_codec *codec, void *const *shards, const size_t *lens,
                             const uint8_t *present, size_t n);
/* Ends the resident dispatcher kernels now (they end by themselves when idle). */
void rse_dispatcher_stop(void);

/* ---- options (rse_set_option / rse_get_option) --------------------------
 * The options a caller of the drop-in may set: run-time specialisation, the
 * host pipeline, the resident dispatcher; and read-only counters.  Results
 * never depend on any option.  The library's tuning and A/B switches (launch
 * shapes, kernel variants, network generators; include/rse_hip_tune.h) are
 * refused with RSE_ERR_INVALID_ARGUMENT unless the environment has
 * RSE_TUNE=1 (the test suite and tools/ set it). */
#define RSE_OPT_BITSLICE_LAUNCHES 6 /* read-only, per thread: number of bit-sliced kernel
                                       launches so far (diagnostics / tests) */
#define RSE_OPT_HOST_CHUNK_KIB 7    /* rse_*_host*: bytes per shard per pipeline chunk, KiB */
#define RSE_OPT_HOST_H2D_STREAMS 8  /* rse_*_host*: streams carrying H2D copies (1..4) */
#define RSE_OPT_JIT 9               /* run-time specialised kernels: 0 off, 1 used once built
                                       (default), 2 the first launch waits for the build */
#define RSE_OPT_JIT_MODULES 10      /* read-only: specialised modules compiled by this process
                                       (builds run in rse_jitc helper processes, several at a
                                       time, when the helper sits next to the library) */
#define RSE_OPT_JIT_PATTERNS 11     /* 1: decode patterns used twice get their own specialised
                                       kernel (reconstruct at encode speed); 0 off */
#define RSE_OPT_PATTERN_LAUNCHES 12 /* read-only, per thread: reconstructs that ran on a
                                       decode-pattern kernel */
#define RSE_OPT_JIT_DISK_CACHE 15   /* 1 (default): specialised modules are cached on disk
                                       ($RSE_JIT_CACHE_DIR, else $XDG_CACHE_HOME/rse_hip, else
                                       ~/.cache/rse_hip), keyed by library version + source, so
                                       another process loads them instead of compiling */
#define RSE_OPT_JIT_CACHE_HITS 16   /* read-only: modules this process loaded from the disk cache */
#define RSE_OPT_SCRATCH_LIVE 24     /* read-only: per-call device resource sets (verdict words, library
                                       stream, host-pipeline streams/events/ring) in existence, leased or
                                       idle.  Calls lease one from a process-wide pool that keeps at most 4
                                       idle per device, so threads that come and go leave nothing behind */
#define RSE_OPT_HOST_PLANNED_STRIPES 25 /* read-only, per thread: stripes rse_reconstruct_batch
                                       planned on the host (a batch past the device planner's LDS
                                       budget: more than 8192 shards or very many erasures) */
#define RSE_OPT_JIT_MAX_PATTERNS 35  /* decode-pattern modules built per process (default 64);
                                        past it, patterns run on the syndrome / table kernels */
#define RSE_OPT_JIT_MAX_PATTERN_BLOCKS 36 /* blocks of wide decode patterns per process (64) */
#define RSE_OPT_DISPATCH 39           /* 1 (default): small *_now calls run on the resident dispatcher;
                                        0: always the launch path (A/B) */
#define RSE_OPT_DISPATCH_IDLE_US 40   /* the resident dispatcher ends after this many microseconds
                                        without a call (default 200).  It runs on a low-priority
                                        stream, so other streams' kernels never queue behind it,
                                        but a device-wide synchronisation (hipDeviceSynchronize,
                                        torch.cuda.synchronize()) right after a *_now call waits
                                        until it has idled out: ~230 us per call+sync at 200,
                                        ~2 ms at 2000 (tools/dispatch_sync_probe.py);
                                        rse_dispatcher_stop() ends it at once */
#define RSE_OPT_DISPATCH_MAX_BYTES 41 /* shard bytes up to which a *_now call is dispatched
                                        (default 65536) */
#define RSE_OPT_DISPATCHED 42         /* read-only: *_now calls the dispatcher served */
#define RSE_OPT_DISPATCH_LAUNCHES 43  /* read-only: launches of the resident dispatcher */
#define RSE_OPT_DISPATCH_WORKGROUPS 45 /* workgroups of the resident dispatcher (1..64, default 8):
                                        a request is coded by as many as its size needs; only
                                        the first polls more than 16 bytes per poll. Read at launch */
/* Process-wide; returns RSE_ERR_INVALID_ARGUMENT for an unknown key, a refused value, or a
 * tuning key without RSE_TUNE=1. */
int rse_set_option(int key, int64_t value);
/* Current value, or -1 for an unknown key. */
int64_t rse_get_option(int key);

/* ---- utilities (benchmarks and tests) -------------------------------- */
/* Fill device memory with the splitmix64 byte stream of (seed, shard_id):
 * 64-bit word w = mix(seed + shard_id * 2^40 + w), little endian. */
int rse_fill_splitmix(void *dst, size_t nbytes, uint64_t seed, uint64_t shard_id,
                      rse_stream_t stream);

#ifdef __cplusplus
}
#endif
#endif /* RSE_HIP_H */
