// rse_codec.cpp -- host side of the drop-in: the ReedSolomon<F> codec of
// core.rs:343-923 (validation, matrix construction, decode-matrix LRU cache,
// reconstruct planning) above the fused HIP kernel, exported as the C ABI of
// include/rse_hip.h.
//
// Differences from the reference are in HOW, never in WHAT:
//  * code_some_slices (core.rs:481-509) makes k*p passes over memory; here one
//    kernel launch reads each input once and writes each output once.
//  * verify (core.rs:637-651) encodes into a scratch buffer and compares; here
//    the compare is fused into the same pass and no buffer is written.
//  * reconstruct (core.rs:733-923) regenerates missing data, then missing parity
//    from all data; here the missing parity rows are composed with the decode
//    rows on the host (exact GF algebra) so both come out of ONE pass over the k
//    surviving shards.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <array>
#include <atomic>
#include <cstdlib>
#include <cstring>
#include <list>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <vector>

#include "../../include/rse_hip.h"
#include "../../include/rse_hip_tune.h"
#include "rse_dispatch.hpp"
#include "rse_fft.hpp"
#include "rse_wideblk.hpp"
#include "rse_field.hpp"
#include "rse_kernels.hpp"

namespace {

using rse::CodeArgs;
using rse::kMaxIn;
using rse::kMaxOut;

thread_local int g_last_hip_error = 0;

int dev_fail(hipError_t e) {
  g_last_hip_error = (int)e;
  return e == hipErrorOutOfMemory ? RSE_ERR_NO_MEMORY : RSE_ERR_DEVICE;
}
#define RSE_HIP(call)                              \
  do {                                             \
    hipError_t e_ = (call);                        \
    if (e_ != hipSuccess) return dev_fail(e_);     \
  } while (0)

constexpr size_t kCacheCapacity = 254;  // core.rs:24 DATA_DECODE_MATRIX_CACHE_CAPACITY

// Row-major coefficient block handed to the kernel (uint16 elements).
struct Rows {
  size_t n_out = 0, n_in = 0;
  std::vector<uint16_t> c;
  uint16_t at(size_t r, size_t i) const { return c[r * n_in + i]; }
};

}  // namespace

struct rse_codec {
  int field;
  // The field the kernels code in.  GF(2^16) codecs of at most 256 shards
  // have every matrix entry in the GF(2^8) subfield (the Vandermonde points
  // 0..k+p-1 are subfield elements, galois_16.rs:97-107 nth(), and the
  // subfield is closed under the products and inverses of core.rs:430-436
  // and 697-731).  A subfield constant c multiplies an element a1 x + a0 as
  // (c a1) x + c a0 (galois_16.rs:20-52: no reduction term), i.e. each byte
  // of the element by itself in GF(2^8) (the base field is galois_8's).  So
  // every coding pass of such a codec -- encode, verify, every decode pattern
  // -- is the GF(2^8) pass with the same coefficients over the same bytes:
  // kfield 8 (RSE_OPT_SUBFIELD), half the XOR work of the 16 x 16 bit
  // matrices.  Otherwise kfield = field.
  int kfield;
  size_t k, p, total;
  rse::Matrix<rse::Gf8Field> m8;   // field == 8
  rse::Matrix<rse::Gf16Field> m16;  // field == 16
  // decode-matrix LRU keyed by invalid indices (core.rs:697-731)
  mutable std::mutex mu;
  struct Cached {
    std::vector<uint16_t> dec;  // k x k inverse of the valid rows
    uint32_t uses = 0;          // reconstructs that used this pattern (run-time kernels)
  };
  mutable std::list<std::pair<std::vector<size_t>, Cached>> lru;
  mutable std::map<std::vector<size_t>, decltype(lru)::iterator> index;
  // run-time specialisation requested (rse_jit.cpp; see want_bitslice)
  mutable std::atomic<bool> jit_requested{false};
  mutable std::atomic<uint64_t> wide_bytes{0};  // shard bytes a wide codec has coded (want_bitslice)
  // Per device: the parity rows (p x k halfwords) and, 256-aligned after them,
  // the device planners' GF(2^8) tables (rse::plan_tables), made on the first
  // batched reconstruct there and kept for the codec's life (plan_consts), so
  // a call copies neither.
  static constexpr int kDevs = 64;
  mutable std::atomic<uint8_t*> plan_dev[kDevs] = {};
  ~rse_codec() {
    for (auto& a : plan_dev)
      if (uint8_t* q = a.load()) (void)hipFree(q);
  }

  size_t esize() const { return field == 16 ? 2 : 1; }
  uint16_t mat(size_t r, size_t c) const { return field == 16 ? m16.at(r, c) : m8.at(r, c); }
  uint16_t mul(uint16_t a, uint16_t b) const {
    return field == 16 ? rse::Gf16Field::mul(a, b) : rse::Gf8Field::mul(a, b);
  }
  uint16_t inv(uint16_t a) const {
    return field == 16 ? rse::Gf16Field::inv(a) : rse::Gf8Field::inv(a);
  }
};

namespace {

// ------------------------------------------------------------- validation
// macros.rs:204-245 check_piece_count!
int check_count(size_t got, size_t want, int too_few, int too_many) {
  if (got < want) return too_few;
  if (got > want) return too_many;
  return RSE_OK;
}
// macros.rs:144-155 check_slices!(multi => ...)
int check_multi(const size_t* lens, size_t n) {
  const size_t size = lens[0];
  if (size == 0) return RSE_EMPTY_SHARD;
  for (size_t i = 0; i < n; ++i)
    if (lens[i] != size) return RSE_INCORRECT_SHARD_SIZE;
  return RSE_OK;
}

bool aligned16(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15u) == 0; }

// Every entry point works on the device that owns its stream: allocations
// (per-thread verdict words), run-time specialised modules (loaded per device)
// and launches all follow hipGetDevice, so for a stream of another device the
// call makes that device current and restores the caller's on return.  The
// null stream means the current device, as in HIP.
class OnStreamDevice {
 public:
  explicit OnStreamDevice(void* stream) {
    if (!stream) return;
    int dev = 0, cur = 0;
    if (hipStreamGetDevice(static_cast<hipStream_t>(stream), &dev) != hipSuccess) return;
    if (hipGetDevice(&cur) != hipSuccess || cur == dev) return;
    if (hipSetDevice(dev) == hipSuccess) prev_ = cur;
  }
  ~OnStreamDevice() {
    if (prev_ >= 0) (void)hipSetDevice(prev_);
  }
  OnStreamDevice(const OnStreamDevice&) = delete;
  OnStreamDevice& operator=(const OnStreamDevice&) = delete;

 private:
  int prev_ = -1;
};
#define RSE_ON_STREAM(stream) OnStreamDevice rse_on_stream_device_(stream)

// ------------------------------------------------------------- launching
// One fused pass: outputs (+)= rows x inputs over len_bytes, chunked so every
// launch fits the kernel-argument block (<= kMaxIn inputs, <= kMaxOut outputs).
struct Job {
  int field;
  const Rows* rows;
  const uint8_t* const* in;  // n_in pointers
  uint8_t* const* out;       // n_out pointers (may be null entries in kCheck mode)
  const uint8_t* const* cmp; // n_out pointers (check modes) or null
  size_t len_bytes;
  uint32_t mode;
  bool accumulate;
  uint32_t* mismatch;
  uint64_t stripe_stride;
  size_t n_stripes;
  bool per_stripe = false;  // CHECK modes: one mismatch word per stripe (verify_flat)
  uint32_t* done = nullptr;        // CHECK modes: completion word (run_check)
  uint32_t* done_count = nullptr;  //   and its device workgroup count
};

hipError_t launch_compare(const uint8_t* a, const uint8_t* b, size_t len, uint32_t* mismatch,
                          hipStream_t s);

hipError_t run_chunk(const Job& j, size_t o0, size_t no, size_t i0, size_t ni, uint32_t mode,
                     bool acc, hipStream_t s) {
  CodeArgs a;
  std::memset(&a, 0, sizeof a);
  bool al = (j.stripe_stride % 16u) == 0;
  for (size_t i = 0; i < ni; ++i) {
    a.in[i] = j.in[i0 + i];
    al = al && aligned16(a.in[i]);
  }
  for (size_t r = 0; r < no; ++r) {
    a.out[r] = j.out ? j.out[o0 + r] : nullptr;
    a.cmp[r] = j.cmp ? j.cmp[o0 + r] : nullptr;
    if (mode != rse::kCheck) al = al && aligned16(a.out[r]);
    if (mode != rse::kStore) al = al && aligned16(a.cmp[r]);
    for (size_t i = 0; i < ni; ++i) a.coef[r][i] = j.rows->at(o0 + r, i0 + i);
  }
  a.stripe_stride = j.stripe_stride;
  a.len = j.len_bytes;
  a.n_vec = al ? j.len_bytes / 16u : 0;
  a.mismatch = j.mismatch;
  a.n_in = (uint32_t)ni;
  a.n_out = (uint32_t)no;
  a.mode = mode;
  a.accumulate = acc ? 1u : 0u;
  a.per_stripe = j.per_stripe ? 1u : 0u;
  a.done = j.done;
  a.done_count = j.done_count;
  a.n_stripes = 0;
  hipError_t e = hipSuccess;
  for (size_t done = 0; done < j.n_stripes && e == hipSuccess;) {
    const size_t batch = std::min<size_t>(j.n_stripes - done, 0x7fffffffu);
    a.n_stripes = (uint32_t)batch;
    e = rse::launch_code(j.field, a, s);
    done += batch;
    const uint64_t adv = (uint64_t)batch * j.stripe_stride;  // next batch's stripe 0
    if (a.per_stripe) a.mismatch += batch;
    for (size_t i = 0; i < ni; ++i) a.in[i] += adv;
    for (size_t r = 0; r < no; ++r) {
      if (a.out[r]) a.out[r] += adv;
      if (a.cmp[r]) a.cmp[r] += adv;
    }
  }
  return e;
}

// Shard lengths the bit-sliced kernels code (some of): at least one 4 KiB
// chunk, or exactly 1 or 2 KiB (4 / 2 stripes per chunk, RSE_OPT_SUB_CHUNKS).
bool bitslice_len(size_t len) {
  return len >= 4096 || ((len == 1024 || len == 2048) && rse::get_option(RSE_OPT_SUB_CHUNKS));
}

int run_job(const Job& j, hipStream_t s);

// The bytes of every shard past `done` (a wide launch coded whole chunks up
// to there); the wide launch stays the kernel rse_last_kernel reports.
int run_rest(const Job& j, uint64_t done, hipStream_t s) {
  const size_t n_out = j.rows->n_out, n_in = j.rows->n_in;
  std::vector<const uint8_t*> in(j.in, j.in + n_in);
  std::vector<uint8_t*> out(n_out, nullptr);
  std::vector<const uint8_t*> cmp(n_out, nullptr);
  for (auto& q : in) q += done;
  for (size_t r = 0; r < n_out; ++r) {
    if (j.out && j.out[r]) out[r] = j.out[r] + done;
    if (j.cmp && j.cmp[r]) cmp[r] = j.cmp[r] + done;
  }
  Job rest = j;
  rest.in = in.data();
  rest.out = j.out ? out.data() : nullptr;
  rest.cmp = j.cmp ? cmp.data() : nullptr;
  rest.len_bytes = j.len_bytes - done;
  const std::string wide_kernel = rse::last_kernel();  // the launch to report
  const int rc = run_job(rest, s);
  rse::note_kernel("%s", wide_kernel.c_str());
  return rc;
}

// Executes a Job; `scratch` provides per-output buffers when a CHECK job must
// be split over several input chunks (full sums are needed before comparing).
int run_job(const Job& j, hipStream_t s) {
  const size_t n_out = j.rows->n_out, n_in = j.rows->n_in;
  if (n_out == 0 || j.len_bytes == 0) return RSE_OK;
  // GF(2^16) coefficients all in the GF(2^8) subfield (the low-level entry
  // points; codecs already arrive as kfield 8): the GF(2^8) pass, byte by
  // byte (rse_codec::kfield)
  if (j.field == RSE_FIELD_GF16 && rse::get_option(RSE_OPT_SUBFIELD)) {
    bool sub = true;
    for (size_t q = 0; q < j.rows->c.size() && sub; ++q) sub = j.rows->c[q] < 256;
    if (sub) {
      Job g = j;
      g.field = RSE_FIELD_GF8;
      return run_job(g, s);
    }
  }
  // GF(2^8) k = p = 16 / 32 / 64: the codec's parity rows (encode, verify; also
  // their own inverse, so all data shards rebuilt from the parity) on the
  // additive-FFT kernels (rse_fft.hip): every whole 2 KiB column (1 KiB shards: all), the
  // rest of every shard below
  if (!j.accumulate && j.field == RSE_FIELD_GF8 && n_in == n_out && j.stripe_stride % 16u == 0 &&
      rse::get_option(RSE_OPT_BITSLICE) && j.n_stripes <= 0xffffffffu &&
      rse::fft_applies(8, (uint32_t)n_in, (uint32_t)n_out, j.rows->c.data())) {
    bool al = true;
    for (size_t i = 0; i < n_in; ++i) al = al && aligned16(j.in[i]);
    for (size_t r = 0; r < n_out; ++r) {
      if (j.mode != rse::kCheck) al = al && aligned16(j.out[r]);
      if (j.mode != rse::kStore) al = al && aligned16(j.cmp[r]);
    }
    uint64_t done = 0;
    if (al)
      RSE_HIP(rse::launch_fft(j.field, (uint32_t)n_in, (uint32_t)n_out, j.rows->c.data(), j.in,
                              j.out, j.cmp, j.len_bytes, j.stripe_stride, (uint32_t)j.n_stripes,
                              j.mode, j.mismatch, j.per_stripe, s, &done));
    if (done) return done == j.len_bytes ? RSE_OK : run_rest(j, done, s);
  }
  // a wide codec's (or pattern's) rows with their one-module kernel built:
  // every whole 4 KiB chunk in one launch (each input read once, each output
  // written once), the rest of every shard below
  if (!j.accumulate && bitslice_len(j.len_bytes) && j.stripe_stride % 16u == 0 &&
      rse::get_option(RSE_OPT_BITSLICE) && rse::wide_eligible((uint32_t)n_in, (uint32_t)n_out) &&
      j.n_stripes <= 0xffffffffu) {
    bool al = true;
    for (size_t i = 0; i < n_in; ++i) al = al && aligned16(j.in[i]);
    for (size_t r = 0; r < n_out; ++r) {
      if (j.mode != rse::kCheck) al = al && aligned16(j.out[r]);
      if (j.mode != rse::kStore) al = al && aligned16(j.cmp[r]);
    }
    uint64_t done = 0;
    if (al)
      RSE_HIP(rse::launch_wide(j.field, (uint32_t)n_in, (uint32_t)n_out, j.rows->c.data(), j.in,
                               j.out, j.cmp, j.len_bytes, j.stripe_stride, (uint32_t)j.n_stripes,
                               j.mode, j.mismatch, j.per_stripe, s, &done));
    if (done) return done == j.len_bytes ? RSE_OK : run_rest(j, done, s);
  }
  // too wide for one module (GF(2^16) past 256 shards): the chain of wide
  // modules over input blocks, once all of them are built (want_bitslice)
  if (j.mode == rse::kStore && !j.accumulate && bitslice_len(j.len_bytes) &&
      j.stripe_stride % 16u == 0 && rse::get_option(RSE_OPT_BITSLICE) &&
      j.n_stripes <= 0xffffffffu && rse::wide_blocks_plan((uint32_t)n_in, (uint32_t)n_out, nullptr)) {
    bool al = true;
    for (size_t i = 0; i < n_in; ++i) al = al && aligned16(j.in[i]);
    for (size_t r = 0; r < n_out; ++r) al = al && aligned16(j.out[r]);
    uint64_t done = 0;
    if (al)
      RSE_HIP(rse::launch_wide_blocks(j.field, (uint32_t)n_in, (uint32_t)n_out, j.rows->c.data(),
                                      j.in, j.out, j.len_bytes, j.stripe_stride,
                                      (uint32_t)j.n_stripes, s, &done));
    if (done) return done == j.len_bytes ? RSE_OK : run_rest(j, done, s);
  }
  const bool single_in = n_in <= (size_t)kMaxIn;
  if (j.mode == rse::kStore || single_in) {
    // a wide codec's parity rows whose bit-sliced blocks are built (see
    // want_bitslice): launch them block by block, 8 outputs at a time
    size_t step = kMaxOut;
    if ((n_in > (size_t)kMaxIn || n_out > rse::kJitMaxOut) && j.len_bytes >= 4096 &&
        rse::get_option(5) != 0 &&
        rse::jit_blocks_status(j.field, (uint32_t)n_in, (uint32_t)n_out, j.rows->c.data(),
                               false) == 2)
      step = rse::kJitMaxOut;
    for (size_t o0 = 0; o0 < n_out; o0 += step) {
      const size_t no = std::min<size_t>(step, n_out - o0);
      for (size_t i0 = 0; i0 < n_in; i0 += kMaxIn) {
        const size_t ni = std::min<size_t>(kMaxIn, n_in - i0);
        RSE_HIP(run_chunk(j, o0, no, i0, ni, j.mode, j.accumulate || i0 > 0, s));
      }
    }
    return RSE_OK;
  }
  // CHECK modes with > kMaxIn inputs: materialise the sums, then compare.
  std::vector<uint8_t*> dst(n_out, nullptr);
  std::vector<void*> owned;
  const size_t span = (j.n_stripes - 1) * j.stripe_stride + j.len_bytes;
  for (size_t r = 0; r < n_out; ++r) {
    if (j.mode == rse::kCheckStore) {
      dst[r] = j.out[r];
    } else {
      void* p = nullptr;
      hipError_t e = hipMallocAsync(&p, span, s);
      if (e != hipSuccess) {
        for (void* q : owned) (void)hipFreeAsync(q, s);
        return dev_fail(e);
      }
      owned.push_back(p);
      dst[r] = static_cast<uint8_t*>(p);
    }
  }
  Job st = j;
  st.out = dst.data();
  st.cmp = nullptr;
  st.mode = rse::kStore;
  int rc = run_job(st, s);
  for (size_t r = 0; rc == RSE_OK && r < n_out; ++r)
    for (size_t sidx = 0; sidx < j.n_stripes && rc == RSE_OK; ++sidx) {
      const size_t off = sidx * j.stripe_stride;
      hipError_t e = launch_compare(dst[r] + off, j.cmp[r] + off, j.len_bytes,
                                    j.mismatch + (j.per_stripe ? sidx : 0), s);
      if (e != hipSuccess) rc = dev_fail(e);
    }
  for (void* q : owned) (void)hipFreeAsync(q, s);
  return rc;
}

__global__ void compare_kernel(const uint8_t* a, const uint8_t* b, size_t len, uint32_t* mm) {
  bool diff = false;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < len;
       i += (size_t)gridDim.x * blockDim.x)
    diff |= a[i] != b[i];
  if (diff) *reinterpret_cast<volatile uint32_t*>(mm) = 1u;  // as rse_device.hpp flag_mismatch
}

hipError_t launch_compare(const uint8_t* a, const uint8_t* b, size_t len, uint32_t* mismatch,
                          hipStream_t s) {
  size_t blocks = std::min<size_t>((len + 255) / 256, 4096);
  hipLaunchKernelGGL(compare_kernel, dim3((unsigned)blocks), dim3(256), 0, s, a, b, len, mismatch);
  return hipGetLastError();
}

// ------------------------------------------------------------- scratch pool
// The device resources of the synchronous calls, kept between calls because
// creating them per call costs milliseconds (a one-stripe 10+4 x 16 MiB host
// encode ran at 21 GB/s against 54 for eight before they were kept):
//  * verify verdict words, in pinned host memory mapped into the device
//    (fine-grained, coherent): the check kernels store 1 into them directly
//    (rse_device.hpp flag_mismatch), so a verify is one launch and one
//    synchronisation -- no memset or D2H copy of the verdict;
//  * a library-owned stream for calls that must wait for their own work only
//    (rse_gal_mul: the reference kernel returns when done);
//  * the host pipeline's streams, events and device ring.
// A call leases one Scratch of its device from a process-wide pool and
// returns it idle when it has synchronised, so a Scratch is never shared by
// two calls at once.  The pool keeps at most kIdleScratch idle ones per device
// and destroys the surplus on return: threads that come and go (a service's
// or Python's thread pool) leave nothing behind, and a burst of N concurrent
// calls holds N leases only while it lasts.  Rings above kPipeRingKeep
// (wide codecs, big chunks) are never kept: such a call allocates its own.
// The pool itself is never destroyed (a static destructor could run after
// the HIP runtime has shut down); idle resources end with the process.
constexpr int kMaxDev = 64;
constexpr size_t kIdleScratch = 4;
constexpr size_t kPipeRingKeep = size_t(512) << 20;

struct Scratch {
  int dev = 0;
  uint32_t* wh = nullptr;  // verdict words, host view
  uint32_t* wd = nullptr;  // device view of the same words
  size_t words = 0;
  hipStream_t own = nullptr;
  int nh = 0, ring = 0;  // host pipeline: nh H2D streams + kernel + D2H
  int qmode = -1;        // ... created under this RSE_OPT_HOST_QUEUES
  std::vector<hipStream_t> st;
  std::vector<hipEvent_t> h2d, coded, d2h;
  hipEvent_t start = nullptr;
  hipEvent_t done = nullptr;  // run_check's completion event (RSE_OPT_SYNC_EVENT)
  uint32_t* count = nullptr;  // run_check's device workgroup count (signal_done), zero when idle
  uint8_t* dbuf = nullptr;
  size_t dbytes = 0;
  // rse_reconstruct_batch's device workspace (flags, scan words, per-stripe
  // descriptors), kept between calls up to kPlanKeep bytes
  uint8_t* pbuf = nullptr;
  size_t pbytes = 0;
};
constexpr size_t kPlanKeep = size_t(128) << 20;

// The lease's planner workspace of at least `bytes` (kept when at most
// kPlanKeep; a larger one is a stream-ordered allocation on `st` for the
// call: *owned is set and the caller frees it with hipFreeAsync).
hipError_t lease_plan(Scratch* s, size_t bytes, hipStream_t st, uint8_t** out, bool* owned) {
  *owned = false;
  if (s->pbytes >= bytes) {
    *out = s->pbuf;
    return hipSuccess;
  }
  if (bytes > kPlanKeep) {
    *owned = true;
    return hipMallocAsync(reinterpret_cast<void**>(out), bytes, st);
  }
  if (s->pbuf) (void)hipFree(s->pbuf);  // idle: the previous call synchronised
  s->pbuf = nullptr;
  s->pbytes = 0;
  const hipError_t e = hipMalloc(reinterpret_cast<void**>(&s->pbuf), bytes);
  if (e != hipSuccess) return e;
  s->pbytes = bytes;
  *out = s->pbuf;
  return hipSuccess;
}

void drop_pipe_streams(Scratch& s) {
  for (auto& q : s.st) (void)hipStreamDestroy(q);
  for (auto* ev : {&s.h2d, &s.coded, &s.d2h})
    for (auto& q : *ev) (void)hipEventDestroy(q);
  s.st.clear();
  s.h2d.clear();
  s.coded.clear();
  s.d2h.clear();
  s.nh = s.ring = 0;
}

void destroy_scratch(Scratch* s) {  // idle: its last call synchronised
  drop_pipe_streams(*s);
  if (s->start) (void)hipEventDestroy(s->start);
  if (s->done) (void)hipEventDestroy(s->done);
  if (s->own) (void)hipStreamDestroy(s->own);
  if (s->dbuf) (void)hipFree(s->dbuf);
  if (s->pbuf) (void)hipFree(s->pbuf);
  if (s->count) (void)hipFree(s->count);
  if (s->wh) (void)hipHostFree(s->wh);
  delete s;
}

struct ScratchPool {
  std::mutex mu;
  std::vector<Scratch*> idle[kMaxDev];
  std::atomic<int64_t> live{0};  // Scratch objects in existence (tests: RSE_OPT_SCRATCH_LIVE)
};
ScratchPool& scratch_pool() {
  static ScratchPool& p = *new ScratchPool;
  return p;
}

// One Scratch of the current device for the duration of a call.
class Lease {
 public:
  Lease() = default;
  Lease(const Lease&) = delete;
  Lease& operator=(const Lease&) = delete;
  ~Lease() {
    if (!s_) return;
    ScratchPool& pool = scratch_pool();
    {
      std::lock_guard<std::mutex> g(pool.mu);
      auto& idle = pool.idle[s_->dev];
      if (idle.size() < kIdleScratch) {
        idle.push_back(s_);
        return;
      }
    }
    --pool.live;
    destroy_scratch(s_);
  }
  hipError_t acquire() {
    int dev = 0;
    hipError_t e = hipGetDevice(&dev);
    if (e != hipSuccess) return e;
    if (dev < 0 || dev >= kMaxDev) return hipErrorInvalidDevice;
    ScratchPool& pool = scratch_pool();
    {
      std::lock_guard<std::mutex> g(pool.mu);
      auto& idle = pool.idle[dev];
      if (!idle.empty()) {
        s_ = idle.back();
        idle.pop_back();
        return hipSuccess;
      }
    }
    s_ = new Scratch;
    s_->dev = dev;
    ++pool.live;
    return hipSuccess;
  }
  Scratch* operator->() const { return s_; }
  Scratch* get() const { return s_; }

 private:
  Scratch* s_ = nullptr;
};

hipError_t lease_words(Scratch* s, size_t words) {
  if (s->words >= words) return hipSuccess;
  const size_t n = std::max<size_t>(words, 256);
  uint32_t *h = nullptr, *d = nullptr;
  hipError_t e = hipHostMalloc(reinterpret_cast<void**>(&h), n * sizeof(uint32_t),
                               hipHostMallocMapped | hipHostMallocCoherent);
  if (e != hipSuccess) return e;
  e = hipHostGetDevicePointer(reinterpret_cast<void**>(&d), h, 0);
  if (e != hipSuccess) {
    (void)hipHostFree(h);
    return e;
  }
  if (s->wh) (void)hipHostFree(s->wh);  // idle: the previous call has synchronised
  s->wh = h;
  s->wd = d;
  s->words = n;
  return hipSuccess;
}

// The library stream of the synchronous slice hooks: a blocking stream, so its
// work is ordered after what the caller queued on the null stream (as the
// hooks' null-stream launches were before), while the call still waits for
// this stream only.
hipError_t lease_own_stream(Scratch* s, hipStream_t* out) {
  if (!s->own) {
    const hipError_t e = hipStreamCreateWithFlags(&s->own, hipStreamDefault);
    if (e != hipSuccess) return e;
  }
  *out = s->own;
  return hipSuccess;
}

// A kept device ring of at least dbytes, if that is at most kPipeRingKeep
// (otherwise the ring stays as it is and the caller allocates its own).
hipError_t lease_ring(Scratch* r, size_t dbytes) {
  if (r->dbytes < dbytes && dbytes <= kPipeRingKeep) {
    if (r->dbuf) (void)hipFree(r->dbuf);  // idle: the previous call synchronised
    r->dbuf = nullptr;
    r->dbytes = 0;
    const hipError_t e = hipMalloc(reinterpret_cast<void**>(&r->dbuf), dbytes);
    if (e != hipSuccess) return e;
    r->dbytes = dbytes;
  }
  return hipSuccess;
}

// One stream of the host pipeline.  HIP maps streams onto at most
// GPU_MAX_HW_QUEUES (4) hardware queues per priority, least-used first, so
// once the process holds a few streams (torch's, the caller's, other leases')
// the pipeline's H2D and D2H streams can share one queue.  Commands of one
// queue start in order, so the D2H copy that waits for a chunk's kernel then
// holds up the next chunks' H2D copies behind it and the duplex is lost (the
// bench's pinned-host leg read 41.6 against 76.1 GB/s for the same call,
// VERDICT r05; tools/queue_probe.py: 63 against 73-76 GB/s by where the
// streams land).  RSE_OPT_HOST_QUEUES 1 (default): the D2H stream at high
// priority, a queue pool of its own (rse::side_priority_stream); 0: plain
// streams.
hipError_t pipe_stream(int qmode, bool d2h, hipStream_t* q) {
  if (qmode && d2h) return rse::side_priority_stream(true, q);
  return hipStreamCreateWithFlags(q, hipStreamNonBlocking);
}

// The host pipeline's streams and events for (nh, ring), and a kept ring of
// dbytes if that is at most kPipeRingKeep.
hipError_t lease_pipe(Scratch* r, int nh, int ring, size_t dbytes) {
  hipError_t e = hipSuccess;
  const int qmode = (int)rse::get_option(RSE_OPT_HOST_QUEUES);
  if (r->nh != nh || r->ring != ring || r->qmode != qmode) {
    drop_pipe_streams(*r);
    for (int i = 0; i < nh + 2 && e == hipSuccess; ++i) {
      hipStream_t q = nullptr;
      e = pipe_stream(qmode, i == nh + 1, &q);
      if (e == hipSuccess) r->st.push_back(q);
    }
    for (auto* ev : {&r->h2d, &r->coded, &r->d2h})
      for (int i = 0; i < ring && e == hipSuccess; ++i) {
        hipEvent_t q = nullptr;
        e = hipEventCreateWithFlags(&q, hipEventDisableTiming);
        if (e == hipSuccess) ev->push_back(q);
      }
    if (e != hipSuccess) {
      drop_pipe_streams(*r);
      return e;
    }
    r->nh = nh;
    r->ring = ring;
    r->qmode = qmode;
  }
  if (!r->start) {
    e = hipEventCreateWithFlags(&r->start, hipEventDisableTiming);
    if (e != hipSuccess) return e;
  }
  return lease_ring(r, dbytes);
}

// Runs `j` in a check mode and returns the verdict (synchronises the stream):
// ok[0], or ok[s] for every stripe when j.per_stripe.
int run_check(Job j, hipStream_t s, int* ok) {
  const size_t words = j.per_stripe ? j.n_stripes : 1;
  Lease lease;
  RSE_HIP(lease.acquire());
  RSE_HIP(lease_words(lease.get(), words + 1));  // + the completion word
  uint32_t* wh = lease->wh;
  std::memset(wh, 0, (words + 1) * sizeof(uint32_t));  // leased: no kernel uses them now
  j.mismatch = lease->wd;
  // RSE_OPT_SPIN_WAIT: offer the kernel the completion word; launch_bitslice
  // arms it when one compiled check-kernel launch is the whole verify
  if (!j.per_stripe && rse::get_option(31)) {
    if (!lease->count) {
      RSE_HIP(hipMalloc(reinterpret_cast<void**>(&lease->count), sizeof(uint32_t)));
      RSE_HIP(hipMemset(lease->count, 0, sizeof(uint32_t)));
    }
    j.done = lease->wd + words;
    j.done_count = lease->count;
  }
  rse::t_done_armed = false;
  int rc = run_job(j, s);
  const bool armed = rse::t_done_armed;
  // kernels already queued may still store into the words: drain them before
  // the lease returns them to the pool.  Armed: the kernel's last workgroup
  // stores the completion word after every verdict store (rse_device.hpp
  // signal_done); poll it, asking the stream now and then (a launch that
  // failed, or other work queued behind ours, ends the wait the usual way).
  // RSE_OPT_SYNC_EVENT 1: wait on an event recorded after them instead of on
  // the whole stream (A/B)
  hipError_t se = hipSuccess;
  if (armed && rc == RSE_OK) {
    const volatile uint32_t* dw = wh + words;
    for (uint32_t n = 1; *dw == 0; ++n) {
      __builtin_ia32_pause();
      if ((n & 1023u) == 0 && (se = hipStreamQuery(s)) != hipErrorNotReady) break;
    }
    if (se == hipErrorNotReady) se = hipSuccess;
    if (se == hipSuccess && *dw == 0) {  // finished without signalling: rezero the count
      se = hipMemsetAsync(lease->count, 0, sizeof(uint32_t), s);
      if (se == hipSuccess) se = hipStreamSynchronize(s);
    }
  } else if (rse::get_option(30)) {
    if (!lease->done) se = hipEventCreateWithFlags(&lease->done, hipEventDisableTiming);
    if (se == hipSuccess) se = hipEventRecord(lease->done, s);
    if (se == hipSuccess) se = hipEventSynchronize(lease->done);
    if (se != hipSuccess) (void)hipStreamSynchronize(s);
  } else {
    se = hipStreamSynchronize(s);
  }
  if (rc != RSE_OK) return rc;
  RSE_HIP(se);
  for (size_t i = 0; i < words; ++i)
    ok[i] = reinterpret_cast<volatile uint32_t*>(wh)[i] == 0 ? 1 : 0;
  return RSE_OK;
}

Rows parity_rows(const rse_codec* c) {  // core.rs:420-428
  Rows r;
  r.n_out = c->p;
  r.n_in = c->k;
  r.c.resize(c->p * c->k);
  for (size_t i = 0; i < c->p; ++i)
    for (size_t j = 0; j < c->k; ++j) r.c[i * c->k + j] = c->mat(c->k + i, j);
  return r;
}

// Byte offset of the planner tables in a codec's plan constants.
size_t plan_tab_off(const rse_codec* c) { return (c->p * c->k * 2 + 255) & ~size_t(255); }

// The codec's plan constants on device `dev` (rse_codec::plan_dev): made once
// per device, with a synchronous copy (the first batched reconstruct there
// pays it); two threads racing keep one copy and free the other.
hipError_t plan_consts(const rse_codec* c, int dev, const uint8_t** out) {
  if (dev < 0 || dev >= rse_codec::kDevs) return hipErrorInvalidDevice;
  if (uint8_t* q = c->plan_dev[dev].load(std::memory_order_acquire)) {
    *out = q;
    return hipSuccess;
  }
  const Rows r = parity_rows(c);
  const size_t off = plan_tab_off(c);
  std::vector<uint8_t> h(off + rse::kPlanTabBytes, 0);
  std::memcpy(h.data(), r.c.data(), r.c.size() * 2);
  rse::plan_tables(h.data() + off);
  uint8_t* q = nullptr;
  hipError_t e = hipMalloc(reinterpret_cast<void**>(&q), h.size());
  if (e == hipSuccess) e = hipMemcpy(q, h.data(), h.size(), hipMemcpyHostToDevice);
  if (e != hipSuccess) {
    if (q) (void)hipFree(q);
    return e;
  }
  uint8_t* expect = nullptr;
  if (!c->plan_dev[dev].compare_exchange_strong(expect, q, std::memory_order_acq_rel)) {
    (void)hipFree(q);
    q = expect;
  }
  *out = q;
  return hipSuccess;
}

// Codecs without compiled-in bit-sliced kernels get them built for their
// parity rows at run time (rse_jit.cpp: hiprtc on a background thread, host
// CPU only).  The first call that codes at least one whole bit-sliced chunk
// (4 KiB: the per-wave chunks) requests it, so codecs only ever used on short
// shards never pay for a build.  Wide codecs (k > 32 or p > 8) get one
// module per 8 x 32 block of their parity rows instead (store or accumulate
// mode; run_job launches them block by block), requested once the codec has
// coded 1 GiB of shards on the table kernels (at once under RSE_OPT_JIT 2, or
// `now`: kernel_kind with wait): each block is seconds of hiprtc, worth it
// for a codec that streams data, not for one used a few times.
constexpr uint64_t kWideJitBytes = 1ull << 30;
void want_bitslice(const rse_codec* c, size_t len_bytes, bool now = false, size_t n_stripes = 1) {
  if (!bitslice_len(len_bytes) || c->jit_requested.load(std::memory_order_relaxed)) return;
  const bool wide = c->k > (size_t)kMaxIn || c->p > rse::kJitMaxOut ||
                    rse::wide_eligible((uint32_t)c->k, (uint32_t)c->p);
  if (wide && !now && rse::get_option(RSE_OPT_JIT) < 2) {
    const uint64_t b = (uint64_t)len_bytes * c->total * n_stripes;
    if (c->wide_bytes.fetch_add(b, std::memory_order_relaxed) + b < kWideJitBytes) return;
  }
  c->jit_requested.store(true, std::memory_order_relaxed);
  if (rse::bitslice_compiled(c->kfield, (uint32_t)c->k, (uint32_t)c->p)) return;
  const Rows rows = parity_rows(c);
  // k = p = 16 / 32 / 64: the compiled additive-FFT kernels (rse_fft.hip)
  if (rse::fft_applies(c->kfield, (uint32_t)c->k, (uint32_t)c->p, rows.c.data())) return;
  if (wide && rse::wide_eligible((uint32_t)c->k, (uint32_t)c->p))
    rse::jit_register_wide(c->kfield, (uint32_t)c->k, (uint32_t)c->p, rows.c.data(), false);
  else if (wide)
    rse::jit_register_blocks(c->kfield, (uint32_t)c->k, (uint32_t)c->p, rows.c.data(), false);
  else
    rse::jit_register(c->kfield, (uint32_t)c->k, (uint32_t)c->p, rows.c.data(), rse::kJitCodec);
}

Rows single_column(const rse_codec* c, size_t i_data) {  // code_single_slice, core.rs:492-509
  Rows r;
  r.n_out = c->p;
  r.n_in = 1;
  r.c.resize(c->p);
  for (size_t i = 0; i < c->p; ++i) r.c[i] = c->mat(c->k + i, i_data);
  return r;
}

// core.rs:697-731: k x k inverse of the valid rows, cached by invalid indices.
// *uses: how many reconstructs (this one included) used the pattern while cached.
int decode_matrix(const rse_codec* c, const std::vector<size_t>& valid,
                  const std::vector<size_t>& invalid, std::vector<uint16_t>& out,
                  uint32_t* uses) {
  {
    std::lock_guard<std::mutex> g(c->mu);
    auto it = c->index.find(invalid);
    if (it != c->index.end()) {
      c->lru.splice(c->lru.begin(), c->lru, it->second);
      out = it->second->second.dec;
      *uses = ++it->second->second.uses;
      return RSE_OK;
    }
  }
  *uses = 1;
  const size_t k = c->k;
  bool ok;
  if (c->kfield == 16) {
    rse::Matrix<rse::Gf16Field> sub(k, k), inv;
    for (size_t r = 0; r < k; ++r)
      for (size_t j = 0; j < k; ++j) sub.at(r, j) = c->m16.at(valid[r], j);
    ok = sub.invert(inv);
    out = inv.d;
  } else {  // GF(2^8), or a GF(2^16) codec in the subfield (kfield): the same inverse
    rse::Matrix<rse::Gf8Field> sub(k, k), inv;
    for (size_t r = 0; r < k; ++r)
      for (size_t j = 0; j < k; ++j) sub.at(r, j) = c->mat(valid[r], j);
    ok = sub.invert(inv);
    out = inv.d;
  }
  if (!ok) return RSE_ERR_SINGULAR_MATRIX;  // unreachable for an MDS code
  std::lock_guard<std::mutex> g(c->mu);
  if (c->index.find(invalid) == c->index.end()) {
    c->lru.emplace_front(invalid, rse_codec::Cached{out, 1});
    c->index[invalid] = c->lru.begin();
    if (c->lru.size() > kCacheCapacity) {
      c->index.erase(c->lru.back().first);
      c->lru.pop_back();
    }
  }
  return RSE_OK;
}

// Plan of a reconstruct: the k surviving inputs and the combined rows that
// produce every missing output in one pass (core.rs:733-923).
struct ReconPlan {
  std::vector<const uint8_t*> in;  // sub_shards (core.rs:792)
  std::vector<uint8_t*> out;       // missing data shards, then missing parity shards
  Rows rows;
  size_t len = 0;  // elements
  bool nothing_to_do = false;
  uint32_t pattern_uses = 0;  // decode_matrix *uses
};

int plan_reconstruct(const rse_codec* c, void* const* shards, const size_t* lens,
                     const uint8_t* present, size_t n, bool data_only, ReconPlan& plan) {
  int rc = check_count(n, c->total, RSE_TOO_FEW_SHARDS, RSE_TOO_MANY_SHARDS);
  if (rc) return rc;
  if (!lens || !present) return RSE_ERR_INVALID_ARGUMENT;
  const size_t k = c->k;
  size_t number_present = 0, shard_len = 0;
  bool have = false;
  for (size_t i = 0; i < n; ++i) {  // core.rs:747-761
    if (!present[i]) continue;
    if (lens[i] == 0) return RSE_EMPTY_SHARD;
    ++number_present;
    if (have && lens[i] != shard_len) return RSE_INCORRECT_SHARD_SIZE;
    shard_len = lens[i];
    have = true;
  }
  if (number_present == c->total) {  // core.rs:763-767
    plan.nothing_to_do = true;
    return RSE_OK;
  }
  if (number_present < k) return RSE_TOO_FEW_SHARDS_PRESENT;  // core.rs:770-772
  if (!shards) return RSE_ERR_INVALID_ARGUMENT;

  std::vector<size_t> valid, invalid, miss_data, miss_parity;
  for (size_t row = 0; row < n; ++row) {  // core.rs:801-841
    if (row >= k && data_only) {
      if (present[row]) {
        if (valid.size() < k) valid.push_back(row);
      } else {
        invalid.push_back(row);
      }
      continue;
    }
    if (lens[row] != shard_len) return RSE_INCORRECT_SHARD_SIZE;  // lib.rs:185-199
    if (present[row]) {
      if (valid.size() < k) valid.push_back(row);
    } else {
      if (!shards[row]) return RSE_ERR_INVALID_ARGUMENT;
      (row < k ? miss_data : miss_parity).push_back(row);
      invalid.push_back(row);
    }
  }
  for (size_t v : valid)
    if (!shards[v]) return RSE_ERR_INVALID_ARGUMENT;

  std::vector<uint16_t> dec;
  rc = decode_matrix(c, valid, invalid, dec, &plan.pattern_uses);
  if (rc) return rc;

  // Coefficients that rebuild data shard j from the k valid inputs:
  //   present data j  -> unit vector at its position among the valid inputs
  //   missing data j  -> row j of the decode matrix (core.rs:853-861)
  auto data_row = [&](size_t j, std::vector<uint16_t>& row) {
    row.assign(k, 0);
    auto it = std::find(valid.begin(), valid.end(), j);
    if (it != valid.end()) row[it - valid.begin()] = 1;
    else
      for (size_t i = 0; i < k; ++i) row[i] = dec[j * k + i];
  };
  plan.rows.n_in = k;
  plan.rows.n_out = miss_data.size() + (data_only ? 0 : miss_parity.size());
  plan.rows.c.assign(plan.rows.n_out * k, 0);
  std::vector<uint16_t> row;
  size_t o = 0;
  for (size_t j : miss_data) {
    data_row(j, row);
    std::copy(row.begin(), row.end(), plan.rows.c.begin() + o * k);
    plan.out.push_back(static_cast<uint8_t*>(shards[j]));
    ++o;
  }
  if (!data_only) {
    // missing parity r = sum_j P[r][j] * data_j  (core.rs:872-918), with every
    // data_j expanded over the valid inputs: one combined row per parity shard.
    for (size_t pr : miss_parity) {
      uint16_t* dst = &plan.rows.c[o * k];
      for (size_t j = 0; j < k; ++j) {
        const uint16_t pj = c->mat(pr, j);
        if (!pj) continue;
        data_row(j, row);
        for (size_t i = 0; i < k; ++i) dst[i] ^= c->mul(pj, row[i]);
      }
      plan.out.push_back(static_cast<uint8_t*>(shards[pr]));
      ++o;
    }
  }
  for (size_t v : valid) plan.in.push_back(static_cast<const uint8_t*>(shards[v]));
  plan.len = shard_len;
  return RSE_OK;
}

// Bit-sliced syndrome reconstruct (rse_kernels.hpp BsReconArgs) for codecs
// whose parity rows are compiled into rse_bitslice.hip, over the whole 16 KiB
// chunks of every shard; *done = bytes per shard it coded (0 if it does not
// apply).  Same outputs as the composed-row plan: missing data, and missing
// parity unless data_only.  The e present parity rows used for syndromes are
// the first e present ones -- exactly the parity rows among the reference's
// `valid` set (core.rs:801-841) -- and P[R][S] is invertible for any choice
// (any k rows of the systematic MDS matrix are independent), so the result
// is the reference's.  Shards are already validated by plan_reconstruct.
int bitslice_reconstruct(const rse_codec* c, const uint8_t* const* shards, const uint8_t* present,
                         bool data_only, size_t len_bytes, uint64_t stripe_stride,
                         size_t n_stripes, hipStream_t s, size_t* done) {
  *done = 0;
  const size_t k = c->k, p = c->p;
  want_bitslice(c, len_bytes);
  if (k > (size_t)kMaxIn || p > (size_t)kMaxOut || len_bytes < 4096 || stripe_stride % 16u ||
      !rse::get_option(RSE_OPT_BITSLICE))
    return RSE_OK;
  rse::BsReconArgs a;
  std::memset(&a, 0, sizeof a);
  std::vector<size_t> S, R, M;
  for (size_t d = 0; d < k; ++d) {
    if (present[d]) {
      a.present |= 1u << d;
      a.data[d] = shards[d];
    } else {
      S.push_back(d);
    }
  }
  for (size_t r = 0; r < p; ++r) {
    if (present[k + r]) {
      if (R.size() < S.size()) R.push_back(r);
    } else if (!data_only) {
      M.push_back(r);
    }
  }
  const size_t e = S.size();
  if (e + M.size() == 0 || R.size() != e) return RSE_OK;
  for (size_t d = 0; d < k; ++d)
    if (present[d] && !aligned16(shards[d])) return RSE_OK;
  for (size_t r : R)
    if (!aligned16(shards[k + r])) return RSE_OK;
  for (size_t j : S)
    if (!aligned16(shards[j])) return RSE_OK;
  for (size_t r : M)
    if (!aligned16(shards[k + r])) return RSE_OK;
  // A = P[R][S] and its inverse (Gauss-Jordan; A is invertible, see above)
  std::vector<uint16_t> w(e * 2 * e, 0);
  for (size_t t = 0; t < e; ++t) {
    for (size_t u = 0; u < e; ++u) w[t * 2 * e + u] = c->mat(k + R[t], S[u]);
    w[t * 2 * e + e + t] = 1;
  }
  for (size_t col = 0; col < e; ++col) {
    size_t piv = col;
    while (piv < e && w[piv * 2 * e + col] == 0) ++piv;
    if (piv == e) return RSE_OK;  // cannot happen for this code; stay on the table path
    for (size_t x = 0; x < 2 * e; ++x) std::swap(w[col * 2 * e + x], w[piv * 2 * e + x]);
    const uint16_t sc = c->inv(w[col * 2 * e + col]);
    for (size_t x = 0; x < 2 * e; ++x) w[col * 2 * e + x] = c->mul(sc, w[col * 2 * e + x]);
    for (size_t r = 0; r < e; ++r) {
      const uint16_t f = w[r * 2 * e + col];
      if (r == col || !f) continue;
      for (size_t x = 0; x < 2 * e; ++x) w[r * 2 * e + x] ^= c->mul(f, w[col * 2 * e + x]);
    }
  }
  auto ainv = [&](size_t u, size_t t) { return w[u * 2 * e + e + t]; };
  uint32_t o = 0;
  for (size_t u = 0; u < e; ++u, ++o) {  // missing data S[u] = sum_t Ainv[u][t] s_t
    a.out[o] = const_cast<uint8_t*>(shards[S[u]]);
    a.out_sigma[o] = -1;
    for (size_t t = 0; t < e; ++t) a.w[o][R[t]] = ainv(u, t);
  }
  for (size_t r : M) {  // missing parity r = sigma_r ^ sum_t (P[r][S] Ainv)[t] s_t
    a.out[o] = const_cast<uint8_t*>(shards[k + r]);
    a.out_sigma[o] = (int32_t)r;
    for (size_t t = 0; t < e; ++t) {
      uint16_t v = 0;
      for (size_t u = 0; u < e; ++u) v ^= c->mul(c->mat(k + r, S[u]), ainv(u, t));
      a.w[o][R[t]] = v;
    }
    ++o;
  }
  a.n_out = o;
  for (size_t t = 0; t < e; ++t) {
    a.synd |= 1u << R[t];
    a.sigma |= 1u << R[t];
    a.par[R[t]] = shards[k + R[t]];
  }
  for (size_t r : M) a.sigma |= 1u << r;
  rse::set_horner_masks(a, c->kfield);
  a.stripe_stride = stripe_stride;
  std::vector<uint16_t> rows(p * k);
  for (size_t r = 0; r < p; ++r)
    for (size_t j = 0; j < k; ++j) rows[r * k + j] = c->mat(k + r, j);
  uint64_t coded = 0;  // bytes of every shard the kernels code (the same for every batch)
  for (size_t s0 = 0; s0 < n_stripes; s0 += 0x7fffffffu) {
    rse::BsReconArgs b = a;
    const size_t cnt = std::min<size_t>(n_stripes - s0, 0x7fffffffu);
    const uint64_t adv = (uint64_t)s0 * stripe_stride;
    b.n_stripes = (uint32_t)cnt;
    for (size_t d = 0; d < k; ++d)
      if (b.data[d]) b.data[d] += adv;
    for (size_t r = 0; r < p; ++r)
      if (b.par[r]) b.par[r] += adv;
    for (uint32_t q = 0; q < b.n_out; ++q) b.out[q] += adv;
    RSE_HIP(rse::launch_bitslice_recon(c->kfield, (uint32_t)k, (uint32_t)p, rows.data(), b,
                                       len_bytes / 16u, s, &coded));
    if (!coded) return RSE_OK;  // first batch decides; nothing launched
  }
  *done = coded;
  return RSE_OK;
}

thread_local int64_t g_pattern_launches = 0;  // RSE_OPT_PATTERN_LAUNCHES
thread_local int64_t g_host_planned = 0;      // RSE_OPT_HOST_PLANNED_STRIPES

// Decode patterns used more than once (the decode-matrix LRU of
// core.rs:697-731 counts them) get a bit-sliced kernel built at run time for
// the plan's composed rows (rse_jit.cpp): the encode kernel over the k valid
// inputs, one pass at encode speed with no run-time mixing.  Until it is ready
// the syndrome kernel serves the pattern.  RSE_OPT_JIT 2 builds (and waits
// for) it on first use.  True if the pattern kernel is ready for this plan.
// Wide codecs (k > 32) and patterns with more than 8 rows get block kernels
// instead (jit_register_blocks; run_job launches them once all are ready),
// when a call codes 1 MiB of every shard or more (each block is seconds of
// hiprtc; `volume`: the bytes per shard over all stripes of the call).
// Shards of 4 KiB or more qualify, and of exactly 1 or 2 KiB (bitslice_len;
// the SUB kernels).  Below 16 KiB the syndrome kernels code nothing (16 KiB
// chunks), so without a pattern kernel such shards run on the table kernels.
bool pattern_kernel(const rse_codec* c, const ReconPlan& plan, size_t len_bytes,
                    size_t volume = 0) {
  const int64_t mode = rse::get_option(RSE_OPT_JIT);
  if (mode == 0 || !rse::get_option(RSE_OPT_JIT_PATTERNS) || !rse::get_option(RSE_OPT_BITSLICE) ||
      !bitslice_len(len_bytes) ||
      (mode < 2 && plan.pattern_uses < 2))
    return false;
  const uint32_t k = (uint32_t)c->k, n = (uint32_t)plan.rows.n_out;
  if (n > rse::kJitMaxOut || k > (uint32_t)kMaxIn) {
    if (mode < 2 && std::max(len_bytes, volume) < (1u << 20)) return false;
    if (rse::wide_eligible(k, n)) {  // run_job launches it
      if (!rse::jit_register_wide(c->kfield, k, n, plan.rows.c.data(), true)) return false;
      return rse::jit_wide_status(c->kfield, k, n, plan.rows.c.data(), mode >= 2) == 2;
    }
    if (!rse::jit_register_blocks(c->kfield, k, n, plan.rows.c.data(), true)) return false;
    return rse::jit_blocks_status(c->kfield, k, n, plan.rows.c.data(), mode >= 2) == 2;
  }
  if (!rse::jit_register(c->kfield, k, n, plan.rows.c.data(), rse::kJitPattern)) return false;
  return rse::jit_status(c->kfield, k, n, plan.rows.c.data(), mode >= 2) == 2;
}

// Codes plan.rows over [off, len) of every shard (the table kernels).
int run_plan_tail(const rse_codec* c, const ReconPlan& plan, size_t off, uint64_t stripe_stride,
                  size_t n_stripes, hipStream_t s) {
  const size_t len = plan.len * c->esize();
  if (off >= len) return RSE_OK;
  std::vector<const uint8_t*> in(plan.in);
  std::vector<uint8_t*> out(plan.out);
  for (auto& q : in) q += off;
  for (auto& q : out) q += off;
  Job j{c->kfield, &plan.rows, in.data(), out.data(), nullptr, len - off, rse::kStore, false,
        nullptr, stripe_stride, n_stripes};
  return run_job(j, s);
}

// Every data shard of a k = p = 16 / 32 / 64 GF(2^8) codec rebuilt from its
// parity shards: run_job codes the plan's rows on the additive-FFT kernels
// (rse_fft.hip), so neither a pattern module nor the syndrome kernels apply.
bool fft_plan(const rse_codec* c, const ReconPlan& plan) {
  return plan.rows.n_in == plan.rows.n_out &&
         rse::fft_applies(c->kfield, (uint32_t)plan.rows.n_in, (uint32_t)plan.rows.n_out,
                          plan.rows.c.data());
}

int reconstruct_impl(const rse_codec* c, void* const* shards, const size_t* lens,
                     const uint8_t* present, size_t n, bool data_only, hipStream_t s) {
  if (!c) return RSE_ERR_INVALID_ARGUMENT;
  ReconPlan plan;
  int rc = plan_reconstruct(c, shards, lens, present, n, data_only, plan);
  if (rc || plan.nothing_to_do || plan.rows.n_out == 0) return rc;
  if (fft_plan(c, plan)) return run_plan_tail(c, plan, 0, 0, 1, s);
  if (pattern_kernel(c, plan, plan.len * c->esize())) {
    ++g_pattern_launches;
    return run_plan_tail(c, plan, 0, 0, 1, s);  // launch_code finds the pattern's kernel
  }
  size_t done = 0;
  rc = bitslice_reconstruct(c, reinterpret_cast<const uint8_t* const*>(shards), present, data_only,
                            plan.len * c->esize(), 0, 1, s, &done);
  if (rc) return rc;
  return run_plan_tail(c, plan, done, 0, 1, s);
}

int host_code(int field, const Rows& rows, const void* const* in, void* const* out, size_t len_bytes,
              bool accumulate, hipStream_t s, bool any_mem = false);

// host: the shards are in host memory (rse_encode_sep_host): same validation,
// then the host pipeline instead of device launches.
// n_stripes flat stripes that share one erasure pattern (reconstruct, or
// reconstruct_data: the wasm ABI, wasm/src/lib.rs:57-73): planned once on the
// host (with the LRU), then coded by the pattern's own kernel if it has one,
// else the bit-sliced syndrome kernel, the table kernels for the rest.
int flat_reconstruct(const rse_codec* c, uint8_t* base, size_t shard_len, size_t n_stripes,
                     const uint8_t* present, bool data_only, hipStream_t s) {
  if (n_stripes == 0) return RSE_OK;
  const size_t sb = shard_len * c->esize();
  std::vector<void*> ptrs(c->total);
  std::vector<size_t> lens(c->total, shard_len);
  for (size_t i = 0; i < c->total; ++i) ptrs[i] = base + i * sb;
  ReconPlan plan;
  int rc = plan_reconstruct(c, ptrs.data(), lens.data(), present, c->total, data_only, plan);
  if (rc || plan.nothing_to_do || plan.rows.n_out == 0) return rc;
  const uint64_t stride = (uint64_t)c->total * sb;
  if (fft_plan(c, plan)) return run_plan_tail(c, plan, 0, stride, n_stripes, s);
  if (pattern_kernel(c, plan, sb, sb * n_stripes)) {
    ++g_pattern_launches;
    return run_plan_tail(c, plan, 0, stride, n_stripes, s);
  }
  size_t done = 0;
  rc = bitslice_reconstruct(c, reinterpret_cast<const uint8_t* const*>(ptrs.data()), present,
                            data_only, sb, stride, n_stripes, s, &done);
  if (rc) return rc;
  return run_plan_tail(c, plan, done, stride, n_stripes, s);
}

int encode_sep_impl(const rse_codec* c, const void* const* data, const size_t* data_lens,
                    size_t n_data, void* const* parity, const size_t* parity_lens,
                    size_t n_parity, hipStream_t s, bool host = false) {
  int rc;
  if ((rc = check_count(n_data, c->k, RSE_TOO_FEW_DATA_SHARDS, RSE_TOO_MANY_DATA_SHARDS))) return rc;
  if ((rc = check_count(n_parity, c->p, RSE_TOO_FEW_PARITY_SHARDS, RSE_TOO_MANY_PARITY_SHARDS)))
    return rc;
  if (!data_lens || !parity_lens || !data || !parity) return RSE_ERR_INVALID_ARGUMENT;
  if ((rc = check_multi(data_lens, n_data))) return rc;
  if ((rc = check_multi(parity_lens, n_parity))) return rc;
  if (data_lens[0] != parity_lens[0]) return RSE_INCORRECT_SHARD_SIZE;
  want_bitslice(c, data_lens[0] * c->esize());
  const Rows rows = parity_rows(c);
  if (host) return host_code(c->field, rows, data, parity, data_lens[0] * c->esize(), false, s);
  Job j{c->kfield, &rows, reinterpret_cast<const uint8_t* const*>(data),
        reinterpret_cast<uint8_t* const*>(parity), nullptr, data_lens[0] * c->esize(),
        rse::kStore, false, nullptr, 0, 1};
  return run_job(j, s);
}

int encode_single_sep_impl(const rse_codec* c, size_t i_data, const void* single,
                           size_t single_len, void* const* parity, const size_t* parity_lens,
                           size_t n_parity, hipStream_t s, bool host = false) {
  int rc;
  if (i_data >= c->k) return RSE_INVALID_INDEX;
  if ((rc = check_count(n_parity, c->p, RSE_TOO_FEW_PARITY_SHARDS, RSE_TOO_MANY_PARITY_SHARDS)))
    return rc;
  if (!parity_lens || !parity || !single) return RSE_ERR_INVALID_ARGUMENT;
  if ((rc = check_multi(parity_lens, n_parity))) return rc;
  if (parity_lens[0] != single_len) return RSE_INCORRECT_SHARD_SIZE;
  const Rows rows = single_column(c, i_data);
  if (host) {
    const void* hin[1] = {single};
    return host_code(c->field, rows, hin, parity, single_len * c->esize(), i_data != 0, s);
  }
  const uint8_t* in[1] = {static_cast<const uint8_t*>(single)};
  Job j{c->kfield, &rows, in, reinterpret_cast<uint8_t* const*>(parity), nullptr,
        single_len * c->esize(), rse::kStore, i_data != 0, nullptr, 0, 1};
  return run_job(j, s);
}

// verify / verify_with_buffer argument checks (core.rs:637-669 via macros.rs).
int verify_checks(const rse_codec* c, const void* const* shards, const size_t* lens, size_t n,
                  void* const* buffer, const size_t* buf_lens, size_t n_buf, bool with_buffer,
                  int* ok) {
  int rc;
  if (!c || !ok) return RSE_ERR_INVALID_ARGUMENT;
  if ((rc = check_count(n, c->total, RSE_TOO_FEW_SHARDS, RSE_TOO_MANY_SHARDS))) return rc;
  if (with_buffer &&
      (rc = check_count(n_buf, c->p, RSE_TOO_FEW_BUFFER_SHARDS, RSE_TOO_MANY_BUFFER_SHARDS)))
    return rc;
  if (!lens || !shards) return RSE_ERR_INVALID_ARGUMENT;
  if ((rc = check_multi(lens, n))) return rc;
  if (with_buffer) {
    if (!buf_lens || !buffer) return RSE_ERR_INVALID_ARGUMENT;
    if ((rc = check_multi(buf_lens, n_buf))) return rc;
    if (lens[0] != buf_lens[0]) return RSE_INCORRECT_SHARD_SIZE;
  }
  return RSE_OK;
}

int verify_impl(const rse_codec* c, const void* const* shards, const size_t* lens, size_t n,
                void* const* buffer, const size_t* buf_lens, size_t n_buf, bool with_buffer,
                int* ok, hipStream_t s) {
  int rc = verify_checks(c, shards, lens, n, buffer, buf_lens, n_buf, with_buffer, ok);
  if (rc) return rc;
  want_bitslice(c, lens[0] * c->esize());
  const Rows rows = parity_rows(c);
  Job j{c->kfield, &rows, reinterpret_cast<const uint8_t* const*>(shards),
        with_buffer ? reinterpret_cast<uint8_t* const*>(buffer) : nullptr,
        reinterpret_cast<const uint8_t* const*>(shards) + c->k, lens[0] * c->esize(),
        with_buffer ? rse::kCheckStore : rse::kCheck, false, nullptr, 0, 1};
  return run_check(j, s, ok);
}

// ------------------------------------------------------------ host memory
// The reference's API takes caller slices in host memory (core.rs:597-695).
// The *_host entries do the same work on host shards through a three-stage
// pipeline over chunks of every shard: H2D of the shards the operation reads
// (on one of RSE_OPT_HOST_H2D_STREAMS streams), the device operation on a
// second stream, D2H of the shards it writes on a third.  A ring of device
// buffer sets means chunk c's H2D overlaps chunk c-1's kernels and chunk c-2's
// D2H (and H2D overlaps D2H on the full-duplex link).  Only the shards an
// operation reads cross PCIe towards the device -- for reconstruct the k valid
// shards of core.rs:801-841, not every present one -- and only the shards it
// writes come back.  Pinned host memory gives asynchronous DMA; pageable
// memory works (the runtime stages it) but serialises the copies.
enum class HostOp { kEncode, kVerify, kVerifyBuf, kRecon, kReconData, kCode };

struct HostStripe {
  void* const* sh;         // the stripe's k + p host shards (kCode: inputs, then outputs)
  void* const* buf;        // kVerifyBuf: its p host buffer shards
  const uint8_t* present;  // kRecon*: its k + p presence flags
  bool flat = false;       // shards are parts of ONE caller buffer (the *_flat entries)
};

// Shards one stripe's operation reads (up) and writes (down); index total + r
// is buffer shard r (verify_with_buffer).
// kCode: inputs [0, k), outputs [k, T), read too when accumulating.
void host_sets(uint32_t k, uint32_t T, uint32_t p, HostOp op, bool accumulate,
               const uint8_t* present, std::vector<uint32_t>& up, std::vector<uint32_t>& down) {
  up.clear();
  down.clear();
  switch (op) {
    case HostOp::kCode:
      for (uint32_t i = 0; i < T; ++i) {
        if (i < k || accumulate) up.push_back(i);
        if (i >= k) down.push_back(i);
      }
      break;
    case HostOp::kEncode:
      for (uint32_t i = 0; i < T; ++i) (i < k ? up : down).push_back(i);
      break;
    case HostOp::kVerify:
    case HostOp::kVerifyBuf:
      for (uint32_t i = 0; i < T; ++i) up.push_back(i);
      if (op == HostOp::kVerifyBuf)
        for (uint32_t r = 0; r < p; ++r) down.push_back(T + r);
      break;
    case HostOp::kRecon:
    case HostOp::kReconData: {
      uint32_t nv = 0;  // the valid inputs: the first k present shards
      for (uint32_t i = 0; i < T; ++i) {
        if (present[i]) {
          if (nv < k) {
            up.push_back(i);
            ++nv;
          }
        } else if (i < k || op == HostOp::kRecon) {
          down.push_back(i);
        }
      }
      break;
    }
  }
}

// Copies bytes [off, off + sz) of the listed shards between the host and the
// ring slot `dset` (shard i at dset + i * chunk).  Shards of one caller
// buffer (flat): one 2D copy per run of consecutive indices whose shards are
// equally spaced; otherwise one plain copy per shard (a 2D copy must stay
// inside one host allocation: separate allocations that happen to be equally
// spaced are not one buffer).
template <class HostPtr>
hipError_t copy_shards(bool h2d, uint8_t* dset, size_t chunk, const std::vector<uint32_t>& idx,
                       HostPtr host, size_t off, size_t sz, bool flat, bool any_mem,
                       hipStream_t s) {
  hipError_t e = hipSuccess;
  if (!rse::get_option(RSE_OPT_HOST_COPY_2D)) flat = false;
  for (size_t a = 0; a < idx.size() && e == hipSuccess;) {
    size_t b = a + 1;
    ptrdiff_t pitch = 0;
    if (flat && b < idx.size() && idx[b] == idx[a] + 1) pitch = host(idx[b]) - host(idx[a]);
    if (pitch > 0 && (size_t)pitch >= sz)
      while (b < idx.size() && idx[b] == idx[b - 1] + 1 && host(idx[b]) - host(idx[b - 1]) == pitch)
        ++b;
    else
      b = a + 1;
    uint8_t* d = dset + (size_t)idx[a] * chunk;
    uint8_t* h = host(idx[a]) + off;
    const size_t rows = b - a;
    if (rows == 1)
      e = hipMemcpyAsync(h2d ? d : h, h2d ? h : d, sz,
                         any_mem ? hipMemcpyDefault
                         : h2d   ? hipMemcpyHostToDevice
                                 : hipMemcpyDeviceToHost,
                         s);
    else if (h2d)
      e = hipMemcpy2DAsync(d, chunk, h, (size_t)pitch, sz, rows, hipMemcpyHostToDevice, s);
    else
      e = hipMemcpy2DAsync(h, (size_t)pitch, d, chunk, sz, rows, hipMemcpyDeviceToHost, s);
    a = b;
  }
  return e;
}

// The low-level op (rse_code_shards_host): rows over n_in inputs.  any_mem:
// some of the caller's buffers may be device memory (the Field/FFI hooks on
// mixed arguments), so the copies let the runtime infer their direction.
struct HostCode {
  int field;
  const Rows* rows;
  bool accumulate;
  bool any_mem = false;
};

// Small calls: one stripe moving at most kHostDirectBytes (both ways) skips
// the pipeline.  Its per-shard copies cost ~10 us of runtime work each for
// pageable memory (the runtime stages every one), ~170 us for a 10+4 stripe
// of 1 KiB shards (profiles/r04/s4/bench.log, crossover_10_4), far more than
// the bytes.  Here the CPU copies the shards the operation reads into the
// lease's pinned words, one DMA takes them up, the operation runs on the
// caller's stream, one DMA brings the shards it writes back, and the CPU
// copies them out.
constexpr size_t kHostDirectBytes = size_t(2) << 20;

int host_direct(const rse_codec* c, HostOp op, const HostStripe& hs, size_t bytes, hipStream_t user,
                int* ok, const HostCode* code, bool* handled) {
  *handled = false;
  const bool low = op == HostOp::kCode;
  if (low && code->any_mem) return RSE_OK;  // device memory among the buffers: the pipeline
  const bool verify = op == HostOp::kVerify || op == HostOp::kVerifyBuf;
  const int field = low ? code->field : c->field;
  const size_t k = low ? code->rows->n_in : c->k;
  const size_t T = low ? k + code->rows->n_out : c->total;
  const size_t p = T - k, es = field == RSE_FIELD_GF16 ? 2 : 1;
  const size_t nbuf = T + (op == HostOp::kVerifyBuf ? p : 0);
  std::vector<uint32_t> up, down;
  host_sets((uint32_t)k, (uint32_t)T, (uint32_t)p, op, low && code->accumulate, hs.present, up,
            down);
  if ((up.size() + down.size()) * bytes > kHostDirectBytes) return RSE_OK;
  *handled = true;
  if (down.empty() && !verify) return RSE_OK;  // nothing to rebuild
  // device: shard i at dbuf + i * sz (sz: bytes rounded up to 16), then the verdict word
  const size_t sz = (bytes + 15) & ~size_t(15), words = (nbuf * sz) / 4 + 1;
  Lease res;
  hipError_t e = res.acquire();
  if (e == hipSuccess) e = lease_words(res.get(), words);
  if (e == hipSuccess) e = lease_ring(res.get(), nbuf * sz + 256);
  if (e == hipSuccess && res->dbytes < nbuf * sz + 256) e = hipErrorOutOfMemory;
  if (e != hipSuccess) return dev_fail(e);
  uint8_t* dbuf = res->dbuf;
  uint8_t* hst = reinterpret_cast<uint8_t*>(res->wh);
  uint32_t* dword = reinterpret_cast<uint32_t*>(dbuf + nbuf * sz);
  auto host = [&](uint32_t i) { return static_cast<uint8_t*>(i < T ? hs.sh[i] : hs.buf[i - T]); };
  for (uint32_t i : up) std::memcpy(hst + (size_t)i * sz, host(i), bytes);
  // one DMA up over the span of the shards read, one down over those written
  const size_t u0 = up.empty() ? 0 : up.front(), u1 = up.empty() ? 0 : up.back() + 1;
  if (u1 > u0)
    e = hipMemcpyAsync(dbuf + u0 * sz, hst + u0 * sz, (u1 - u0) * sz, hipMemcpyHostToDevice, user);
  if (e == hipSuccess && verify) e = hipMemsetAsync(dword, 0, 4, user);
  if (e != hipSuccess) {
    (void)hipStreamSynchronize(user);
    return dev_fail(e);
  }
  std::vector<uint8_t*> dev(nbuf);
  for (size_t i = 0; i < nbuf; ++i) dev[i] = dbuf + i * sz;
  const Rows rows = low ? Rows{} : parity_rows(c);
  const Rows& code_rows = low ? *code->rows : rows;
  std::vector<size_t> lens(T, bytes / es);
  int rc = RSE_OK;
  switch (op) {
    case HostOp::kEncode:
    case HostOp::kCode: {
      Job j{field, &code_rows, dev.data(), dev.data() + k, nullptr, bytes, rse::kStore,
            low && code->accumulate, nullptr, 0, 1};
      rc = run_job(j, user);
      break;
    }
    case HostOp::kVerify:
    case HostOp::kVerifyBuf: {
      const bool wb = op == HostOp::kVerifyBuf;
      Job j{field, &rows, dev.data(), wb ? dev.data() + T : nullptr, dev.data() + k, bytes,
            wb ? rse::kCheckStore : rse::kCheck, false, dword, 0, 1};
      rc = run_job(j, user);
      break;
    }
    case HostOp::kRecon:
    case HostOp::kReconData:
      rc = reconstruct_impl(c, reinterpret_cast<void* const*>(dev.data()), lens.data(), hs.present,
                            T, op == HostOp::kReconData, user);
      break;
  }
  const size_t d0 = down.empty() ? 0 : down.front(), d1 = down.empty() ? 0 : down.back() + 1;
  if (rc == RSE_OK && d1 > d0)
    e = hipMemcpyAsync(hst + d0 * sz, dbuf + d0 * sz, (d1 - d0) * sz, hipMemcpyDeviceToHost, user);
  uint32_t* hword = res->wh + (words - 1);
  if (rc == RSE_OK && e == hipSuccess && verify)
    e = hipMemcpyAsync(hword, dword, 4, hipMemcpyDeviceToHost, user);
  const hipError_t e2 = hipStreamSynchronize(user);
  if (rc) return rc;
  if (e != hipSuccess) return dev_fail(e);
  if (e2 != hipSuccess) return dev_fail(e2);
  for (uint32_t i : down) std::memcpy(host(i), hst + (size_t)i * sz, bytes);
  if (verify && ok) ok[0] = *reinterpret_cast<volatile uint32_t*>(hword) == 0 ? 1 : 0;
  return RSE_OK;
}

// The device address of pinned, device-mapped host memory at p (interior
// pointers too), or nullptr (pageable memory, device memory, no mapping).
uint8_t* mapped_host(const void* p) {
  hipPointerAttribute_t a;
  std::memset(&a, 0, sizeof a);
  const hipError_t pending = hipPeekAtLastError();
  if (hipPointerGetAttributes(&a, p) != hipSuccess) {
    if (pending == hipSuccess) (void)hipGetLastError();
    return nullptr;
  }
  if (a.type != hipMemoryTypeHost || !a.devicePointer) return nullptr;
  return static_cast<uint8_t*>(a.devicePointer);
}

// Runs `op` over `bytes` of every shard of every stripe (codec ops: `c`;
// kCode: `code`).  verify ops: ok[s] receives stripe s's verdict.
//
// Outputs written in place (RSE_OPT_HOST_ZC_OUT, default 1): when the shards
// an encode or reconstruct writes are pinned, device-mapped host memory, the
// coding kernel stores them there through the mapping (posted PCIe writes)
// instead of into the device ring for a D2H copy.  The pipeline then has no
// D2H copies: the copy engines carry only the H2D traffic, so a D2H copy can
// never queue in front of (or share an engine with) the next chunk's H2D
// copies.  In the bench's sequence the two-copy pipeline ran at 40 GB/s for
// its first second of calls and 75 GB/s after (profiles/r06/s9/probe.log).
int host_pipeline(const rse_codec* c, HostOp op, const std::vector<HostStripe>& stripes,
                  size_t bytes, hipStream_t user, int* ok, const HostCode* code = nullptr) {
  if (stripes.size() == 1 && rse::get_option(RSE_OPT_HOST_DIRECT)) {
    bool handled = false;
    const int rc = host_direct(c, op, stripes[0], bytes, user, ok, code, &handled);
    if (handled || rc) return rc;
  }
  const int64_t chunk_kib = rse::get_option(RSE_OPT_HOST_CHUNK_KIB);
  const int nh = (int)std::max<int64_t>(1, std::min<int64_t>(4, rse::get_option(RSE_OPT_HOST_H2D_STREAMS)));
  const int ring = std::max(3, nh + 2);  // slots: nh filling, one coding, one draining
  const size_t chunk = std::min<size_t>(bytes, (size_t)std::max<int64_t>(64, chunk_kib) << 10);
  const size_t per_stripe = (bytes + chunk - 1) / chunk;
  const size_t nchunks = per_stripe * stripes.size();
  const bool verify = op == HostOp::kVerify || op == HostOp::kVerifyBuf;
  const bool low = op == HostOp::kCode;
  const bool any_mem = low && code->any_mem;
  const int field = low ? code->field : c->field;
  const size_t k = low ? code->rows->n_in : c->k;
  const size_t T = low ? k + code->rows->n_out : c->total;
  const size_t p = T - k, es = field == RSE_FIELD_GF16 ? 2 : 1;
  const size_t nbuf = T + (op == HostOp::kVerifyBuf ? p : 0);  // shards per slot
  // streams: [0, nh) H2D, nh kernel, nh + 1 D2H (leased: Scratch)
  Lease res;
  hipError_t e = res.acquire();
  if (e == hipSuccess) e = lease_pipe(res.get(), nh, ring, ring * nbuf * chunk);
  if (e != hipSuccess) return dev_fail(e);
  const std::vector<hipStream_t>& st = res->st;
  const std::vector<hipEvent_t>&h2d = res->h2d, &coded = res->coded, &d2h = res->d2h;
  hipEvent_t start = res->start;
  uint8_t* dbuf = res->dbuf;
  uint8_t* call_ring = nullptr;  // a ring too big to keep: this call's own
  if (res->dbytes < ring * nbuf * chunk) {
    e = hipMallocAsync(reinterpret_cast<void**>(&call_ring), ring * nbuf * chunk, user);
    if (e != hipSuccess) return dev_fail(e);
    dbuf = call_ring;
  }
  uint32_t *dwords = nullptr, *hwords = nullptr;
  if (verify) {  // one mismatch word per stripe
    const size_t wb = stripes.size() * sizeof(uint32_t);
    if (e == hipSuccess) e = hipMallocAsync(reinterpret_cast<void**>(&dwords), wb, user);
    if (e == hipSuccess) e = hipMemsetAsync(dwords, 0, wb, user);
    if (e == hipSuccess) e = hipHostMalloc(reinterpret_cast<void**>(&hwords), wb, hipHostMallocDefault);
  }
  if (e == hipSuccess) e = hipEventRecord(start, user);  // everything starts after the caller's work
  for (auto& q : st)
    if (e == hipSuccess) e = hipStreamWaitEvent(q, start, 0);
  if (op == HostOp::kEncode || verify) want_bitslice(c, chunk);
  const Rows rows = low ? Rows{} : parity_rows(c);
  const Rows& code_rows = low ? *code->rows : rows;
  std::vector<uint8_t*> dev(nbuf);
  std::vector<size_t> lens(T);
  std::vector<uint32_t> up, down;
  hipStream_t kst = st[nh], dst = st[nh + 1];
  int rc = RSE_OK;
  size_t set_for = ~size_t(0);
  // outputs in place: encode / reconstruct, outputs not read (no accumulate)
  const bool zc = rse::get_option(RSE_OPT_HOST_ZC_OUT) &&
                  (op == HostOp::kEncode || op == HostOp::kRecon || op == HostOp::kReconData ||
                   (low && !code->accumulate && !any_mem));
  std::vector<uint8_t*> zmap(nbuf, nullptr);  // the stripe's written shards' device mappings
  bool zc_stripe = false;
  for (size_t ci = 0; e == hipSuccess && rc == RSE_OK && ci < nchunks; ++ci) {
    const size_t si = ci / per_stripe;
    const HostStripe& hs = stripes[si];
    auto host = [&](uint32_t i) {
      return static_cast<uint8_t*>(i < T ? hs.sh[i] : hs.buf[i - T]);
    };
    if (si != set_for) {
      host_sets((uint32_t)k, (uint32_t)T, (uint32_t)p, op, low && code->accumulate, hs.present,
                up, down);
      set_for = si;
      zc_stripe = zc && !down.empty();
      for (size_t d = 0; zc_stripe && d < down.size(); ++d) {
        const uint32_t i = down[d];
        zmap[i] = i < nbuf ? mapped_host(host(i)) : nullptr;
        zc_stripe = zmap[i] && aligned16(zmap[i]);
      }
    }
    if (down.empty() && !verify) continue;  // nothing to rebuild in this stripe
    const size_t off = (ci % per_stripe) * chunk, sz = std::min(chunk, bytes - off);
    const int b = (int)(ci % ring);
    hipStream_t hst = st[ci % nh];
    uint8_t* set = dbuf + b * nbuf * chunk;
    if (ci >= (size_t)ring) e = hipStreamWaitEvent(hst, d2h[b], 0);  // slot drained
    if (e == hipSuccess) e = copy_shards(true, set, chunk, up, host, off, sz, hs.flat, any_mem, hst);
    if (e == hipSuccess) e = hipEventRecord(h2d[b], hst);
    if (e == hipSuccess) e = hipStreamWaitEvent(kst, h2d[b], 0);
    if (e != hipSuccess) break;
    for (size_t i = 0; i < nbuf; ++i) dev[i] = set + i * chunk;
    if (zc_stripe)
      for (uint32_t i : down) dev[i] = zmap[i] + off;
    switch (op) {
      case HostOp::kEncode:
      case HostOp::kCode: {
        Job j{field, &code_rows, dev.data(), dev.data() + k, nullptr, sz, rse::kStore,
              low && code->accumulate, nullptr, 0, 1};
        rc = run_job(j, kst);
        break;
      }
      case HostOp::kVerify:
      case HostOp::kVerifyBuf: {
        const bool wb = op == HostOp::kVerifyBuf;
        Job j{field, &rows, dev.data(), wb ? dev.data() + T : nullptr, dev.data() + k, sz,
              wb ? rse::kCheckStore : rse::kCheck, false, dwords + si, 0, 1};
        rc = run_job(j, kst);
        break;
      }
      case HostOp::kRecon:
      case HostOp::kReconData:
        std::fill(lens.begin(), lens.end(), sz / es);
        rc = reconstruct_impl(c, reinterpret_cast<void* const*>(dev.data()), lens.data(),
                              hs.present, T, op == HostOp::kReconData, kst);
        break;
    }
    if (rc) break;
    if (zc_stripe) {  // written in place: the slot is free when the kernel is done
      e = hipEventRecord(d2h[b], kst);
      continue;
    }
    e = hipEventRecord(coded[b], kst);
    if (e == hipSuccess) e = hipStreamWaitEvent(dst, coded[b], 0);
    if (e == hipSuccess) e = copy_shards(false, set, chunk, down, host, off, sz, hs.flat, any_mem, dst);
    if (e == hipSuccess) e = hipEventRecord(d2h[b], dst);
  }
  // join: the caller's stream waits for every stream, frees the ring, syncs
  hipError_t e2 = hipSuccess;
  for (auto& q : st)
    if (q && e2 == hipSuccess) {
      e2 = hipEventRecord(start, q);
      if (e2 == hipSuccess) e2 = hipStreamWaitEvent(user, start, 0);
    }
  if (verify && dwords && hwords && e == hipSuccess && e2 == hipSuccess && rc == RSE_OK)
    e2 = hipMemcpyAsync(hwords, dwords, stripes.size() * sizeof(uint32_t), hipMemcpyDeviceToHost,
                        user);
  if (dwords) (void)hipFreeAsync(dwords, user);
  if (call_ring) (void)hipFreeAsync(call_ring, user);
  const hipError_t e3 = hipStreamSynchronize(user);
  if (e2 == hipSuccess) e2 = e3;
  if (e2 != hipSuccess || e != hipSuccess || rc != RSE_OK)
    for (auto& q : st) (void)hipStreamSynchronize(q);  // idle before the next call reuses them
  if (verify && ok && hwords && e == hipSuccess && e2 == hipSuccess && rc == RSE_OK)
    for (size_t s = 0; s < stripes.size(); ++s) ok[s] = hwords[s] == 0 ? 1 : 0;
  if (hwords) (void)hipHostFree(hwords);
  if (rc) return rc;
  if (e != hipSuccess) return dev_fail(e);
  if (e2 != hipSuccess) return dev_fail(e2);
  return RSE_OK;
}

// rows x host inputs -> host outputs through the pipeline (kCode).
int host_code(int field, const Rows& rows, const void* const* in, void* const* out, size_t len_bytes,
              bool accumulate, hipStream_t s, bool any_mem) {
  std::vector<void*> ptrs(rows.n_in + rows.n_out);
  for (size_t i = 0; i < rows.n_in; ++i) ptrs[i] = const_cast<void*>(in[i]);
  for (size_t o = 0; o < rows.n_out; ++o) ptrs[rows.n_in + o] = out[o];
  for (void* q : ptrs)
    if (!q) return RSE_ERR_INVALID_ARGUMENT;
  const HostCode hc{field, &rows, accumulate, any_mem};
  return host_pipeline(nullptr, HostOp::kCode, {HostStripe{ptrs.data(), nullptr, nullptr}},
                       len_bytes, s, nullptr, &hc);
}

// Flat host stripes: shard i of stripe s at base + (s * total + i) * sb.
std::vector<void*> flat_ptrs(const rse_codec* c, void* base, size_t sb, size_t n_stripes) {
  std::vector<void*> ptrs(n_stripes * c->total);
  for (size_t i = 0; i < ptrs.size(); ++i) ptrs[i] = static_cast<uint8_t*>(base) + i * sb;
  return ptrs;
}

// Makes `dev` current for a scope (dev < 0: no change) and restores the
// caller's device.
class OnDevice {
 public:
  explicit OnDevice(int dev) {
    int cur = 0;
    if (dev < 0 || hipGetDevice(&cur) != hipSuccess || cur == dev) return;
    if (hipSetDevice(dev) == hipSuccess) prev_ = cur;
  }
  ~OnDevice() {
    if (prev_ >= 0) (void)hipSetDevice(prev_);
  }
  OnDevice(const OnDevice&) = delete;
  OnDevice& operator=(const OnDevice&) = delete;

 private:
  int prev_ = -1;
};

// Where a caller buffer lives.  True for device memory (hipMalloc'd or
// managed) and sets *dev; false for host memory -- pageable (unknown to the
// runtime), pinned or registered.
bool device_memory(const void* p, int* dev) {
  hipPointerAttribute_t a;
  std::memset(&a, 0, sizeof a);
  // an unregistered host pointer is not an error here: clear the error the
  // query leaves behind, but only when the caller had none pending (an
  // earlier asynchronous launch failure must stay visible to them)
  const hipError_t pending = hipPeekAtLastError();
  if (hipPointerGetAttributes(&a, p) != hipSuccess) {
    if (pending == hipSuccess) (void)hipGetLastError();
    return false;
  }
  if (a.type != hipMemoryTypeDevice && a.type != hipMemoryTypeManaged) return false;
  *dev = a.device;
  return true;
}

// The Field/FFI slice hooks (galois_8.rs:291-327 mul_slice(_xor) over
// reedsolomon_gal_mul(_xor); galois_16's Field::mul_slice(_add), lib.rs:99-118):
// out (+)= c * in over len elements, wherever the caller's slices live -- the
// reference's callers pass host slices.
//  * in and out in device memory of one device: the kernel, asynchronous on
//    `stream`; with `sync`, on a leased library stream of that device, waited
//    for (only this call's work, not the whole device).
//  * either in host memory: the host pipeline (H2D, kernel, D2H; synchronous),
//    on `stream` or, with `sync`, a leased library stream.  A side that is
//    device memory is copied device to device by the same pipeline.
int mul_slice_any(int field, const uint8_t* coef, const void* in, void* out, size_t len,
                  bool acc, hipStream_t stream, bool sync) {
  if (!coef || (len && (!in || !out))) return RSE_ERR_INVALID_ARGUMENT;
  if (len == 0) return RSE_OK;
  int din = -1, dout = -1;
  const bool di = device_memory(in, &din), dd = device_memory(out, &dout);
  Rows r;
  r.n_out = r.n_in = 1;
  r.c.assign(1, field == RSE_FIELD_GF16 ? (uint16_t)((coef[0] << 8) | coef[1]) : coef[0]);
  const size_t bytes = len * (field == RSE_FIELD_GF16 ? 2 : 1);
  std::unique_ptr<OnStreamDevice> on_stream;
  std::unique_ptr<OnDevice> on_dev;
  if (sync) on_dev.reset(new OnDevice(dd ? dout : din));  // the data's device
  else on_stream.reset(new OnStreamDevice(stream));
  Lease lease;
  if (sync) {
    RSE_HIP(lease.acquire());
    RSE_HIP(lease_own_stream(lease.get(), &stream));
  }
  if (di && dd && din == dout) {
    const uint8_t* ins[1] = {static_cast<const uint8_t*>(in)};
    uint8_t* outs[1] = {static_cast<uint8_t*>(out)};
    Job j{field, &r, ins, outs, nullptr, bytes, rse::kStore, acc, nullptr, 0, 1};
    const int rc = run_job(j, stream);
    const hipError_t e = sync ? hipStreamSynchronize(stream) : hipSuccess;
    if (rc) return rc;
    RSE_HIP(e);
    return RSE_OK;
  }
  const void* ins[1] = {in};
  void* outs[1] = {out};
  return host_code(field, r, ins, outs, bytes, acc, stream, di || dd);
}

}  // namespace

// =========================================================================
// C ABI
// =========================================================================
extern "C" {

const char* rse_strerror(int status) {
  switch (status) {  // errors.rs:20-38
    case RSE_OK: return "Ok";
    case RSE_TOO_FEW_SHARDS: return "The number of provided shards is smaller than the one in codec";
    case RSE_TOO_MANY_SHARDS: return "The number of provided shards is greater than the one in codec";
    case RSE_TOO_FEW_DATA_SHARDS: return "The number of provided data shards is smaller than the one in codec";
    case RSE_TOO_MANY_DATA_SHARDS: return "The number of provided data shards is greater than the one in codec";
    case RSE_TOO_FEW_PARITY_SHARDS: return "The number of provided parity shards is smaller than the one in codec";
    case RSE_TOO_MANY_PARITY_SHARDS: return "The number of provided parity shards is greater than the one in codec";
    case RSE_TOO_FEW_BUFFER_SHARDS: return "The number of provided buffer shards is smaller than the number of parity shards in codec";
    case RSE_TOO_MANY_BUFFER_SHARDS: return "The number of provided buffer shards is greater than the number of parity shards in codec";
    case RSE_INCORRECT_SHARD_SIZE: return "At least one of the provided shards is not of the correct size";
    case RSE_TOO_FEW_SHARDS_PRESENT: return "The number of shards present is smaller than number of parity shards, cannot reconstruct missing shards";
    case RSE_EMPTY_SHARD: return "The first shard provided is of zero length";
    case RSE_INVALID_SHARD_FLAGS: return "The number of flags does not match the total number of shards";
    case RSE_INVALID_INDEX: return "The data shard index provided is greater or equal to the number of data shards in codec";
    case RSE_ERR_INVALID_ARGUMENT: return "Invalid argument (null pointer, unknown field or size)";
    case RSE_ERR_DEVICE: return "HIP runtime error";
    case RSE_ERR_NO_MEMORY: return "Out of memory";
    case RSE_ERR_SINGULAR_MATRIX: return "Singular matrix";
    default: return "Unknown status";
  }
}

int rse_last_device_error(void) { return g_last_hip_error; }
const char* rse_last_kernel(void) { return rse::last_kernel(); }
const char* rse_version(void) { return "rse-mi355x 0.1.0 (gfx950)"; }

int rse_codec_new(int field, size_t data_shards, size_t parity_shards, rse_codec** out) {
  if (!out || (field != RSE_FIELD_GF8 && field != RSE_FIELD_GF16)) return RSE_ERR_INVALID_ARGUMENT;
  const size_t order = field == RSE_FIELD_GF16 ? 65536 : 256;
  if (data_shards == 0) return RSE_TOO_FEW_DATA_SHARDS;      // core.rs:446-448
  if (parity_shards == 0) return RSE_TOO_FEW_PARITY_SHARDS;  // core.rs:449-451
  if (data_shards + parity_shards > order) return RSE_TOO_MANY_SHARDS;  // core.rs:452-454
  try {
    std::unique_ptr<rse_codec> c(new rse_codec());
    c->field = field;
    c->k = data_shards;
    c->p = parity_shards;
    c->total = data_shards + parity_shards;
    // core.rs:430-436: V * (V[0..k])^-1
    if (field == RSE_FIELD_GF16) {
      auto v = rse::Matrix<rse::Gf16Field>::vandermonde(c->total, c->k);
      rse::Matrix<rse::Gf16Field> top(c->k, c->k), inv;
      for (size_t r = 0; r < c->k; ++r)
        for (size_t j = 0; j < c->k; ++j) top.at(r, j) = v.at(r, j);
      if (!top.invert(inv)) return RSE_ERR_SINGULAR_MATRIX;
      c->m16 = v.multiply(inv);
      bool sub = rse::get_option(RSE_OPT_SUBFIELD) != 0;
      for (size_t r = 0; r < c->total && sub; ++r)
        for (size_t j = 0; j < c->k && sub; ++j) sub = c->m16.at(r, j) < 256;
      c->kfield = sub ? RSE_FIELD_GF8 : RSE_FIELD_GF16;
    } else {
      auto v = rse::Matrix<rse::Gf8Field>::vandermonde(c->total, c->k);
      rse::Matrix<rse::Gf8Field> top(c->k, c->k), inv;
      for (size_t r = 0; r < c->k; ++r)
        for (size_t j = 0; j < c->k; ++j) top.at(r, j) = v.at(r, j);
      if (!top.invert(inv)) return RSE_ERR_SINGULAR_MATRIX;
      c->m8 = v.multiply(inv);
      c->kfield = RSE_FIELD_GF8;
    }
    *out = c.release();
    return RSE_OK;
  } catch (const std::bad_alloc&) {
    return RSE_ERR_NO_MEMORY;
  }
}

void rse_codec_free(rse_codec* codec) { delete codec; }
int rse_codec_field(const rse_codec* c) { return c ? c->field : 0; }
size_t rse_codec_data_shard_count(const rse_codec* c) { return c ? c->k : 0; }
size_t rse_codec_parity_shard_count(const rse_codec* c) { return c ? c->p : 0; }
size_t rse_codec_total_shard_count(const rse_codec* c) { return c ? c->total : 0; }

int rse_codec_kernel_kind(const rse_codec* c, int wait) {
  if (!c) return RSE_ERR_INVALID_ARGUMENT;
  if (rse::bitslice_compiled(c->kfield, (uint32_t)c->k, (uint32_t)c->p)) return RSE_KERNELS_COMPILED;
  const Rows rows = parity_rows(c);
  if (rse::fft_applies(c->kfield, (uint32_t)c->k, (uint32_t)c->p, rows.c.data()))
    return RSE_KERNELS_FFT;
  if (wait) want_bitslice(c, rse::bitslice_chunk_bytes(), true);
  const bool wide = c->k > (size_t)kMaxIn || c->p > rse::kJitMaxOut ||
                    rse::wide_eligible((uint32_t)c->k, (uint32_t)c->p);
  const bool one = rse::wide_eligible((uint32_t)c->k, (uint32_t)c->p);
  switch (wide ? (one ? rse::jit_wide_status(c->kfield, (uint32_t)c->k, (uint32_t)c->p,
                                             rows.c.data(), wait != 0)
                      : rse::jit_blocks_status(c->kfield, (uint32_t)c->k, (uint32_t)c->p,
                                               rows.c.data(), wait != 0))
               : rse::jit_status(c->kfield, (uint32_t)c->k, (uint32_t)c->p, rows.c.data(),
                                 wait != 0)) {
    case 2: return RSE_KERNELS_SPECIALISED;
    case 1: return RSE_KERNELS_SPECIALISING;
    case -1: return RSE_KERNELS_SPECIALISE_FAILED;
    default: return RSE_KERNELS_TABLE;
  }
}

int rse_codec_matrix(const rse_codec* c, uint8_t* out, size_t out_bytes) {
  if (!c || !out) return RSE_ERR_INVALID_ARGUMENT;
  const size_t es = c->esize(), need = c->total * c->k * es;
  if (out_bytes < need) return RSE_ERR_INVALID_ARGUMENT;
  for (size_t r = 0; r < c->total; ++r)
    for (size_t j = 0; j < c->k; ++j) {
      const uint16_t v = c->mat(r, j);
      if (es == 2) {
        out[(r * c->k + j) * 2] = (uint8_t)(v >> 8);
        out[(r * c->k + j) * 2 + 1] = (uint8_t)v;
      } else {
        out[r * c->k + j] = (uint8_t)v;
      }
    }
  return RSE_OK;
}

int rse_encode(const rse_codec* c, void* const* shards, const size_t* lens, size_t n,
               rse_stream_t stream) {
  RSE_ON_STREAM(stream);
  if (!c) return RSE_ERR_INVALID_ARGUMENT;
  int rc;
  if ((rc = check_count(n, c->total, RSE_TOO_FEW_SHARDS, RSE_TOO_MANY_SHARDS))) return rc;
  if (!lens || !shards) return RSE_ERR_INVALID_ARGUMENT;
  if ((rc = check_multi(lens, n))) return rc;
  return encode_sep_impl(c, const_cast<const void* const*>(shards), lens, c->k, shards + c->k,
                         lens + c->k, c->p, (hipStream_t)stream);
}

int rse_encode_sep(const rse_codec* c, const void* const* data, const size_t* data_lens,
                   size_t n_data, void* const* parity, const size_t* parity_lens,
                   size_t n_parity, rse_stream_t stream) {
  RSE_ON_STREAM(stream);
  if (!c) return RSE_ERR_INVALID_ARGUMENT;
  return encode_sep_impl(c, data, data_lens, n_data, parity, parity_lens, n_parity,
                         (hipStream_t)stream);
}

int rse_encode_single(const rse_codec* c, size_t i_data, void* const* shards, const size_t* lens,
                      size_t n, rse_stream_t stream) {
  RSE_ON_STREAM(stream);
  if (!c) return RSE_ERR_INVALID_ARGUMENT;
  int rc;
  if (i_data >= c->k) return RSE_INVALID_INDEX;  // core.rs:552
  if ((rc = check_count(n, c->total, RSE_TOO_FEW_SHARDS, RSE_TOO_MANY_SHARDS))) return rc;
  if (!lens || !shards) return RSE_ERR_INVALID_ARGUMENT;
  if ((rc = check_multi(lens, n))) return rc;
  return encode_single_sep_impl(c, i_data, shards[i_data], lens[i_data], shards + c->k,
                                lens + c->k, c->p, (hipStream_t)stream);
}

int rse_encode_single_sep(const rse_codec* c, size_t i_data, const void* single,
                          size_t single_len, void* const* parity, const size_t* parity_lens,
                          size_t n_parity, rse_stream_t stream) {
  RSE_ON_STREAM(stream);
  if (!c) return RSE_ERR_INVALID_ARGUMENT;
  return encode_single_sep_impl(c, i_data, single, single_len, parity, parity_lens, n_parity,
                                (hipStream_t)stream);
}

int rse_verify(const rse_codec* c, const void* const* shards, const size_t* lens, size_t n,
               int* ok, rse_stream_t stream) {
  RSE_ON_STREAM(stream);
  return verify_impl(c, shards, lens, n, nullptr, nullptr, 0, false, ok, (hipStream_t)stream);
}

int rse_verify_with_buffer(const rse_codec* c, const void* const* shards, const size_t* lens,
                           size_t n, void* const* buffer, const size_t* buf_lens, size_t n_buf,
                           int* ok, rse_stream_t stream) {
  RSE_ON_STREAM(stream);
  return verify_impl(c, shards, lens, n, buffer, buf_lens, n_buf, true, ok, (hipStream_t)stream);
}

int rse_reconstruct(const rse_codec* c, void* const* shards, const size_t* lens,
                    const uint8_t* present, size_t n, rse_stream_t stream) {
  RSE_ON_STREAM(stream);
  return reconstruct_impl(c, shards, lens, present, n, false, (hipStream_t)stream);
}

int rse_reconstruct_data(const rse_codec* c, void* const* shards, const size_t* lens,
                         const uint8_t* present, size_t n, rse_stream_t stream) {
  RSE_ON_STREAM(stream);
  return reconstruct_impl(c, shards, lens, present, n, true, (hipStream_t)stream);
}

}  // extern "C"

namespace {

// One synchronous coding pass of the *_now entries: out = rows x in (check:
// compared with cmp, *mismatch).  The resident dispatcher when it applies
// (rse_dispatch.hip: no launch, no stream); otherwise run_job's launches on a
// leased library stream, waited for.  Either way the call returns with the
// result in device memory, and neither is ordered after the caller's streams:
// the caller has finished writing the inputs (the reference's synchronous
// contract, core.rs:597-695).
// The device that holds every shard of a *_now call (the call has no stream
// to take it from): *dev, or RSE_ERR_INVALID_ARGUMENT for host memory or
// shards on different devices.  One runtime query per allocation, not per
// shard: a shard inside the allocation range found last needs none.
int now_device(const uint8_t* const* a, size_t na, const uint8_t* const* b, size_t nb, int* dev) {
  int d0 = -1;
  uintptr_t lo = 0, hi = 0;
  for (size_t i = 0; i < na + nb; ++i) {
    const uint8_t* q = i < na ? a[i] : b[i - na];
    const uintptr_t u = reinterpret_cast<uintptr_t>(q);
    if (u >= lo && u < hi) continue;
    int d = -1;
    if (!device_memory(q, &d) || (d0 >= 0 && d != d0)) return RSE_ERR_INVALID_ARGUMENT;
    d0 = d;
    void* base = nullptr;
    size_t size = 0;
    if (hipMemGetAddressRange(&base, &size, const_cast<uint8_t*>(q)) == hipSuccess && base) {
      lo = reinterpret_cast<uintptr_t>(base);
      hi = lo + size;
    } else {
      (void)hipGetLastError();
      lo = hi = 0;
    }
  }
  *dev = d0;
  return RSE_OK;
}

int run_now(const rse_codec* c, const Rows& rows, const uint8_t* const* in, uint8_t* const* out,
            const uint8_t* const* cmp, size_t len_bytes, bool* mismatch) {
  const bool check = cmp != nullptr;
  uint8_t* const* tgt = check ? const_cast<uint8_t* const*>(cmp) : out;
  // the shards' device for the whole call (not whichever is current)
  int dev = -1;
  if (const int rc = now_device(in, rows.n_in, tgt, rows.n_out, &dev)) return rc;
  OnDevice on_dev(dev);
  if (rse::dispatch_applies(c->kfield, (uint32_t)rows.n_in, (uint32_t)rows.n_out, len_bytes, in,
                            tgt)) {
    bool mm = false;
    const hipError_t e = rse::dispatch_run(rows.c.data(), (uint32_t)rows.n_in,
                                           (uint32_t)rows.n_out, in, tgt, len_bytes, check, &mm);
    if (e == hipSuccess) {
      if (mismatch) *mismatch = mm;
      return RSE_OK;
    }
    if (e != hipErrorNotSupported) RSE_HIP(e);  // not usable on this device: launch instead
  }
  Lease lease;
  RSE_HIP(lease.acquire());
  hipStream_t st = nullptr;
  RSE_HIP(lease_own_stream(lease.get(), &st));
  Job j{c->kfield, &rows, in, check ? nullptr : out, cmp, len_bytes,
        check ? rse::kCheck : rse::kStore, false, nullptr, 0, 1};
  if (check) {
    int ok = 0;
    const int rc = run_check(j, st, &ok);
    if (rc) return rc;
    if (mismatch) *mismatch = !ok;
    return RSE_OK;
  }
  const int rc = run_job(j, st);
  const hipError_t e = hipStreamSynchronize(st);
  if (rc) return rc;
  RSE_HIP(e);
  return RSE_OK;
}

}  // namespace

extern "C" {

int rse_encode_now(const rse_codec* c, void* const* shards, const size_t* lens, size_t n) {
  if (!c) return RSE_ERR_INVALID_ARGUMENT;
  int rc;
  if ((rc = check_count(n, c->total, RSE_TOO_FEW_SHARDS, RSE_TOO_MANY_SHARDS))) return rc;
  if (!lens || !shards) return RSE_ERR_INVALID_ARGUMENT;
  if ((rc = check_multi(lens, n))) return rc;
  for (size_t i = 0; i < n; ++i)
    if (!shards[i]) return RSE_ERR_INVALID_ARGUMENT;
  const Rows rows = parity_rows(c);
  return run_now(c, rows, reinterpret_cast<const uint8_t* const*>(shards),
                 reinterpret_cast<uint8_t* const*>(shards) + c->k, nullptr, lens[0] * c->esize(),
                 nullptr);
}

int rse_verify_now(const rse_codec* c, const void* const* shards, const size_t* lens, size_t n,
                   int* ok) {
  int rc = verify_checks(c, shards, lens, n, nullptr, nullptr, 0, false, ok);
  if (rc) return rc;
  for (size_t i = 0; i < n; ++i)
    if (!shards[i]) return RSE_ERR_INVALID_ARGUMENT;
  const Rows rows = parity_rows(c);
  bool mm = false;
  rc = run_now(c, rows, reinterpret_cast<const uint8_t* const*>(shards), nullptr,
               reinterpret_cast<const uint8_t* const*>(shards) + c->k, lens[0] * c->esize(), &mm);
  if (rc) return rc;
  *ok = mm ? 0 : 1;
  return RSE_OK;
}

static int reconstruct_now(const rse_codec* c, void* const* shards, const size_t* lens,
                           const uint8_t* present, size_t n, bool data_only) {
  if (!c) return RSE_ERR_INVALID_ARGUMENT;
  ReconPlan plan;
  int rc = plan_reconstruct(c, shards, lens, present, n, data_only, plan);
  if (rc || plan.nothing_to_do || plan.rows.n_out == 0) return rc;
  return run_now(c, plan.rows, plan.in.data(), plan.out.data(), nullptr, plan.len * c->esize(),
                 nullptr);
}

int rse_reconstruct_now(const rse_codec* c, void* const* shards, const size_t* lens,
                        const uint8_t* present, size_t n) {
  return reconstruct_now(c, shards, lens, present, n, false);
}

int rse_reconstruct_data_now(const rse_codec* c, void* const* shards, const size_t* lens,
                             const uint8_t* present, size_t n) {
  return reconstruct_now(c, shards, lens, present, n, true);
}

void rse_dispatcher_stop(void) { rse::dispatch_stop_all(); }

int rse_encode_flat(const rse_codec* c, void* stripes, size_t shard_len, size_t n_stripes,
                    rse_stream_t stream) {
  RSE_ON_STREAM(stream);
  if (!c || !stripes) return RSE_ERR_INVALID_ARGUMENT;
  if (shard_len == 0) return RSE_EMPTY_SHARD;
  if (n_stripes == 0) return RSE_OK;
  const size_t sb = shard_len * c->esize();
  uint8_t* base = static_cast<uint8_t*>(stripes);
  std::vector<const uint8_t*> in(c->k);
  std::vector<uint8_t*> out(c->p);
  for (size_t i = 0; i < c->k; ++i) in[i] = base + i * sb;
  for (size_t r = 0; r < c->p; ++r) out[r] = base + (c->k + r) * sb;
  want_bitslice(c, sb, false, n_stripes);
  const Rows rows = parity_rows(c);
  Job j{c->kfield, &rows, in.data(), out.data(), nullptr, sb, rse::kStore, false, nullptr,
        (uint64_t)c->total * sb, n_stripes};
  return run_job(j, (hipStream_t)stream);
}

int rse_verify_flat(const rse_codec* c, const void* stripes, size_t shard_len, size_t n_stripes,
                    uint8_t* ok, rse_stream_t stream) {
  RSE_ON_STREAM(stream);
  if (!c || !stripes || !ok) return RSE_ERR_INVALID_ARGUMENT;
  if (shard_len == 0) return RSE_EMPTY_SHARD;
  if (n_stripes == 0) return RSE_OK;
  const size_t sb = shard_len * c->esize();
  const uint8_t* base = static_cast<const uint8_t*>(stripes);
  std::vector<const uint8_t*> in(c->k), cmp(c->p);
  for (size_t i = 0; i < c->k; ++i) in[i] = base + i * sb;
  for (size_t r = 0; r < c->p; ++r) cmp[r] = base + (c->k + r) * sb;
  want_bitslice(c, sb, false, n_stripes);
  const Rows rows = parity_rows(c);
  Job j{c->kfield, &rows, in.data(), nullptr, cmp.data(), sb, rse::kCheck, false, nullptr,
        (uint64_t)c->total * sb, n_stripes, true};
  std::vector<int> res;
  try {
    res.resize(n_stripes);
  } catch (const std::bad_alloc&) {
    return RSE_ERR_NO_MEMORY;
  }
  const int rc = run_check(j, (hipStream_t)stream, res.data());
  if (rc == RSE_OK)
    for (size_t s = 0; s < n_stripes; ++s) ok[s] = (uint8_t)res[s];
  return rc;
}

int rse_reconstruct_data_flat(const rse_codec* c, void* stripes, size_t shard_len,
                              size_t n_stripes, const uint8_t* present, rse_stream_t stream) {
  RSE_ON_STREAM(stream);
  if (!c || !stripes || !present) return RSE_ERR_INVALID_ARGUMENT;
  return flat_reconstruct(c, static_cast<uint8_t*>(stripes), shard_len, n_stripes, present, true,
                          (hipStream_t)stream);
}

// Many stripes, each with its own erasure pattern, in two launches: the plan
// (partition + k x k inverse + composed rows, core.rs:733-923) is computed per
// stripe on the device, then every stripe is coded from its descriptor.  No
// host round trip and no decode-matrix cache: a batch of distinct patterns
// costs one inversion per stripe on the GPU instead of one per stripe on the
// host.  Validation happens up front (on the host, or for large batches in a
// device pass before anything is coded), so an error leaves every stripe
// untouched.
// One stripe's validation (core.rs:747-772) and the counts the planners size
// their work by: the highest sigma row + 1 it uses (its syndrome rows R and
// missing parity rows), its missing data shards and its outputs.
int batch_stripe(const uint8_t* pr, size_t k, size_t p, bool data_only, size_t shard_len,
                 uint32_t* need, uint32_t* ne_out, uint32_t* nout) {
  uint32_t ne = 0, nr = 0, nmp = 0, nd = 0;
  for (size_t j = 0; j < k; ++j) ne += pr[j] ? 0u : 1u;
  size_t np = k - ne;
  for (size_t r = 0; r < p; ++r) {
    const bool here = pr[k + r] != 0;
    np += here ? 1 : 0;
    const bool syn = here && nr < ne;
    nr += syn ? 1u : 0u;
    if (!here && !data_only) ++nmp;
    if (syn || (!here && !data_only)) nd = (uint32_t)r + 1;
  }
  if (np && shard_len == 0) return RSE_EMPTY_SHARD;
  if (np < k) return RSE_TOO_FEW_SHARDS_PRESENT;
  *need = nd;
  *ne_out = ne;
  *nout = ne + nmp;
  return RSE_OK;
}

// Batches from this many stripes on are validated on the device (one
// synchronisation instead of a host pass over every flag).
constexpr size_t kDeviceScanStripes = 2048;

int rse_reconstruct_batch(const rse_codec* c, void* stripes, size_t shard_len, size_t n_stripes,
                          const uint8_t* present, int data_only, rse_stream_t stream) {
  RSE_ON_STREAM(stream);
  if (!c || !stripes || !present) return RSE_ERR_INVALID_ARGUMENT;
  if (n_stripes == 0) return RSE_OK;
  const size_t k = c->k, p = c->p, T = c->total, sb = shard_len * c->esize();
  uint8_t* base = static_cast<uint8_t*>(stripes);
  hipStream_t st = (hipStream_t)stream;
  // The flags may live in device memory (a scrubber that found the damage on
  // the GPU): then they are never copied; the scan and the planners read them
  // where they are, and the shared-pattern detection below (a host pass) is
  // skipped.  Paths that need them on the host copy them there.
  int fdev = -1;
  const bool dev_flags = device_memory(present, &fdev);
  if (dev_flags) {
    // device flags must sit on the stripes' device: the scan and the
    // planners read them in place (peer memory would fault or crawl)
    int sdev = -1;
    if (!device_memory(base, &sdev) || sdev != fdev) return RSE_ERR_INVALID_ARGUMENT;
  }
  std::vector<uint8_t> hflags;  // host copy of device flags, made on demand
  auto host_flags = [&](size_t n) -> const uint8_t* {
    if (!dev_flags) return present;
    if (hflags.size() < n * T) {
      hflags.resize(n * T);
      if (hipMemcpy(hflags.data(), present, n * T, hipMemcpyDeviceToHost) != hipSuccess)
        return nullptr;
    }
    return hflags.data();
  };
  // Runs of consecutive stripes with one erasure pattern (a lost disk: every
  // stripe misses the same shards) go through the shared-pattern path: one
  // plan per run, and the pattern's own kernel once it has one (core.rs:
  // 697-731 caches the pattern; used twice, it is specialised), instead of a
  // plan and a mixing per stripe.  Used when the runs are long (at most one
  // run per 16 stripes on average).  Every run is validated before any runs.
  if (!dev_flags) {
    std::vector<std::pair<size_t, size_t>> runs;  // [first, count)
    for (size_t s0 = 0; s0 < n_stripes;) {
      size_t s1 = s0 + 1;
      while (s1 < n_stripes && std::memcmp(present + s1 * T, present + s0 * T, T) == 0) ++s1;
      runs.emplace_back(s0, s1 - s0);
      if (runs.size() * 16 > n_stripes) break;
      // per-stripe patterns show in the first stripes: stop once a prefix
      // holds many runs at over twice the admitted density (this only picks
      // the faster path; both give the same bytes)
      if (runs.size() >= 64 && runs.size() * 8 > s1) break;
      s0 = s1;
    }
    size_t covered = 0;
    for (auto& r : runs) covered += r.second;
    if (covered == n_stripes && runs.size() * 16 <= n_stripes) {
      uint32_t nout_any = 0;
      for (auto& r : runs) {
        uint32_t nd, ne, no;
        const int rc = batch_stripe(present + r.first * T, k, p, data_only != 0, shard_len, &nd,
                                    &ne, &no);
        if (rc) return rc;
        nout_any |= no;
      }
      if (nout_any == 0) return RSE_OK;
      for (auto& r : runs) {
        const int rc = flat_reconstruct(c, base + r.first * T * sb, shard_len, r.second,
                                        present + r.first * T, data_only != 0, st);
        if (rc) return rc;
      }
      return RSE_OK;
    }
  }
  // Validation of every stripe, and the largest counts any stripe needs.
  // The flags go to the device once (the planners read them there); a large
  // batch is validated there too, one lane per stripe.
  uint32_t need = 0, e_cap = 0, nout_cap = 0;
  // The device workspace, the lease's (kept between calls): n_stripes * T
  // flags, the scan's 6 result words, then (bit-sliced path) the per-stripe
  // descriptors.  Every return after work was queued has synchronised the
  // stream, so the lease goes back to the pool idle.
  uint8_t* dflags = nullptr;
  bool ws_owned = false;  // past kPlanKeep: allocated for this call
  const size_t fl_bytes = (n_stripes * T + 255) & ~size_t(255);
  const size_t desc_off = (fl_bytes + 64 + 255) & ~size_t(255);
  const bool fits = k <= (size_t)kMaxIn && p <= (size_t)kMaxOut && n_stripes <= 0xffffffffu;
  const bool bs_path = fits && sb >= 4096 && sb % 16u == 0 && aligned16(base) &&
                       rse::get_option(RSE_OPT_BITSLICE);
  auto release = [&](hipError_t e) {  // after the stream's work on the workspace
    if (dflags && ws_owned) (void)hipFreeAsync(dflags, st);
    dflags = nullptr;
    return e;
  };
  if (shard_len == 0) {  // stripe 0 fails: EmptyShard, or TooFewShardsPresent (none present)
    uint32_t nd, ne, no;
    const uint8_t* f0 = host_flags(1);
    if (!f0) return dev_fail(hipGetLastError());
    return batch_stripe(f0, k, p, data_only != 0, shard_len, &nd, &ne, &no);
  }
  const bool dev_scan = dev_flags || n_stripes >= kDeviceScanStripes;
  if (!dev_scan) {
    for (size_t s = 0; s < n_stripes; ++s) {
      uint32_t nd, ne, no;
      const int rc = batch_stripe(present + s * T, k, p, data_only != 0, shard_len, &nd, &ne, &no);
      if (rc) return rc;
      need = std::max(need, nd);
      e_cap = std::max(e_cap, ne);
      nout_cap = std::max(nout_cap, no);
    }
    if (nout_cap == 0) return RSE_OK;  // nothing this call rebuilds, in any stripe
  }
  Lease lease;
  RSE_HIP(lease.acquire());
  RSE_HIP(lease_plan(lease.get(),
                     desc_off + (bs_path ? n_stripes * sizeof(rse::BsReconArgs) : 0), st,
                     &dflags, &ws_owned));
  const uint8_t* dfl = dev_flags ? present : dflags;  // the flags the device reads
  if (!dev_scan) {
    hipError_t e = hipMemcpyAsync(dflags, present, n_stripes * T, hipMemcpyHostToDevice, st);
    if (e != hipSuccess) return dev_fail(release(e));
  } else {
    // the flags through the lease's pinned words (an asynchronous DMA rather
    // than the runtime's staged pageable copy), the scan's results back into
    // the first words
    // (pinned words only up to 16 MiB of flags: a lease keeps its words, and
    // the pool keeps up to kIdleScratch leases)
    const bool staged = !dev_flags && n_stripes * T <= (size_t(16) << 20);
    hipError_t e = lease_words(lease.get(), 8 + (staged ? (n_stripes * T + 3) / 4 : 0));
    uint32_t* res = reinterpret_cast<uint32_t*>(dflags + fl_bytes);
    if (e == hipSuccess && !dev_flags) {
      if (staged) std::memcpy(lease->wh + 8, present, n_stripes * T);
      e = hipMemcpyAsync(dflags, staged ? static_cast<const void*>(lease->wh + 8) : present,
                         n_stripes * T, hipMemcpyHostToDevice, st);
    }
    if (e == hipSuccess) e = hipMemsetAsync(res, 0, 4 * sizeof(uint32_t), st);
    if (e == hipSuccess) e = hipMemsetAsync(res + 4, 0xFF, 2 * sizeof(uint32_t), st);
    if (e == hipSuccess)
      e = rse::launch_batch_scan(dfl, n_stripes, (uint32_t)k, (uint32_t)p, data_only ? 1u : 0u,
                                 res, st);
    if (e == hipSuccess)
      e = hipMemcpyAsync(lease->wh, res, 6 * sizeof(uint32_t), hipMemcpyDeviceToHost, st);
    if (e == hipSuccess) e = hipStreamSynchronize(st);
    if (e != hipSuccess) {
      (void)hipStreamSynchronize(st);
      return dev_fail(release(e));
    }
    const volatile uint32_t* w = lease->wh;
    need = w[0];
    e_cap = w[1];
    nout_cap = w[2];
    if (((uint64_t)w[5] << 32 | w[4]) != ~0ull) {  // too few shards in some stripe
      (void)release(hipSuccess);
      return RSE_TOO_FEW_SHARDS_PRESENT;
    }
  }
  if (nout_cap == 0) {  // nothing this call rebuilds, in any stripe
    (void)release(hipSuccess);
    RSE_HIP(hipStreamSynchronize(st));
    return RSE_OK;
  }
  size_t done = 0;  // bytes of every shard coded so far
  // host inputs of the copies below: alive until the stream is synchronised
  const Rows prow = parity_rows(c);
  // 1. whole 16 KiB chunks on the bit-sliced syndrome kernels (compiled or
  //    run-time specialised codecs), planned per stripe on the device
  if (bs_path) {
    want_bitslice(c, sb, false, n_stripes);
    if (need > 0) {
      const Rows& rows = prow;
      // the parity rows and the planner's tables: the codec's device copy
      const uint8_t* consts = nullptr;
      int dev = 0;
      hipError_t e = hipGetDevice(&dev);
      if (e == hipSuccess) e = plan_consts(c, dev, &consts);
      if (e != hipSuccess) {
        (void)hipStreamSynchronize(st);  // the flags' copy into the lease may be in flight
        return dev_fail(release(e));
      }
      uint8_t* ws = dflags + desc_off;  // the descriptors
      uint64_t bs_done = 0;
      e = rse::launch_bitslice_recon_batch(
          c->kfield, (uint32_t)k, (uint32_t)p, rows.c.data(),
          reinterpret_cast<const uint16_t*>(consts), consts + plan_tab_off(c), dfl,
          data_only ? 1u : 0u, base, sb, (uint32_t)n_stripes, need, e_cap,
          reinterpret_cast<rse::BsReconArgs*>(ws), st, &bs_done);
      if (e == hipSuccess && bs_done == sb) {
        e = release(hipSuccess);
        if (e == hipSuccess) e = hipStreamSynchronize(st);  // `prow` dies next
      }
      if (e != hipSuccess) {
        (void)hipStreamSynchronize(st);
        return dev_fail(release(e));
      }
      done = bs_done;
    } else {
      (void)release(hipSuccess);
      RSE_HIP(hipStreamSynchronize(st));
      return RSE_OK;  // nothing missing that this call rebuilds, in any stripe
    }
  }
  if (done == sb) return RSE_OK;
  // 2. the rest of every shard (all of it if step 1 did not apply): planned
  //    per stripe on the device (recon_plan_kernel: e x e syndrome inverse,
  //    composed rows as descriptors), coded by the table kernels
  if (T > 0xffffu ||
      rse::recon_plan_lds((uint32_t)k, (uint32_t)T, e_cap, nout_cap) > rse::kReconPlanLdsMax) {
    // past the device planner's LDS budget: the host planner, stripe by stripe
    (void)release(hipSuccess);
    const uint8_t* hfl = host_flags(n_stripes);
    if (!hfl) {
      (void)hipStreamSynchronize(st);
      return dev_fail(hipGetLastError());
    }
    std::vector<void*> ptrs(T);
    std::vector<size_t> lens(T, (sb - done) / c->esize());
    for (size_t s = 0; s < n_stripes; ++s) {
      for (size_t i = 0; i < T; ++i) ptrs[i] = base + (s * T + i) * sb + done;
      int rc = reconstruct_impl(c, ptrs.data(), lens.data(), hfl + s * T, T, data_only != 0, st);
      if (rc) {
        (void)hipStreamSynchronize(st);  // step 1's copies read `prow`
        return rc;
      }
      ++g_host_planned;
    }
    RSE_HIP(hipStreamSynchronize(st));
    return RSE_OK;
  }
  const size_t n_ib = (k + 31) / 32, n_ob = (nout_cap + 15) / 16;
  const size_t per_stripe = n_ib * n_ob * sizeof(CodeArgs);
  // stripes per planning group: descriptors of at most 256 MiB at a time
  const size_t grp = std::max<size_t>(1, std::min<size_t>(n_stripes, (size_t(256) << 20) / per_stripe));
  const uint8_t* consts = nullptr;  // the parity rows on the device (plan_consts)
  uint8_t* ws = nullptr;            // the descriptors
  {
    int dev = 0;
    hipError_t e = hipGetDevice(&dev);
    if (e == hipSuccess) e = plan_consts(c, dev, &consts);
    if (e == hipSuccess) e = hipMallocAsync(reinterpret_cast<void**>(&ws), grp * per_stripe, st);
    if (e != hipSuccess) {
      (void)hipStreamSynchronize(st);  // step 1's work and the flags' copy may be in flight
      return dev_fail(release(e));
    }
  }
  hipError_t e = hipSuccess;
  for (size_t g0 = 0; g0 < n_stripes && e == hipSuccess; g0 += grp) {
    const size_t ng = std::min(grp, n_stripes - g0);
    e = rse::launch_recon_plan(c->kfield, reinterpret_cast<const uint16_t*>(consts), dfl + g0 * T,
                               (uint32_t)k, (uint32_t)T, data_only ? 1u : 0u, e_cap, nout_cap,
                               base + g0 * T * sb, sb, done, sb - done, (uint32_t)ng,
                               reinterpret_cast<CodeArgs*>(ws), st);
  }
  const hipError_t f = hipFreeAsync(ws, st);
  const hipError_t g = release(hipSuccess);
  // `prow` and the caller's flags must outlive the copies that read them
  const hipError_t y = hipStreamSynchronize(st);
  if (e != hipSuccess) return dev_fail(e);
  if (f != hipSuccess) return dev_fail(f);
  if (g != hipSuccess) return dev_fail(g);
  RSE_HIP(y);
  return RSE_OK;
}

int rse_code_shards(int field, const uint8_t* rows, size_t n_out, size_t n_in,
                    const void* const* inputs, void* const* outputs, size_t len, int accumulate,
                    rse_stream_t stream) {
  RSE_ON_STREAM(stream);
  if ((field != RSE_FIELD_GF8 && field != RSE_FIELD_GF16) || !rows || !inputs || !outputs)
    return RSE_ERR_INVALID_ARGUMENT;
  if (n_out == 0 || n_in == 0 || len == 0) return RSE_OK;
  const size_t es = field == RSE_FIELD_GF16 ? 2 : 1;
  Rows r;
  r.n_out = n_out;
  r.n_in = n_in;
  r.c.resize(n_out * n_in);
  for (size_t i = 0; i < n_out * n_in; ++i)
    r.c[i] = es == 2 ? (uint16_t)((rows[2 * i] << 8) | rows[2 * i + 1]) : rows[i];
  Job j{field, &r, reinterpret_cast<const uint8_t* const*>(inputs),
        reinterpret_cast<uint8_t* const*>(outputs), nullptr, len * es, rse::kStore,
        accumulate != 0, nullptr, 0, 1};
  return run_job(j, (hipStream_t)stream);
}

int rse_gf8_mul_slice(uint8_t c, const void* in, void* out, size_t len, int xor_into,
                      rse_stream_t stream) {
  return mul_slice_any(RSE_FIELD_GF8, &c, in, out, len, xor_into != 0, (hipStream_t)stream, false);
}

int rse_code_shards_host(int field, const uint8_t* rows, size_t n_out, size_t n_in,
                         const void* const* inputs, void* const* outputs, size_t len,
                         int accumulate, rse_stream_t stream) {
  RSE_ON_STREAM(stream);
  if ((field != RSE_FIELD_GF8 && field != RSE_FIELD_GF16) || !rows || !inputs || !outputs)
    return RSE_ERR_INVALID_ARGUMENT;
  if (n_out == 0 || n_in == 0 || len == 0) return RSE_OK;
  const size_t es = field == RSE_FIELD_GF16 ? 2 : 1;
  Rows r;
  r.n_out = n_out;
  r.n_in = n_in;
  r.c.resize(n_out * n_in);
  for (size_t i = 0; i < n_out * n_in; ++i)
    r.c[i] = es == 2 ? (uint16_t)((rows[2 * i] << 8) | rows[2 * i + 1]) : rows[i];
  return host_code(field, r, inputs, outputs, len * es, accumulate != 0, (hipStream_t)stream);
}

int rse_encode_sep_host(const rse_codec* c, const void* const* data, const size_t* data_lens,
                        size_t n_data, void* const* parity, const size_t* parity_lens,
                        size_t n_parity, rse_stream_t stream) {
  RSE_ON_STREAM(stream);
  if (!c) return RSE_ERR_INVALID_ARGUMENT;
  return encode_sep_impl(c, data, data_lens, n_data, parity, parity_lens, n_parity,
                         (hipStream_t)stream, true);
}

int rse_encode_single_host(const rse_codec* c, size_t i_data, void* const* shards,
                           const size_t* lens, size_t n, rse_stream_t stream) {
  RSE_ON_STREAM(stream);
  if (!c) return RSE_ERR_INVALID_ARGUMENT;
  int rc;
  if (i_data >= c->k) return RSE_INVALID_INDEX;  // core.rs:552
  if ((rc = check_count(n, c->total, RSE_TOO_FEW_SHARDS, RSE_TOO_MANY_SHARDS))) return rc;
  if (!lens || !shards) return RSE_ERR_INVALID_ARGUMENT;
  if ((rc = check_multi(lens, n))) return rc;
  return encode_single_sep_impl(c, i_data, shards[i_data], lens[i_data], shards + c->k,
                                lens + c->k, c->p, (hipStream_t)stream, true);
}

int rse_encode_single_sep_host(const rse_codec* c, size_t i_data, const void* single,
                               size_t single_len, void* const* parity, const size_t* parity_lens,
                               size_t n_parity, rse_stream_t stream) {
  RSE_ON_STREAM(stream);
  if (!c) return RSE_ERR_INVALID_ARGUMENT;
  return encode_single_sep_impl(c, i_data, single, single_len, parity, parity_lens, n_parity,
                                (hipStream_t)stream, true);
}

// low[n] = c * n and high[n] = c * (n << 4) (build.rs:75-94), so c = low[1].
// Synchronous on a library stream, like the CPU kernel; 0 on error (nothing
// written; rse_last_device_error tells why).
size_t rse_gal_mul(const uint8_t* low, const uint8_t* high, const uint8_t* in, uint8_t* out,
                   size_t len) {
  if (!low || !high || (len && (!in || !out))) return 0;
  return mul_slice_any(RSE_FIELD_GF8, &low[1], in, out, len, false, nullptr, true) == RSE_OK ? len
                                                                                            : 0;
}

size_t rse_gal_mul_xor(const uint8_t* low, const uint8_t* high, const uint8_t* in, uint8_t* out,
                       size_t len) {
  if (!low || !high || (len && (!in || !out))) return 0;
  return mul_slice_any(RSE_FIELD_GF8, &low[1], in, out, len, true, nullptr, true) == RSE_OK ? len
                                                                                           : 0;
}

int rse_gf16_mul_slice(const uint8_t* c, const void* in, void* out, size_t len, int add_into,
                       rse_stream_t stream) {
  return mul_slice_any(RSE_FIELD_GF16, c, in, out, len, add_into != 0, (hipStream_t)stream, false);
}

// Batched device inversion (matrix.rs:195-261 semantics, either field); the
// augmented matrices go to a stream-ordered workspace when they exceed LDS.
static int invert_batch(int field, const void* d_in, void* d_out, uint32_t* d_singular, size_t n,
                        size_t batch, hipStream_t st) {
  const size_t max_n = field == RSE_FIELD_GF8 ? 255 : 4096;
  if (!d_in || !d_out || !d_singular || n == 0 || n > max_n || batch == 0 || batch > 0x7fffffff)
    return RSE_ERR_INVALID_ARGUMENT;
  const size_t w = n * 2 * n * sizeof(uint16_t);
  uint16_t* gws = nullptr;
  if (w > rse::invert_lds_max_bytes()) RSE_HIP(hipMallocAsync(reinterpret_cast<void**>(&gws), w * batch, st));
  hipError_t e = rse::launch_invert(field, static_cast<const uint8_t*>(d_in),
                                    static_cast<uint8_t*>(d_out), d_singular, (uint32_t)n,
                                    (uint32_t)batch, gws, st);
  if (gws) {
    const hipError_t f = hipFreeAsync(gws, st);
    if (e == hipSuccess) e = f;
  }
  RSE_HIP(e);
  return RSE_OK;
}

int rse_gf8_invert_batch(const void* d_in, void* d_out, uint32_t* d_singular, size_t n,
                         size_t batch, rse_stream_t stream) {
  RSE_ON_STREAM(stream);
  return invert_batch(RSE_FIELD_GF8, d_in, d_out, d_singular, n, batch, (hipStream_t)stream);
}

int rse_gf16_invert_batch(const void* d_in, void* d_out, uint32_t* d_singular, size_t n,
                          size_t batch, rse_stream_t stream) {
  RSE_ON_STREAM(stream);
  return invert_batch(RSE_FIELD_GF16, d_in, d_out, d_singular, n, batch, (hipStream_t)stream);
}

int rse_encode_host(const rse_codec* c, void* const* shards, const size_t* lens, size_t n,
                    rse_stream_t stream) {
  RSE_ON_STREAM(stream);
  if (!c) return RSE_ERR_INVALID_ARGUMENT;
  int rc;
  if ((rc = check_count(n, c->total, RSE_TOO_FEW_SHARDS, RSE_TOO_MANY_SHARDS))) return rc;
  if (!lens || !shards) return RSE_ERR_INVALID_ARGUMENT;
  if ((rc = check_multi(lens, n))) return rc;
  for (size_t i = 0; i < n; ++i)
    if (!shards[i]) return RSE_ERR_INVALID_ARGUMENT;
  return host_pipeline(c, HostOp::kEncode, {HostStripe{shards, nullptr, nullptr}},
                       lens[0] * c->esize(), (hipStream_t)stream, nullptr);
}

int rse_encode_host_flat(const rse_codec* c, void* stripes, size_t shard_len, size_t n_stripes,
                         rse_stream_t stream) {
  RSE_ON_STREAM(stream);
  if (!c || !stripes) return RSE_ERR_INVALID_ARGUMENT;
  if (n_stripes == 0) return RSE_OK;
  if (shard_len == 0) return RSE_EMPTY_SHARD;
  const size_t sb = shard_len * c->esize();
  const std::vector<void*> ptrs = flat_ptrs(c, stripes, sb, n_stripes);
  std::vector<HostStripe> list(n_stripes);
  for (size_t s = 0; s < n_stripes; ++s) list[s] = HostStripe{&ptrs[s * c->total], nullptr, nullptr, true};
  return host_pipeline(c, HostOp::kEncode, list, sb, (hipStream_t)stream, nullptr);
}

int rse_verify_host(const rse_codec* c, const void* const* shards, const size_t* lens, size_t n,
                    int* ok, rse_stream_t stream) {
  RSE_ON_STREAM(stream);
  int rc = verify_checks(c, shards, lens, n, nullptr, nullptr, 0, false, ok);
  if (rc) return rc;
  for (size_t i = 0; i < n; ++i)
    if (!shards[i]) return RSE_ERR_INVALID_ARGUMENT;
  return host_pipeline(c, HostOp::kVerify,
                       {HostStripe{const_cast<void* const*>(shards), nullptr, nullptr}},
                       lens[0] * c->esize(), (hipStream_t)stream, ok);
}

int rse_verify_with_buffer_host(const rse_codec* c, const void* const* shards, const size_t* lens,
                                size_t n, void* const* buffer, const size_t* buf_lens,
                                size_t n_buf, int* ok, rse_stream_t stream) {
  RSE_ON_STREAM(stream);
  int rc = verify_checks(c, shards, lens, n, buffer, buf_lens, n_buf, true, ok);
  if (rc) return rc;
  for (size_t i = 0; i < n; ++i)
    if (!shards[i]) return RSE_ERR_INVALID_ARGUMENT;
  for (size_t i = 0; i < n_buf; ++i)
    if (!buffer[i]) return RSE_ERR_INVALID_ARGUMENT;
  return host_pipeline(c, HostOp::kVerifyBuf,
                       {HostStripe{const_cast<void* const*>(shards), buffer, nullptr}},
                       lens[0] * c->esize(), (hipStream_t)stream, ok);
}

int rse_verify_host_flat(const rse_codec* c, const void* stripes, size_t shard_len,
                         size_t n_stripes, uint8_t* ok, rse_stream_t stream) {
  RSE_ON_STREAM(stream);
  if (!c || !stripes || !ok) return RSE_ERR_INVALID_ARGUMENT;
  if (shard_len == 0) return RSE_EMPTY_SHARD;
  if (n_stripes == 0) return RSE_OK;
  const size_t sb = shard_len * c->esize();
  const std::vector<void*> ptrs = flat_ptrs(c, const_cast<void*>(stripes), sb, n_stripes);
  std::vector<HostStripe> list(n_stripes);
  for (size_t s = 0; s < n_stripes; ++s) list[s] = HostStripe{&ptrs[s * c->total], nullptr, nullptr, true};
  std::vector<int> res(n_stripes, 0);
  const int rc = host_pipeline(c, HostOp::kVerify, list, sb, (hipStream_t)stream, res.data());
  if (rc == RSE_OK)
    for (size_t s = 0; s < n_stripes; ++s) ok[s] = (uint8_t)res[s];
  return rc;
}

static int reconstruct_host_impl(const rse_codec* c, void* const* shards, const size_t* lens,
                                 const uint8_t* present, size_t n, bool data_only,
                                 hipStream_t stream) {
  if (!c) return RSE_ERR_INVALID_ARGUMENT;
  ReconPlan plan;  // validation only (core.rs:744-772, lib.rs:185-199): no memory is touched
  int rc = plan_reconstruct(c, shards, lens, present, n, data_only, plan);
  if (rc || plan.nothing_to_do || plan.rows.n_out == 0) return rc;
  return host_pipeline(c, data_only ? HostOp::kReconData : HostOp::kRecon,
                       {HostStripe{shards, nullptr, present}}, plan.len * c->esize(), stream,
                       nullptr);
}

int rse_reconstruct_host(const rse_codec* c, void* const* shards, const size_t* lens,
                         const uint8_t* present, size_t n, rse_stream_t stream) {
  RSE_ON_STREAM(stream);
  return reconstruct_host_impl(c, shards, lens, present, n, false, (hipStream_t)stream);
}

int rse_reconstruct_data_host(const rse_codec* c, void* const* shards, const size_t* lens,
                              const uint8_t* present, size_t n, rse_stream_t stream) {
  RSE_ON_STREAM(stream);
  return reconstruct_host_impl(c, shards, lens, present, n, true, (hipStream_t)stream);
}

int rse_reconstruct_host_batch(const rse_codec* c, void* stripes, size_t shard_len,
                               size_t n_stripes, const uint8_t* present, int data_only,
                               rse_stream_t stream) {
  RSE_ON_STREAM(stream);
  if (!c || !stripes || !present) return RSE_ERR_INVALID_ARGUMENT;
  if (n_stripes == 0) return RSE_OK;
  const size_t k = c->k, T = c->total;
  for (size_t s = 0; s < n_stripes; ++s) {  // core.rs:747-772, stripe by stripe
    size_t np = 0;
    for (size_t i = 0; i < T; ++i) np += present[s * T + i] ? 1 : 0;
    if (np && shard_len == 0) return RSE_EMPTY_SHARD;
    if (np < k) return RSE_TOO_FEW_SHARDS_PRESENT;
  }
  const size_t sb = shard_len * c->esize();
  const std::vector<void*> ptrs = flat_ptrs(c, stripes, sb, n_stripes);
  std::vector<HostStripe> list(n_stripes);
  for (size_t s = 0; s < n_stripes; ++s)
    list[s] = HostStripe{&ptrs[s * T], nullptr, present + s * T, true};
  return host_pipeline(c, data_only ? HostOp::kReconData : HostOp::kRecon, list, sb,
                       (hipStream_t)stream, nullptr);
}

// The keys include/rse_hip.h gives callers; every other settable key is a
// tuning / A-B switch (include/rse_hip_tune.h), refused unless the process
// environment has RSE_TUNE=1.
bool caller_option(int key) {
  switch (key) {
    case RSE_OPT_HOST_CHUNK_KIB: case RSE_OPT_HOST_H2D_STREAMS: case RSE_OPT_JIT:
    case RSE_OPT_JIT_PATTERNS: case RSE_OPT_JIT_DISK_CACHE: case RSE_OPT_JIT_MAX_PATTERNS:
    case RSE_OPT_JIT_MAX_PATTERN_BLOCKS: case RSE_OPT_DISPATCH: case RSE_OPT_DISPATCH_IDLE_US:
    case RSE_OPT_DISPATCH_MAX_BYTES: case RSE_OPT_DISPATCH_WORKGROUPS:
      return true;
    default:
      return false;
  }
}

int rse_set_option(int key, int64_t value) {
  if (!caller_option(key)) {
    const char* t = std::getenv("RSE_TUNE");
    if (!t || std::strcmp(t, "1") != 0) return RSE_ERR_INVALID_ARGUMENT;
  }
  return rse::set_option(key, value) == 0 ? RSE_OK : RSE_ERR_INVALID_ARGUMENT;
}

int64_t rse_get_option(int key) {
  if (key == RSE_OPT_PATTERN_LAUNCHES) return g_pattern_launches;
  if (key == RSE_OPT_SCRATCH_LIVE) return scratch_pool().live.load();
  if (key == RSE_OPT_HOST_PLANNED_STRIPES) return g_host_planned;
  if (key == RSE_OPT_DISPATCHED) return rse::dispatch_count();
  if (key == RSE_OPT_DISPATCH_LAUNCHES) return rse::dispatch_launch_count();
  return rse::get_option(key);
}

int rse_fill_splitmix(void* dst, size_t nbytes, uint64_t seed, uint64_t shard_id,
                      rse_stream_t stream) {
  RSE_ON_STREAM(stream);
  if (!dst && nbytes) return RSE_ERR_INVALID_ARGUMENT;
  RSE_HIP(rse::launch_fill_splitmix(dst, nbytes, seed, shard_id, (hipStream_t)stream));
  return RSE_OK;
}

}  // extern "C"
