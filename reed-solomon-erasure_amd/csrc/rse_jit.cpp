// rse_jit.cpp -- run-time specialisation of the bit-sliced kernels for codecs
// that are not compiled into the library.
//
// The bit-sliced kernels (rse_bitslice_core.hpp) are fastest because every
// coefficient's 8x8 / 16x16 bit matrix is a compile-time constant: the
// multiply-accumulate becomes straight-line v_bitop3 XOR networks.  The
// encoding matrix of ReedSolomon::new (core.rs:430-436) depends only on the
// field and (k, p), so when a codec is created its parity rows are known and a
// module can be built for them: this file turns the rows into the constant
// plane-selection table the kernels take (the same algebra as the constexpr
// Planes of rse_bitslice.hip), appends it and the kernel entry points to the
// device source of rse_bitslice_core.hpp (embedded at build time), and
// compiles that for gfx950 with hiprtc on a background thread.  hiprtc runs on
// the host CPU only; the code object is loaded on a device the first time a
// launch there needs it.  Until the module is ready the table kernels serve the
// codec (RSE_OPT_JIT 1), or the first launch waits for it (RSE_OPT_JIT 2).
// Which kernel runs never changes a result.
#include <dlfcn.h>
#include <hip/hip_runtime.h>
#include <hip/hiprtc.h>
#include <spawn.h>
#include <sys/stat.h>
#include <sys/wait.h>
#include <unistd.h>

#include <array>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cerrno>
#include <csignal>
#include <cstring>
#include <fstream>
#include <sstream>
#include <deque>
#include <cstdio>
#include <cstdlib>
#include <future>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <utility>
#include <vector>

#include "../../include/rse_hip.h"
#include "rse_field.hpp"
#include "rse_kernels.hpp"
#include "rse_netgen.hpp"
#include "rse_wideblk.hpp"

extern char** environ;

namespace rse {
namespace {

// rse_kernels.hpp + rse_device.hpp + rse_bitslice_core.hpp, concatenated with
// their #include "..." lines removed (Makefile: build/rse_jit_src.inc).
const char kJitSource[] =
#include "rse_jit_src.inc"
    ;
// rse_sub_ext.hpp (build/rse_jit_sub.inc): the 1 / 2 KiB-shard body with
// several inputs in flight, for modules built under RSE_OPT_SUB_DEPTH > 1.
const char kJitSubSource[] =
#include "rse_jit_sub.inc"
    ;

struct Compiled {
  bool ok = false;
  std::string code;  // gfx950 code object
  std::string log;
  double ms = 0;
  int wide_w = 0;  // kJitWide: waves per workgroup the module was generated for
  bool wide_half = false;  // kJitWide: 2 KiB chunks per wave (wide_body_half)
};

// Two modules per codec, built in this order: the encode/verify kernel
// (needed first, ~2 s of hiprtc), then the reconstruct kernels (~8 s).
enum Stage { kEnc = 0, kRec = 1 };

struct Entry {
  int field = 0;
  uint32_t k = 0, p = 0;
  std::vector<uint16_t> rows;  // p x k: a codec's parity rows, or a decode pattern's rows
  JitKind kind = kJitCodec;
  bool pattern_block = false;  // a block of a decode pattern's rows (own budget)
  int stages = 2;              // kEnc only (decode pattern, block) or kEnc + kRec (codec)
  std::promise<std::shared_ptr<const Compiled>> promise[2];
  std::shared_future<std::shared_ptr<const Compiled>> built[2];
  std::mutex mu;  // guards loaded
  struct Loaded {
    int dev;
    bool have_rec = false;
    JitFns fns;
    uint32_t wide_cap[3] = {};  // kJitWide: resident workgroups on the device (4 KiB, 1, 2 KiB kernels)
  };
  std::vector<Loaded> loaded;
};

// The registry, the queues and their lock are never destroyed: a thread of
// the host program may still be waiting on a build when the library is
// unloaded at exit (the Worker destructor wakes it), and must find them alive.
std::mutex& g_mu = *new std::mutex;  // guards the registry and the job queues
std::condition_variable& g_cv = *new std::condition_variable;
// Build queues, in priority order: encode modules of codecs and decode
// patterns, reconstruct modules, then wide-codec blocks (many, each seconds of
// hiprtc: they must not delay the modules the narrow codecs wait for).
constexpr int kBlkQueue = 2;
constexpr int kQueues = 3;
std::deque<Entry*>* const g_jobs = new std::deque<Entry*>[kQueues];
int queue_of(const Entry& e, int stage) {
  return (e.kind == kJitBlock || e.kind == kJitBlockAcc || e.kind == kJitWide) ? kBlkQueue : stage;
}
std::atomic<int64_t> g_built{0};
int g_patterns = 0;  // decode-pattern entries (capped: max_patterns)
// per process: RSE_OPT_JIT_MAX_PATTERNS (default 64) decode-pattern modules,
// RSE_OPT_JIT_MAX_PATTERN_BLOCKS (64) blocks of wide decode patterns
int max_patterns() { return (int)std::min<int64_t>(get_option(35), 1 << 30); }
int max_pattern_blocks() { return (int)std::min<int64_t>(get_option(36), 1 << 30); }
int g_blocks = 0;  // wide-codec block entries (capped: kMaxBlocks)
constexpr int kMaxBlocks = 1024;  // 128+128: 64, GF(2^16) 1000+24: 120
// blocks of wide decode patterns: a separate budget, so patterns can never
// use up the codecs' own (and never queue more than a few patterns' builds)
int g_pattern_blocks = 0;
constexpr int kMaxPendingPatternBlocks = 16;
int g_pending_pattern_blocks = 0;  // queued, not yet built
constexpr size_t kMaxPendingPatternJobs = 8;

std::vector<std::unique_ptr<Entry>>& registry() {
  static auto* v = new std::vector<std::unique_ptr<Entry>>;  // never destroyed (see g_mu)
  return *v;
}

bool same_rows(const Entry& e, const uint16_t* rows, size_t stride) {
  for (uint32_t o = 0; o < e.p; ++o)
    for (uint32_t i = 0; i < e.k; ++i)
      if (rows[o * stride + i] != e.rows[o * e.k + i]) return false;
  return true;
}

// Caller holds g_mu.  want >= 0: only entries of that kind match; -2: any
// with encode/verify kernels over CodeArgs (not kJitBlockAcc, not kJitWide).
Entry* find_locked(int field, uint32_t k, uint32_t p, const uint16_t* rows, size_t stride,
                   int want = -1) {
  for (auto& e : registry())
    if (e->field == field && e->k == k && e->p == p &&
        (want == -1 || (want == -2 ? (e->kind != kJitBlockAcc && e->kind != kJitWide)
                                   : e->kind == want)) &&
        same_rows(*e, rows, stride))
      return e.get();
  return nullptr;
}

Entry* find_entry(int field, uint32_t k, uint32_t p, const uint16_t* rows, size_t stride,
                  int want = -1) {
  std::lock_guard<std::mutex> g(g_mu);
  return find_locked(field, k, p, rows, stride, want);
}

// Sigma-row counts of the reconstruct kernels: 1, 2, 4, 8 up to p, and p.
int recon_ns(uint32_t p, int* ns) {
  int n = 0;
  for (int v : {1, 2, 4, 8})
    if ((uint32_t)v <= p) ns[n++] = v;
  if (ns[n - 1] != (int)p) ns[n++] = (int)p;
  return n;
}

// The code struct `name` of p x k rows (rse_netgen.hpp), inside the
// kernels' namespace.
void emit_code(std::string& s, const char* name, int field, uint32_t k, uint32_t p,
               const std::vector<uint16_t>& rows, int temps, bool pairs = false) {
  const netgen::Net net = pairs ? netgen::build_pairs(k, p, rows.data(), temps)
                                : netgen::build(field, k, p, rows.data(), temps, get_option(23) != 0);
  s += "\nnamespace rse {\nnamespace {\n";
  s += netgen::emit(net, name, rows.data());
  s += "}  // namespace\n}  // namespace rse\n";
}

// A wide codec's outputs split over the waves of one workgroup, shares as
// equal as possible (the waves run side by side): W = ceil(p / 8) waves, or
// with RSE_OPT_WIDE_BALANCE (default), for p >= 4, at least 4 and a power of
// two.  A CU's 4 SIMDs then hold equally many of the workgroups' waves (3-wave
// workgroups two to a CU leave two SIMDs with a single wave, which issues VALU
// every 4 cycles at best), and the smaller shares need fewer registers, so
// more waves fit.  Same-box A/B (profiles/r02_wide4/): GF(2^8) 50+20 3.72 TB/s
// in 4 waves vs 3.37 in 3; 10+16 5.07 in 4 vs 4.92 in 2; GF(2^16) 40+12 4.29
// vs 4.18 in 2; 100+30 2.63 in 4 vs 2.54 in 8.
// RSE_OPT_WIDE_SPLIT 0 (auto, the default): 8 outputs per wave, but 4 for
// GF(2^8) codecs past 48 parity rows -- 64+64 in 16 waves of ~120 VGPRs, 4
// per SIMD, against 8 of ~170 at 2 (same box, alternating processes, launches
// in resident workgroups: 2.70-2.73 against 2.55-2.60 TB/s, profiles/r05/s45/
// s64.log; 32+32 and 50+20 are not faster at 4, s32.log, s50.log).
int wide_waves(uint32_t p, int field = 0) {
  uint32_t per = wide_per_wave();
  if (get_option(18) == 0 && field == 8 && p > 48) per = 4;
  int w = (int)((p + per - 1) / per);
  if (get_option(19) != 0 && p >= 4) {
    int b = 4;
    while (b < w) b *= 2;
    if ((uint32_t)b <= p) w = b;
  }
  return w;
}

// Waves per SIMD the wide kernel is compiled for (a lower bound: the compiler
// may use up to 256 VGPRs).  2 by default: asking for 3 makes the scheduler
// spill (GF(2^8) 50+20 in 4 waves: 168 VGPRs and 25 spills at 3, 156 and none
// at 2 -- which runs 3 waves per SIMD all the same).
int wide_waves_per_eu(uint32_t) {
  const int64_t o = get_option(20);  // RSE_OPT_WIDE_OCCUPANCY
  return o ? (int)o : 2;
}
void wide_share(uint32_t p, int W_, int w, uint32_t* o0, uint32_t* n) {
  const uint32_t W = (uint32_t)W_, base = p / W, extra = p % W;
  *o0 = w * base + std::min<uint32_t>(w, extra);
  *n = base + (w < (int)extra ? 1u : 0u);
}

// The device source of one codec: the shared kernel code, the codec's
// plane-selection table, and extern "C" entry points.
std::string make_source(int field, uint32_t k, uint32_t p, const std::vector<uint16_t>& rows,
                        int stage, JitKind kind, int* wide_w = nullptr,
                        bool* wide_half = nullptr) {
  std::string s;
  s.reserve(sizeof(kJitSource) + 1024 + (size_t)8 * k * p * (field == 16 ? 16 : 8));
  // hiprtc has no <stdint.h>: its runtime header declares the fixed-width
  // types in __hip_internal
  s += "#define RSE_JIT 1\n"
       "using __hip_internal::uint8_t;\nusing __hip_internal::uint16_t;\n"
       "using __hip_internal::uint32_t;\nusing __hip_internal::uint64_t;\n"
       "using __hip_internal::int32_t;\n";
#ifdef RSE_TUNE_SPLITS
  // timing split (tools/tune.py's build only, WRONG bytes): wide modules
  // without their workgroup barriers, what the per-round synchronisation costs
  if (kind == kJitWide && get_option(47) == 1) s += "#define __syncthreads() ((void)0)\n";
#endif
  s += kJitSource;
  // RSE_OPT_SUB_DEPTH > 1: the narrow modules' 1 / 2 KiB-shard kernels with
  // that many inputs in flight per wave (rse_sub_ext.hpp)
  const int sub_depth = kind != kJitWide && stage == kEnc ? (int)get_option(50) : 1;
  if (sub_depth > 1) s += kJitSubSource;
  if (kind == kJitWide) {
    // one code struct per wave's share of the outputs, and the kernel (the
    // launch takes W from the build: the options may change meanwhile)
    const int W = wide_waves(p, field);
    if (wide_w) *wide_w = W;
    const bool shared = W > 1 && get_option(14) != 0;  // RSE_OPT_WIDE_LDS
    // GF(2^8) networks over pairs of inputs (RSE_OPT_WIDE_PAIRS): the LDS
    // kernels code a round's inputs two at a time, so W must be even
    const bool pairs = field == 8 && shared && W % 2 == 0 && get_option(29) != 0;
    // RSE_OPT_WIDE_HALF: the paired GF(2^8) networks on 2 KiB chunks, one plane
    // group per lane (rse_bitslice_core.hpp wide_body_half: half the
    // accumulators; 8 outputs per wave no longer spill)
    const bool half = pairs && get_option(38) != 0;
    if (wide_half) *wide_half = half;
    for (int w = 0; w < W; ++w) {
      uint32_t o0, n;
      wide_share(p, W, w, &o0, &n);
      std::vector<uint16_t> sub(rows.begin() + (size_t)o0 * k, rows.begin() + (size_t)(o0 + n) * k);
      char name[32];
      std::snprintf(name, sizeof name, "JitWide%d", w);
      // an input feeds many outputs here: shared temporaries in both fields
      // (GF(2^8): per input or input pair, computed per plane group)
      emit_code(s, name, field, k, n, sub,
                field == 16 ? (int)get_option(13)
                            : std::min(pairs ? 32 : 16, (int)get_option(13)),
                pairs);
    }
    char buf[512];
    std::snprintf(buf, sizeof buf,
                  "struct WideArgs {\n  rse::WideHdr h;\n  const uint8_t* in[%u];\n"
                  "  uint8_t* out[%u];\n  const uint8_t* cmp[%u];\n};\n",
                  k, p, p);
    s += buf;
    // rse_jit_wide over 4 KiB chunks, and _s1 / _s2 over 1 / 2 KiB shards,
    // 4 / 2 stripes per chunk (the bodies' SUB)
    for (int q = 0; q <= 2; ++q) {
      std::snprintf(buf, sizeof buf,
                    // at least 2 waves per SIMD (256 VGPRs): __launch_bounds__ of a
                    // 64-thread group would give 64 VGPRs and spill
                    "extern \"C\" __global__ __attribute__((amdgpu_flat_work_group_size(%d, %d),\n"
                    "    amdgpu_waves_per_eu(%d))) void rse_jit_wide%s(const WideArgs a) {\n"
                    "  __shared__ rse::%s<%d> lds;\n"
                    "  switch (__builtin_amdgcn_readfirstlane(threadIdx.x >> 6)) {\n",
                    64 * W, 64 * W, wide_waves_per_eu(p), q == 0 ? "" : q == 1 ? "_s1" : "_s2",
                    half ? "WideHalfPlanes" : "WidePlanes", W);
      s += buf;
      for (int w = 0; w < W; ++w) {
        uint32_t o0, n;
        wide_share(p, W, w, &o0, &n);
        if (half)
          std::snprintf(buf, sizeof buf,
                        "    case %d: rse::wide_body_half<rse::JitWide%d, %u, %d, %d, %d, "
                        "WideArgs, %du>(a, lds); break;\n",
                        w, w, o0, W, w, (int)get_option(26), 1024 * q);
        else if (shared)
          std::snprintf(buf, sizeof buf,
                        "    case %d: rse::wide_body_lds_deep<rse::JitWide%d, %u, %d, %d, %d, "
                        "WideArgs, %du>(a, lds); break;\n",
                        w, w, o0, W, w, (int)get_option(26), 1024 * q);
        else
          std::snprintf(buf, sizeof buf,
                        "    case %d: rse::wide_body<rse::JitWide%d, %u, WideArgs, %du>(a); "
                        "break;\n",
                        w, w, o0, 1024 * q);
        s += buf;
      }
      s += "    default: break;\n  }\n}\n";
    }
    return s;
  }
  // GF(2^8) temporaries only above 4 outputs (2 waves/SIMD: room for them; at
  // 3 waves/SIMD the extra live sources would cost spills)
  emit_code(s, "JitCode", field, k, p, rows,
            field == 16 ? (int)get_option(13) : p > 4 ? std::min(16, (int)get_option(13)) : 0);
  char buf[512];
  if (stage == kEnc) {
    // encode/verify kernels (16 KiB and 4 KiB chunks); a later block of a wide
    // codec: the same adding to the outputs' bytes instead
    const bool acc = kind == kJitBlockAcc;
    for (int w4 = 0; w4 < 2; ++w4) {
      std::snprintf(buf, sizeof buf,
                    "extern \"C\" __global__ __launch_bounds__(256, %d) void rse_jit_encode%s%s(\n"
                    "    const rse::CodeArgs a, uint64_t cps) {\n"
                    "  rse::bitslice_body<rse::JitCode, true, true, false, false, false, %s, %s>"
                    "(a, cps);\n}\n",
                    p > 4 ? 2 : 3, w4 ? "4" : "", acc ? "_acc" : "", w4 ? "true" : "false",
                    acc ? "true" : "false");
      s += buf;
    }
    if (!acc) {
      // the check kernel of a synchronous verify: the stored parity loaded
      // before un-slicing, and the completion word (rse_device.hpp
      // signal_done) that lets the call return without synchronising
      std::snprintf(buf, sizeof buf,
                    "extern \"C\" __global__ __launch_bounds__(256, %d) void rse_jit_check(\n"
                    "    const rse::CodeArgs a, uint64_t cps) {\n"
                    "  rse::bitslice_body<rse::JitCode, true, true, false, false, false, false, "
                    "false, true>(a, cps);\n  rse::signal_done(a);\n}\n",
                    p > 4 ? 2 : 3);
      s += buf;
      // 1 / 2 KiB shards: 4 / 2 stripes per 4 KiB chunk (bitslice_body SUB)
      for (int q = 1; q <= 2; ++q) {
        if (sub_depth > 1)
          std::snprintf(buf, sizeof buf,
                        "extern \"C\" __global__ __launch_bounds__(256, %d) void rse_jit_encode_s%d(\n"
                        "    const rse::CodeArgs a, uint64_t cps) {\n"
                        "  rse::bitslice_body_sub_deep<rse::JitCode, %d, %du>(a, cps);\n}\n",
                        p > 4 ? 2 : 3, q, sub_depth, 1024 * q);
        else
          std::snprintf(buf, sizeof buf,
                        "extern \"C\" __global__ __launch_bounds__(256, %d) void rse_jit_encode_s%d(\n"
                        "    const rse::CodeArgs a, uint64_t cps) {\n"
                        "  rse::bitslice_body<rse::JitCode, true, true, false, false, false, true, "
                        "false, false, %du>(a, cps);\n}\n",
                        p > 4 ? 2 : 3, q, 1024 * q);
        s += buf;
      }
    }
    return s;
  }
  int ns[5];
  const int n = recon_ns(p, ns);
  const int depth = (int)std::min<int64_t>(3, get_option(27));  // RSE_OPT_RECON_DEPTH
  // 8 sigma rows on wave pairs (RSE_OPT_RECON_PAIRS): 8 KiB units, 3 waves
  // per SIMD; the launchers' grid-stride loops cover either unit size
  // (two pairs per 256-lane workgroup: the launchers' block size)
  const bool pairs = get_option(28) != 0 && depth <= 1 && p >= 8;
  for (int q = 0; q < n; ++q) {
    const int wpe = ns[q] > 4 ? 2 : 3;
    if (pairs && ns[q] == 8) {
      s += "extern \"C\" __global__ __launch_bounds__(256, 3) void rse_jit_recon8(\n"
           "    const rse::BsReconArgs a, uint64_t cps) {\n"
           "  rse::bitslice_recon_pair_body<rse::JitCode, true, 2>(a, cps);\n}\n"
           "extern \"C\" __global__ __launch_bounds__(256, 3) void rse_jit_recon_desc8(\n"
           "    const rse::BsReconArgs* d, uint64_t cps, uint64_t n) {\n"
           "  rse::bitslice_recon_desc_pair_body<rse::JitCode, true, 2>(d, cps, n);\n}\n";
    } else {
      if (depth > 1)
        std::snprintf(buf, sizeof buf,
                      "extern \"C\" __global__ __launch_bounds__(256, %d) void rse_jit_recon%d(\n"
                      "    const rse::BsReconArgs a, uint64_t cps) {\n"
                      "  rse::bitslice_recon_body_deep<rse::JitCode, true, %d, %d>(a, cps);\n}\n",
                      wpe, ns[q], ns[q], depth);
      else
        std::snprintf(buf, sizeof buf,
                      "extern \"C\" __global__ __launch_bounds__(256, %d) void rse_jit_recon%d(\n"
                      "    const rse::BsReconArgs a, uint64_t cps) {\n"
                      "  rse::bitslice_recon_body<rse::JitCode, true, %d, rse::kReconMixDefault>(a, cps);\n}\n",
                      wpe, ns[q], ns[q]);
      s += buf;
      if (depth > 1)
        std::snprintf(buf, sizeof buf,
                      "extern \"C\" __global__ __launch_bounds__(256, %d) void rse_jit_recon_desc%d(\n"
                      "    const rse::BsReconArgs* d, uint64_t cps, uint64_t n) {\n"
                      "  rse::bitslice_recon_desc_body_deep<rse::JitCode, true, %d, %d>(d, cps, n);\n}\n",
                      wpe, ns[q], ns[q], depth);
      else
        std::snprintf(buf, sizeof buf,
                      "extern \"C\" __global__ __launch_bounds__(256, %d) void rse_jit_recon_desc%d(\n"
                      "    const rse::BsReconArgs* d, uint64_t cps, uint64_t n) {\n"
                      "  rse::bitslice_recon_desc_body<rse::JitCode, true, %d>(d, cps, n);\n}\n",
                      wpe, ns[q], ns[q]);
      s += buf;
    }
    std::snprintf(buf, sizeof buf,
                  "extern \"C\" __global__ __launch_bounds__(256, %d) void rse_jit_recon_desc4_%d(\n"
                  "    const rse::BsReconArgs* d, uint64_t cps, uint64_t n, uint64_t base) {\n"
                  "  rse::bitslice_recon_desc_body_w4<rse::JitCode, true, %d>(d, cps, n, base);\n}\n"
                  "extern \"C\" __global__ __launch_bounds__(256, %d) void rse_jit_recon4_%d(\n"
                  "    const rse::BsReconArgs a, uint64_t cps, uint64_t base) {\n"
                  "  rse::bitslice_recon_body_w4<rse::JitCode, true, %d>(a, cps, base);\n}\n",
                  wpe, ns[q], ns[q], wpe, ns[q], ns[q]);
    s += buf;
  }
  return s;
}

// ---------------------------------------------------------------- building
// A module's code object comes from, in order: the on-disk cache (keyed by a
// hash of the library version, the hiprtc options and the complete source --
// the source holds the codec's bit matrices, so equal keys mean equal code);
// the rse_jitc helper process next to the library (several build at once, and
// a build in flight is stopped when the library is unloaded); or hiprtc in
// this process.  Fresh builds are written to the cache (atomic rename), so the
// next process that needs the module loads it in milliseconds.
const char* const kJitOpts[] = {"--offload-arch=gfx950", "-O3", "-std=c++17"};
std::atomic<int64_t> g_cache_hits{0};

std::string hash_key(const std::string& src) {
  uint64_t h1 = 0xcbf29ce484222325ull, h2 = 0x84222325cbf29ce4ull;
  auto mix = [&](const char* p, size_t n) {
    for (size_t i = 0; i < n; ++i) {
      h1 = (h1 ^ (uint8_t)p[i]) * 0x100000001b3ull;
      h2 = (h2 ^ (uint8_t)p[i]) * 0x100000001b3ull + (h2 >> 29);
    }
  };
  const char* ver = rse_version();
  mix(ver, std::strlen(ver));
  for (const char* o : kJitOpts) mix(o, std::strlen(o) + 1);
  mix(src.data(), src.size());
  char buf[40];
  std::snprintf(buf, sizeof buf, "%016llx%016llx", (unsigned long long)h1,
                (unsigned long long)h2);
  return buf;
}

bool make_dirs(const std::string& path) {
  for (size_t i = 1; i <= path.size(); ++i)
    if (i == path.size() || path[i] == '/') {
      const std::string part = path.substr(0, i);
      if (mkdir(part.c_str(), 0755) != 0 && errno != EEXIST) return false;
    }
  return access(path.c_str(), W_OK) == 0;
}

// The cache directory ("" = none): $RSE_JIT_CACHE_DIR, else
// $XDG_CACHE_HOME/rse_hip, else $HOME/.cache/rse_hip.
// (Never destroyed, like the registry: build threads read it until the
// Worker destructor has stopped them, which may run after static strings die.)
const std::string& cache_dir() {
  static const std::string& dir = *new std::string([] {
    std::string d;
    if (const char* e = std::getenv("RSE_JIT_CACHE_DIR")) d = e;
    else if (const char* x = std::getenv("XDG_CACHE_HOME")) d = std::string(x) + "/rse_hip";
    else if (const char* h = std::getenv("HOME")) d = std::string(h) + "/.cache/rse_hip";
    return (!d.empty() && make_dirs(d)) ? d : std::string();
  }());
  return dir;
}

// rse_jitc next to librse_hip.so, if present.
const std::string& helper_path() {
  static const std::string& path = *new std::string([] {
    Dl_info info;
    if (!dladdr(reinterpret_cast<void*>(&hash_key), &info) || !info.dli_fname) return std::string();
    std::string p = info.dli_fname;
    const size_t slash = p.rfind('/');
    p = (slash == std::string::npos ? std::string(".") : p.substr(0, slash)) + "/rse_jitc";
    return access(p.c_str(), X_OK) == 0 ? p : std::string();
  }());
  return path;
}

bool read_file(const std::string& path, std::string* out) {
  std::ifstream f(path, std::ios::binary);
  if (!f) return false;
  std::stringstream ss;
  ss << f.rdbuf();
  *out = ss.str();
  return !out->empty();
}

bool write_file(const std::string& path, const std::string& data) {
  std::ofstream f(path, std::ios::binary | std::ios::trunc);
  f.write(data.data(), (std::streamsize)data.size());
  return f.good();
}

// Children of the build threads (slot per thread), stopped at unload.
constexpr int kMaxBuilders = 8;
std::atomic<pid_t> g_child[kMaxBuilders];
std::atomic<bool> g_unloading{false};

// The helper's source and output files live in a directory private to this
// process (mkdtemp: mode 0700, a fresh name), inside the cache directory when
// there is one (so a finished code object is renamed into the cache on the
// same file system), else in $TMPDIR or /tmp.  Nobody else can plant a
// symlink or swap a file in it between the write and the load.  "" if it
// cannot be made (the builds then run hiprtc in process).  Never destroyed,
// like cache_dir(); removed (when empty) by the Worker destructor.
const std::string& private_dir() {
  static const std::string& dir = *new std::string([] {
    std::string base = cache_dir();
    if (base.empty()) {
      const char* t = std::getenv("TMPDIR");
      base = t && *t ? t : "/tmp";
    }
    std::string tmpl = base + "/rse_jit.XXXXXX";
    return mkdtemp(&tmpl[0]) ? tmpl : std::string();
  }());
  return dir;
}

// Builds src with the helper process (thread slot `slot`); false if it could
// not run or did not finish cleanly (the caller falls back to hiprtc in
// process).  Only the helper's two clean outcomes are final: exit 0 with a
// code object, or exit 1 (the source does not compile, which hiprtc in
// process would repeat).  A helper that cannot start on this system (exit
// 127), dies on a signal or reports an I/O error (exit 2) hands the build
// back -- except at unload, when the build threads kill their helpers on
// purpose and the build completes as failed.
bool build_with_helper(const std::string& src, const std::string& key, int slot, Compiled* out) {
  const std::string& helper = helper_path();
  if (helper.empty()) return false;
  const std::string& dir = private_dir();
  if (dir.empty()) return false;
  // the pid too: a process forked after the first build inherits the same
  // private directory name, and parent and child must not share file paths
  char tag[48];
  std::snprintf(tag, sizeof tag, ".%d.%d", (int)getpid(), slot);
  const std::string src_path = dir + "/" + key + tag + ".hip";
  const std::string out_path = dir + "/" + key + tag + ".co";
  if (!write_file(src_path, src)) return false;
  std::vector<std::string> args = {helper, src_path, out_path};
  for (const char* o : kJitOpts) args.push_back(o);
  std::vector<char*> argv;
  for (auto& a : args) argv.push_back(&a[0]);
  argv.push_back(nullptr);
  pid_t pid = 0;
  if (g_unloading.load()) {  // completes as failed; never handed to in-process hiprtc
    unlink(src_path.c_str());
    out->log = "library unloading";
    return true;
  }
  if (posix_spawn(&pid, helper.c_str(), nullptr, nullptr, argv.data(), environ) != 0) {
    unlink(src_path.c_str());
    return false;
  }
  g_child[slot].store(pid);
  int status = 0;
  pid_t w;
  do {
    w = waitpid(pid, &status, 0);
  } while (w < 0 && errno == EINTR);
  g_child[slot].store(0);
  unlink(src_path.c_str());
  const bool exited = w == pid && WIFEXITED(status);
  if (exited && WEXITSTATUS(status) == 0 && read_file(out_path, &out->code)) {
    out->ok = true;
    if (cache_dir().empty() || get_option(15) == 0 ||
        rename(out_path.c_str(), (cache_dir() + "/" + key + ".co").c_str()) != 0)
      unlink(out_path.c_str());
    return true;
  }
  unlink(out_path.c_str());
  out->code.clear();
  out->log = "rse_jitc failed";
  return (exited && WEXITSTATUS(status) == 1) || g_unloading.load();
}

// In-process hiprtc (no helper, or it could not run).
void build_in_process(const std::string& src, Compiled* out) {
  hiprtcProgram prog;
  if (hiprtcCreateProgram(&prog, src.c_str(), "rse_jit.hip", 0, nullptr, nullptr) !=
      HIPRTC_SUCCESS) {
    out->log = "hiprtcCreateProgram failed";
    return;
  }
  const hiprtcResult r =
      hiprtcCompileProgram(prog, (int)(sizeof kJitOpts / sizeof kJitOpts[0]), kJitOpts);
  size_t n = 0;
  if (hiprtcGetProgramLogSize(prog, &n) == HIPRTC_SUCCESS && n > 1) {
    out->log.assign(n, '\0');
    hiprtcGetProgramLog(prog, &out->log[0]);
  }
  if (r == HIPRTC_SUCCESS && hiprtcGetCodeSize(prog, &n) == HIPRTC_SUCCESS && n > 0) {
    out->code.assign(n, '\0');
    out->ok = hiprtcGetCode(prog, &out->code[0]) == HIPRTC_SUCCESS;
  }
  hiprtcDestroyProgram(&prog);
}

std::shared_ptr<const Compiled> compile(const Entry& e, int stage, int slot) {
  auto out = std::make_shared<Compiled>();
  const std::string src =
      make_source(e.field, e.k, e.p, e.rows, stage, e.kind, &out->wide_w, &out->wide_half);
  const auto t0 = std::chrono::steady_clock::now();
  const std::string key = hash_key(src);
  const bool disk = get_option(15) != 0 && !cache_dir().empty();
  if (disk && read_file(cache_dir() + "/" + key + ".co", &out->code)) {
    out->ok = true;
    ++g_cache_hits;
  } else {
    // at unload (the source can take seconds to generate for a wide codec, so
    // the process may be exiting by now) the build completes as failed
    if (!build_with_helper(src, key, slot, out.get()) && !g_unloading.load()) {
      build_in_process(src, out.get());
      if (out->ok && disk) {  // cache it (atomic: another process may read it)
        const std::string tmp = cache_dir() + "/" + key + "." + std::to_string(getpid()) + ".tmp";
        if (!write_file(tmp, out->code) ||
            rename(tmp.c_str(), (cache_dir() + "/" + key + ".co").c_str()) != 0)
          unlink(tmp.c_str());
      }
    }
    if (out->ok) ++g_built;
  }
  out->ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
  if (const char* dir = std::getenv("RSE_JIT_DUMP")) {  // debugging aid
    char path[1024];
    std::snprintf(path, sizeof path, "%s/rse_jit_gf%d_%u_%u_%s_%p.hip", dir, e.field, e.k, e.p,
                  stage == kEnc ? (e.kind == kJitBlockAcc ? "block_acc"
                                   : e.kind == kJitWide   ? "wide"
                                                          : "encode")
                                : "reconstruct",
                  (const void*)&e);
    if (FILE* f = std::fopen(path, "w")) {
      std::fputs(src.c_str(), f);
      std::fprintf(f, "\n/* %s, %.0f ms\n%s\n*/\n", out->ok ? "ok" : "FAILED", out->ms,
                   out->log.c_str());
      std::fclose(f);
    }
  }
  return out;
}

// Build threads, started with the first registration: several when the
// helper process is available (each runs one rse_jitc at a time), else one
// (comgr serialises in-process compiles anyway).  They take jobs in queue
// priority order.  At library unload the threads are stopped: a helper still
// compiling is killed (its job completes as failed), jobs still queued are
// completed as failed, so nothing waits forever and exit is not held up by a
// build (an in-process hiprtc call, without the helper, still runs to its end).
class Worker {
 public:
  void start() {
    std::lock_guard<std::mutex> g(start_mu_);
    if (!th_.empty()) return;
    int n = 1;
    if (!helper_path().empty()) {
      const unsigned hw = std::thread::hardware_concurrency();
      n = (int)std::max(1u, std::min<unsigned>(kMaxBuilders, hw / 2));
      if (const char* e = std::getenv("RSE_JIT_THREADS")) n = std::max(1, std::min(kMaxBuilders, std::atoi(e)));
    }
    for (int i = 0; i < n; ++i) th_.emplace_back([this, i] { run(i); });
  }
  ~Worker() {
    {
      std::lock_guard<std::mutex> g(g_mu);
      stop_ = true;
    }
    g_unloading.store(true);
    g_cv.notify_all();
    for (auto& c : g_child)
      if (pid_t pid = c.load()) kill(pid, SIGKILL);
    for (auto& t : th_)
      if (t.joinable()) t.join();
    if (!th_.empty() && !private_dir().empty()) rmdir(private_dir().c_str());  // empty by now
    std::lock_guard<std::mutex> g(g_mu);
    for (int q = 0; q < kQueues; ++q) {
      for (Entry* e : g_jobs[q])
        e->promise[q == kRec ? kRec : kEnc].set_value(std::make_shared<Compiled>());
      g_jobs[q].clear();
    }
  }

 private:
  void run(int slot) {
    for (;;) {
      Entry* e = nullptr;
      int stage = 0;
      {
        std::unique_lock<std::mutex> g(g_mu);
        g_cv.wait(g, [&] {
          return stop_ || !g_jobs[kEnc].empty() || !g_jobs[kRec].empty() ||
                 !g_jobs[kBlkQueue].empty();
        });
        if (stop_) return;
        const int q = !g_jobs[kEnc].empty() ? kEnc : !g_jobs[kRec].empty() ? kRec : kBlkQueue;
        stage = q == kRec ? kRec : kEnc;
        e = g_jobs[q].front();
        g_jobs[q].pop_front();
      }
      e->promise[stage].set_value(compile(*e, stage, slot));
      if (e->pattern_block) {
        std::lock_guard<std::mutex> g(g_mu);
        --g_pending_pattern_blocks;
      }
    }
  }
  std::mutex start_mu_;
  std::vector<std::thread> th_;
  bool stop_ = false;
};

Worker& worker() {
  static Worker w;  // constructed after registry(): destroyed (joined) before it
  return w;
}

// Caller holds g_mu; rows[o * stride + i].  Queues the entry's builds.
void add_locked(int field, uint32_t k, uint32_t p, const uint16_t* rows, size_t stride,
                JitKind kind, bool pattern_block = false) {
  auto e = std::make_unique<Entry>();
  e->field = field;
  e->k = k;
  e->p = p;
  e->kind = kind;
  e->pattern_block = pattern_block;
  e->stages = kind == kJitCodec ? 2 : 1;
  e->rows.resize((size_t)k * p);
  for (uint32_t o = 0; o < p; ++o)
    for (uint32_t i = 0; i < k; ++i) e->rows[o * k + i] = rows[o * stride + i];
  for (int st = 0; st < e->stages; ++st) {
    e->built[st] = e->promise[st].get_future().share();
    g_jobs[queue_of(*e, st)].push_back(e.get());
  }
  if (kind == kJitPattern) ++g_patterns;
  // a wide module costs about as much hiprtc as its blocks would: it counts
  // as that many against the same budgets
  const int cost = kind == kJitWide ? (int)(((k + kMaxIn - 1) / kMaxIn) *
                                            ((p + kJitMaxOut - 1) / kJitMaxOut))
                                    : 1;
  if (pattern_block) {
    g_pattern_blocks += cost;
    ++g_pending_pattern_blocks;
  } else if (kind == kJitBlock || kind == kJitBlockAcc || kind == kJitWide) {
    g_blocks += cost;
  }
  registry().push_back(std::move(e));
}

// The blocks of a wide p x k matrix and their kinds, in build order (output
// block by output block, the way run_job launches them).
template <class F>
void for_each_block(uint32_t k, uint32_t p, F&& f) {
  for (uint32_t o0 = 0; o0 < p; o0 += kJitMaxOut)
    for (uint32_t i0 = 0; i0 < k; i0 += (uint32_t)kMaxIn)
      f(o0, i0, std::min<uint32_t>(kJitMaxOut, p - o0), std::min<uint32_t>(kMaxIn, k - i0),
        i0 == 0 ? kJitBlock : kJitBlockAcc);
}

// A caller about to wait for `e`: its queued builds move to the front of
// their queues (a codec waited for is not built after every block queued
// before it).
void promote(Entry* e) {
  std::lock_guard<std::mutex> g(g_mu);
  for (int qi = 0; qi < kQueues; ++qi) {
    std::deque<Entry*>& q = g_jobs[qi];
    for (auto it = q.begin(); it != q.end(); ++it)
      if (*it == e) {
        q.erase(it);
        q.push_front(e);
        break;
      }
  }
}

int status_of(Entry* e, bool wait) {
  if (!e) return 0;
  if (wait) promote(e);
  for (int st = 0; st < e->stages; ++st) {
    if (wait) e->built[st].wait();
    else if (e->built[st].wait_for(std::chrono::seconds(0)) != std::future_status::ready) return 1;
  }
  for (int st = 0; st < e->stages; ++st)
    if (!e->built[st].get()->ok) return -1;
  return 2;
}

// ------------------------------------------ wide modules over input blocks
// A codec too wide for one wide module's argument block (k + 2p >
// kWideMaxPtrs: GF(2^16) past 256 shards, e.g. 1000+24) runs as a chain of
// wide modules over blocks of its inputs, each coding ALL p outputs: block 0
// is rows[:, 0..b0) and stores the outputs; block i > 0 is rows[:, block i]
// followed by the p x p identity over the outputs themselves, so it reads the
// sums so far as p more inputs and stores the new ones (a workgroup reads a
// chunk of an output before it writes the same chunk; no two workgroups share
// one).  Each input is read once and each output read and written once per
// later block, against once per 8-output block and once per 32-input block
// for the kJitBlock modules (~4.5x the algorithmic bytes at 1000+24).
// RSE_OPT_WIDE_BLOCK_INPUTS caps the data inputs per block (hiprtc time grows
// with the module); blocks are balanced.
//
// Past one module's 64 outputs (round 6): the outputs split into balanced
// groups of at most 64, each coded on its own over every input -- one wide
// module when the group fits one (k + 2 np <= 480 and k within
// RSE_OPT_WIDE_BLOCK_INPUTS: GF(2^8) 128+128 is two modules of 128 inputs x 64
// outputs), else a chain as above.  Every input is read once per group and
// every output written once (plus the chain's re-reads), against once per 8
// outputs for the 8 x 32 block modules.
struct WideBlock {
  uint32_t o0, np;              // the output group: outputs o0..o0+np of the codec
  uint32_t i0, ni, kk;          // data inputs i0..i0+ni, module inputs kk (ni, or ni + np)
  bool first;                   // the group's first block (it stores; later ones add)
  std::vector<uint16_t> rows;   // np x kk
};

// A chain's length over k inputs for p outputs, or 0; fits: also when one
// module would hold them (an output group with k past the block limit).
uint32_t chain_len(uint32_t k, uint32_t p, bool fits) {
  const int64_t lim = get_option(46);
  if (lim <= 0 || k == 0 || p == 0 || (!fits && wide_eligible(k, p)) || 3u * p >= kWideMaxPtrs)
    return 0;
  const uint32_t kmax = (uint32_t)std::min<int64_t>(lim, (int64_t)(kWideMaxPtrs - 3u * p));
  const uint32_t n = (k + kmax - 1) / kmax;
  if (n < 2) return 0;
  const uint32_t base = k / n;  // blocks of base or base + 1 inputs
  if (!wide_eligible(base, p) || !wide_eligible(base + p, p) || !wide_eligible(base + 1 + p, p))
    return 0;
  return n;
}

bool wide_blocks_plan_impl(uint32_t k, uint32_t p, uint32_t* nb) {
  const int64_t lim = get_option(46);
  if (lim <= 0 || k == 0 || p == 0 || wide_eligible(k, p) || 3u * p >= kWideMaxPtrs) return false;
  const uint32_t kmax = (uint32_t)std::min<int64_t>(lim, (int64_t)(kWideMaxPtrs - 3u * p));
  const uint32_t n = (k + kmax - 1) / kmax;
  if (n < 2) return false;
  const uint32_t base = k / n;  // blocks of base or base + 1 inputs
  if (!wide_eligible(base, p) || !wide_eligible(base + p, p) || !wide_eligible(base + 1 + p, p))
    return false;
  *nb = n;
  return true;
}

std::vector<WideBlock> wide_blocks_of(uint32_t k, uint32_t p, const uint16_t* rows, uint32_t n,
                                      uint32_t o0 = 0) {
  std::vector<WideBlock> v(n);
  const uint32_t base = k / n, extra = k % n;
  uint32_t i0 = 0;
  for (uint32_t b = 0; b < n; ++b) {
    WideBlock& w = v[b];
    w.o0 = o0;
    w.np = p;
    w.first = b == 0;
    w.i0 = i0;
    w.ni = base + (b < extra ? 1u : 0u);
    w.kk = w.ni + (b ? p : 0u);
    w.rows.assign((size_t)p * w.kk, 0);
    for (uint32_t o = 0; o < p; ++o) {
      for (uint32_t i = 0; i < w.ni; ++i) w.rows[(size_t)o * w.kk + i] = rows[(size_t)o * k + i0 + i];
      if (b) w.rows[(size_t)o * w.kk + w.ni + o] = 1;  // the output's sum so far
    }
    i0 += w.ni;
  }
  return v;
}

// The output groups of a p x k matrix: {o0, np, modules}; false when neither
// the chain of every output nor groups of <= 64 outputs apply.
bool wide_groups_of(uint32_t k, uint32_t p, std::vector<std::array<uint32_t, 3>>* g) {
  g->clear();
  uint32_t nb = 0;
  if (wide_blocks_plan_impl(k, p, &nb)) {  // p <= 64: one chain (round 5, unchanged)
    g->push_back({0u, p, nb});
    return true;
  }
  const int64_t lim = get_option(46);
  if (lim <= 0 || k == 0 || p <= kJitMaxOut * 8u || wide_eligible(k, p)) return false;
  const uint32_t G = (p + kJitMaxOut * 8u - 1) / (kJitMaxOut * 8u), base = p / G, extra = p % G;
  uint32_t o0 = 0;
  for (uint32_t i = 0; i < G; ++i) {
    const uint32_t np = base + (i < extra ? 1u : 0u);
    const uint32_t n = (int64_t)k <= lim && wide_eligible(k, np) ? 1u : chain_len(k, np, true);
    if (n == 0) return false;
    g->push_back({o0, np, n});
    o0 += np;
  }
  return true;
}

// Every module of the plan, group by group.
std::vector<WideBlock> wide_plan_blocks(uint32_t k, uint32_t p, const uint16_t* rows,
                                        const std::vector<std::array<uint32_t, 3>>& g) {
  std::vector<WideBlock> v;
  std::vector<uint16_t> gr;
  for (const auto& x : g) {
    const uint32_t o0 = x[0], np = x[1], n = x[2];
    gr.assign(rows + (size_t)o0 * k, rows + (size_t)(o0 + np) * k);
    if (n == 1) {  // one module over every input
      WideBlock w;
      w.o0 = o0;
      w.np = np;
      w.first = true;
      w.i0 = 0;
      w.ni = k;
      w.kk = k;
      w.rows = gr;
      v.push_back(std::move(w));
    } else {
      std::vector<WideBlock> c = wide_blocks_of(k, np, gr.data(), n, o0);
      for (auto& w : c) v.push_back(std::move(w));
    }
  }
  return v;
}

}  // namespace

int jit_register(int field, uint32_t k, uint32_t p, const uint16_t* rows, JitKind kind) {
  if (get_option(9) == 0 || (field != 8 && field != 16) || k == 0 || k > (uint32_t)kMaxIn ||
      p == 0 || p > kJitMaxOut || (kind == kJitCodec && bitslice_compiled(field, k, p)))
    return 0;
  registry();
  Worker& w = worker();
  std::lock_guard<std::mutex> g(g_mu);
  if (find_locked(field, k, p, rows, k, kind)) return 1;
  // decode patterns are an optimisation: never queue without bound -- except
  // under RSE_OPT_JIT 2, where the caller waits for this very build
  if (kind == kJitPattern &&
      (g_patterns >= max_patterns() ||
       (get_option(9) < 2 && g_jobs[kEnc].size() >= kMaxPendingPatternJobs)))
    return 0;
  if ((kind == kJitBlock || kind == kJitBlockAcc) && g_blocks >= kMaxBlocks) return 0;
  add_locked(field, k, p, rows, k, kind);
  w.start();
  g_cv.notify_all();
  return 1;
}

int jit_register_blocks(int field, uint32_t k, uint32_t p, const uint16_t* rows, bool pattern) {
  if (get_option(9) == 0 || (field != 8 && field != 16) || k == 0 || p == 0) return 0;
  registry();
  Worker& w = worker();
  std::vector<std::array<uint32_t, 3>> groups;
  if (wide_groups_of(k, p, &groups)) {
    const std::vector<WideBlock> bl = wide_plan_blocks(k, p, rows, groups);
    std::lock_guard<std::mutex> g(g_mu);
    int need = 0, pending = 0;
    for (const WideBlock& b : bl)
      if (!find_locked(field, b.kk, b.np, b.rows.data(), b.kk, kJitWide)) {
        need += (int)(((b.kk + kMaxIn - 1) / kMaxIn) * ((b.np + kJitMaxOut - 1) / kJitMaxOut));
        ++pending;
      }
    if (need == 0) return 1;
    if (pattern ? (g_pattern_blocks + need > max_pattern_blocks() ||
                   g_pending_pattern_blocks + pending > kMaxPendingPatternBlocks)
                : g_blocks + need > kMaxBlocks)
      return 0;
    for (const WideBlock& b : bl)
      if (!find_locked(field, b.kk, b.np, b.rows.data(), b.kk, kJitWide))
        add_locked(field, b.kk, b.np, b.rows.data(), b.kk, kJitWide, pattern);
    w.start();
    g_cv.notify_all();
    return 1;
  }
  std::lock_guard<std::mutex> g(g_mu);
  int need = 0;
  for_each_block(k, p, [&](uint32_t o0, uint32_t i0, uint32_t no, uint32_t ni, JitKind kind) {
    need += !find_locked(field, ni, no, rows + (size_t)o0 * k + i0, k, kind);
  });
  if (need == 0) return 1;
  if (pattern ? (g_pattern_blocks + need > max_pattern_blocks() ||
                 g_pending_pattern_blocks + need > kMaxPendingPatternBlocks)
              : g_blocks + need > kMaxBlocks)
    return 0;
  for_each_block(k, p, [&](uint32_t o0, uint32_t i0, uint32_t no, uint32_t ni, JitKind kind) {
    const uint16_t* r = rows + (size_t)o0 * k + i0;
    if (!find_locked(field, ni, no, r, k, kind)) add_locked(field, ni, no, r, k, kind, pattern);
  });
  w.start();
  g_cv.notify_all();
  return 1;
}

uint32_t wide_per_wave() {
  const int64_t v = get_option(18);
  return v >= 2 && v <= (int64_t)kJitMaxOut ? (uint32_t)v : kJitMaxOut;
}

// One module for k > 32 or p > per outputs per wave (RSE_OPT_WIDE_SPLIT), up to
// 8 waves -- or, with fewer outputs per wave than the default 8, up to 16
// waves (1024 lanes) for the same p <= 64 (e.g. 64+64 at 4 outputs per wave).
bool wide_eligible(uint32_t k, uint32_t p) {
  const uint32_t per = wide_per_wave();
  const bool fits = p <= per * 8u || (per < kJitMaxOut && p <= kJitMaxOut * 8u &&
                                      (p + per - 1) / per <= 16u);
  return k >= 1 && p >= 1 && (k > (uint32_t)kMaxIn || p > per) && fits &&
         k + 2u * p <= kWideMaxPtrs;
}

int jit_register_wide(int field, uint32_t k, uint32_t p, const uint16_t* rows, bool pattern) {
  if (get_option(9) == 0 || (field != 8 && field != 16) || !wide_eligible(k, p)) return 0;
  registry();
  Worker& w = worker();
  std::lock_guard<std::mutex> g(g_mu);
  if (find_locked(field, k, p, rows, k, kJitWide)) return 1;
  const int cost = (int)(((k + kMaxIn - 1) / kMaxIn) * ((p + kJitMaxOut - 1) / kJitMaxOut));
  if (pattern ? (g_pattern_blocks + cost > max_pattern_blocks() ||
                 g_pending_pattern_blocks + 1 > kMaxPendingPatternBlocks)
              : g_blocks + cost > kMaxBlocks)
    return 0;
  add_locked(field, k, p, rows, k, kJitWide, pattern);
  w.start();
  g_cv.notify_all();
  return 1;
}

int jit_wide_status(int field, uint32_t k, uint32_t p, const uint16_t* rows, bool wait) {
  return status_of(find_entry(field, k, p, rows, k, kJitWide), wait);
}

hipError_t launch_wide(int field, uint32_t k, uint32_t p, const uint16_t* rows,
                       const uint8_t* const* in, uint8_t* const* out, const uint8_t* const* cmp,
                       uint64_t len, uint64_t stripe_stride, uint32_t n_stripes, uint32_t mode,
                       uint32_t* mismatch, bool per_stripe, hipStream_t stream, uint64_t* done) {
  *done = 0;
  // shards of exactly 1 or 2 KiB: 4 or 2 stripes per 4 KiB chunk (SUB)
  const int subq = (len == 1024u || len == 2048u) && get_option(33) != 0 ? (int)(len / 1024u) : 0;
  const uint64_t cps = len / 4096u;
  if ((cps == 0 && !subq) || n_stripes == 0) return hipSuccess;
  Entry* e = find_entry(field, k, p, rows, k, kJitWide);
  if (!e || status_of(e, get_option(9) >= 2) != 2) return hipSuccess;
  const std::shared_ptr<const Compiled> c = e->built[kEnc].get();
  int dev = 0;
  hipError_t he = hipGetDevice(&dev);
  if (he != hipSuccess) return he;
  hipFunction_t fn = nullptr;
  uint32_t cap = 0;
  {
    std::lock_guard<std::mutex> g(e->mu);
    const Entry::Loaded* have = nullptr;
    for (auto& d : e->loaded)
      if (d.dev == dev) have = &d;
    if (!have) {
      hipModule_t m = nullptr;
      he = hipModuleLoadData(&m, c->code.data());
      if (he == hipSuccess) he = hipModuleGetFunction(&fn, m, "rse_jit_wide");
      if (he != hipSuccess) {
        if (m) (void)hipModuleUnload(m);
        return he;
      }
      Entry::Loaded l{dev};
      l.fns.wide = fn;
      // and the 1 / 2 KiB kernels
      for (int q = 0; q < 2 && he == hipSuccess; ++q)
        he = hipModuleGetFunction(&l.fns.wide_sub[q], m, q ? "rse_jit_wide_s2" : "rse_jit_wide_s1");
      if (he != hipSuccess) {
        (void)hipModuleUnload(m);
        return he;
      }
      // how many workgroups of each kernel the device holds at once
      // (RSE_OPT_WIDE_GRID sizes launches in multiples of it)
      int n_cu = 0;
      if (hipDeviceGetAttribute(&n_cu, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess)
        for (int q = 0; q < 3; ++q) {
          int per = 0;
          const hipFunction_t f = q == 0 ? l.fns.wide : l.fns.wide_sub[q - 1];
          if (hipModuleOccupancyMaxActiveBlocksPerMultiprocessor(&per, f, 64 * c->wide_w, 0) ==
              hipSuccess)
            l.wide_cap[q] = (uint32_t)(per > 0 ? per : 0) * (uint32_t)n_cu;
        }
      e->loaded.push_back(l);
      have = &e->loaded.back();
    }
    fn = subq ? have->fns.wide_sub[subq - 1] : have->fns.wide;
    cap = have->wide_cap[subq];
  }
  // argument block: header, then the k input, p output and p compare pointers
  std::vector<uint8_t> buf(sizeof(WideHdr) + sizeof(void*) * (k + 2 * (size_t)p), 0);
  WideHdr h{};
  h.stripe_stride = stripe_stride;
  h.chunks_per_stripe = cps;
  h.mismatch = mismatch;
  h.n_stripes = n_stripes;
  h.mode = mode;
  h.per_stripe = per_stripe ? 1u : 0u;
  std::memcpy(buf.data(), &h, sizeof h);
  const uint8_t** ptrs = reinterpret_cast<const uint8_t**>(buf.data() + sizeof h);
  for (uint32_t i = 0; i < k; ++i) ptrs[i] = in[i];
  for (uint32_t o = 0; o < p; ++o) {
    ptrs[k + o] = out ? out[o] : nullptr;
    ptrs[k + p + o] = cmp ? cmp[o] : nullptr;
  }
  size_t size = buf.size();
  void* extra[] = {HIP_LAUNCH_PARAM_BUFFER_POINTER, buf.data(), HIP_LAUNCH_PARAM_BUFFER_SIZE, &size,
                   HIP_LAUNCH_PARAM_END};
  // chunks of the module's own size: 4 KiB, or 2 KiB (wide_body_half); with
  // 1 / 2 KiB shards, 4096 (2048) / len stripes per chunk
  const uint64_t cb = c->wide_half ? 2048u : 4096u, spc = cb / (subq ? len : cb);
  const uint64_t total = subq ? (n_stripes + spc - 1) / spc : cps * (4096u / cb) * n_stripes;
  const int64_t grid = get_option(2);
  // tools/tune.py grid sweeps, 128 stripes x 1 MiB (profiles/r04/s2/): GF(2^16)
  // 40+12 16384 workgroups 5.29 TB/s against 5.05 at 4096; GF(2^8) 50+20 flat
  // from 2048 to 8192 (4.72), 4.68 at 16384
  // RSE_OPT_WIDE_GRID m > 0: m x the workgroups the device holds at once;
  // 0 (auto): that once for 1 / 2 KiB shards of codecs with k x p >= 1000,
  // whose launches are a few chunks per workgroup: each workgroup then walks
  // its chunks with the next one's loads in flight instead of a fresh
  // workgroup starting cold (same box, profiles/r05/s45/g*.log: 32+32 x 1 KiB
  // 4.01 -> 4.22 TB/s, 64+64 2.49 -> 2.57, 50+20 4.53 -> 4.58; 16+16 5.78 ->
  // 5.32 and the 1 MiB codecs 5-7 % slower, so not for those); -1 fixed counts
  int64_t mult = get_option(44);
  if (mult == 0) mult = (subq && (uint64_t)k * p >= 1000u) ? 1 : -1;
  uint64_t gx = grid > 0                ? (uint64_t)grid
                : (mult > 0 && cap > 0) ? (uint64_t)mult * cap
                : field == 16           ? 16384u
                                        : 8192u;
  if (gx > total) gx = total;
  if (gx > 0x7fffffffu) gx = 0x7fffffffu;
  const int W = c->wide_w;  // the module's own workgroup shape
  if (subq)
    note_kernel("bitslice-wide gf%d %u+%u w%d%s sub%d", field, k, p, W, c->wide_half ? " half" : "",
                subq);
  else
    note_kernel("bitslice-wide gf%d %u+%u w%d%s", field, k, p, W, c->wide_half ? " half" : "");
  he = hipModuleLaunchKernel(fn, (uint32_t)gx, 1, 1, 64u * (uint32_t)W, 1, 1, 0, stream, nullptr,
                             extra);
  if (he != hipSuccess) return he;
  count_bitslice_launch();
  *done = subq ? len : cps * 4096u;
  return hipSuccess;
}

int jit_blocks_status(int field, uint32_t k, uint32_t p, const uint16_t* rows, bool wait) {
  int worst = 2;
  std::vector<std::array<uint32_t, 3>> groups;
  if (wide_groups_of(k, p, &groups)) {
    for (const WideBlock& b : wide_plan_blocks(k, p, rows, groups)) {
      const int s = status_of(find_entry(field, b.kk, b.np, b.rows.data(), b.kk, kJitWide), wait);
      if (s < worst) worst = s;
      if (worst <= 0) break;
    }
    return worst;
  }
  for_each_block(k, p, [&](uint32_t o0, uint32_t i0, uint32_t no, uint32_t ni, JitKind kind) {
    if (worst <= 0) return;  // one block not registered: the rows are not a wide codec's
    const int s = status_of(find_entry(field, ni, no, rows + (size_t)o0 * k + i0, k, kind), wait);
    if (s < worst) worst = s;
  });
  return worst;
}

bool wide_blocks_plan(uint32_t k, uint32_t p, uint32_t* n_blocks) {
  std::vector<std::array<uint32_t, 3>> groups;
  const bool ok = wide_groups_of(k, p, &groups);
  uint32_t nb = 0;
  for (const auto& x : groups) nb += x[2];
  if (n_blocks) *n_blocks = ok ? nb : 0;
  return ok;
}

hipError_t launch_wide_blocks(int field, uint32_t k, uint32_t p, const uint16_t* rows,
                              const uint8_t* const* in, uint8_t* const* out, uint64_t len,
                              uint64_t stripe_stride, uint32_t n_stripes, hipStream_t stream,
                              uint64_t* done) {
  *done = 0;
  std::vector<std::array<uint32_t, 3>> groups;
  if (!wide_groups_of(k, p, &groups) || n_stripes == 0) return hipSuccess;
  const std::vector<WideBlock> bl = wide_plan_blocks(k, p, rows, groups);
  const bool wait = get_option(9) >= 2;
  for (const WideBlock& b : bl)  // every module built, or none is launched
    if (status_of(find_entry(field, b.kk, b.np, b.rows.data(), b.kk, kJitWide), wait) != 2)
      return hipSuccess;
  std::vector<const uint8_t*> ins;
  uint64_t d0 = 0;
  for (size_t bi = 0; bi < bl.size(); ++bi) {
    const WideBlock& b = bl[bi];
    ins.assign(in + b.i0, in + b.i0 + b.ni);
    if (!b.first) ins.insert(ins.end(), out + b.o0, out + b.o0 + b.np);  // the group's sums so far
    uint64_t d = 0;
    const hipError_t he = launch_wide(field, b.kk, b.np, b.rows.data(), ins.data(), out + b.o0,
                                      nullptr, len, stripe_stride, n_stripes, kStore, nullptr,
                                      false, stream, &d);
    if (he != hipSuccess) return he;
    // every block codes the same whole chunks (same length, every module built)
    if (bi == 0) d0 = d;
    else if (d != d0) return hipErrorInvalidValue;
    if (d0 == 0) return hipSuccess;
  }
  if (groups.size() == 1)
    note_kernel("bitslice-wide-blocks gf%d %u+%u x%u (%u+%u w%d)", field, k, p, groups[0][2],
                bl[0].ni, p, wide_waves(p));
  else
    note_kernel("bitslice-wide-groups gf%d %u+%u g%u x%u (%u+%u w%d)", field, k, p,
                (uint32_t)groups.size(), groups[0][2], bl[0].ni, bl[0].np, wide_waves(bl[0].np));
  *done = d0;
  return hipSuccess;
}

int jit_status(int field, uint32_t k, uint32_t p, const uint16_t* rows, bool wait) {
  return status_of(find_entry(field, k, p, rows, k), wait);
}

bool jit_find(int field, uint32_t k, uint32_t p, const uint16_t* rows, size_t stride, int stage,
              JitFns* out, hipError_t* err, bool acc) {
  *err = hipSuccess;
  const int64_t mode = get_option(9);
  if (mode == 0 || p > kJitMaxOut || (acc && stage != kEnc)) return false;
  Entry* e = find_entry(field, k, p, rows, stride, acc ? (int)kJitBlockAcc : -2);
  if (!e || stage >= e->stages) return false;
  auto& b = e->built[stage];
  if (mode >= 2) {
    promote(e);
    b.wait();
  }
  else if (b.wait_for(std::chrono::seconds(0)) != std::future_status::ready) return false;
  const std::shared_ptr<const Compiled> c = b.get();
  if (!c->ok) return false;
  int dev = 0;
  hipError_t he = hipGetDevice(&dev);
  if (he != hipSuccess) {
    *err = he;
    return false;
  }
  std::lock_guard<std::mutex> g(e->mu);
  Entry::Loaded* l = nullptr;
  for (auto& d : e->loaded)
    if (d.dev == dev) l = &d;
  if (!l) {
    e->loaded.push_back(Entry::Loaded{dev});
    l = &e->loaded.back();
  }
  const bool have = stage == kEnc ? (acc ? l->fns.enc_acc : l->fns.enc) != nullptr : l->have_rec;
  if (!have) {  // load this stage's module on this device; it stays loaded
    hipModule_t m = nullptr;
    he = hipModuleLoadData(&m, c->code.data());
    JitFns f = l->fns;
    if (stage == kEnc) {
      if (acc) {
        if (he == hipSuccess) he = hipModuleGetFunction(&f.enc_acc, m, "rse_jit_encode_acc");
        if (he == hipSuccess) he = hipModuleGetFunction(&f.enc4_acc, m, "rse_jit_encode4_acc");
      } else {
        if (he == hipSuccess) he = hipModuleGetFunction(&f.enc, m, "rse_jit_encode");
        if (he == hipSuccess) he = hipModuleGetFunction(&f.enc4, m, "rse_jit_encode4");
        if (he == hipSuccess) he = hipModuleGetFunction(&f.chk, m, "rse_jit_check");
        if (he == hipSuccess) he = hipModuleGetFunction(&f.sub[0], m, "rse_jit_encode_s1");
        if (he == hipSuccess) he = hipModuleGetFunction(&f.sub[1], m, "rse_jit_encode_s2");
      }
    } else {
      f.n_rec = recon_ns(p, f.rec_ns);
      for (int q = 0; q < f.n_rec && he == hipSuccess; ++q) {
        char name[32];
        std::snprintf(name, sizeof name, "rse_jit_recon%d", f.rec_ns[q]);
        he = hipModuleGetFunction(&f.rec[q], m, name);
        if (he != hipSuccess) break;
        std::snprintf(name, sizeof name, "rse_jit_recon_desc%d", f.rec_ns[q]);
        he = hipModuleGetFunction(&f.rec_desc[q], m, name);
        if (he != hipSuccess) break;
        std::snprintf(name, sizeof name, "rse_jit_recon_desc4_%d", f.rec_ns[q]);
        he = hipModuleGetFunction(&f.rec_desc4[q], m, name);
        if (he != hipSuccess) break;
        std::snprintf(name, sizeof name, "rse_jit_recon4_%d", f.rec_ns[q]);
        he = hipModuleGetFunction(&f.rec4[q], m, name);
      }
    }
    if (he != hipSuccess) {
      if (m) (void)hipModuleUnload(m);
      *err = he;
      return false;
    }
    l->fns = f;
    if (stage == kRec) l->have_rec = true;
  }
  *out = l->fns;
  return true;
}

int64_t jit_modules_built() { return g_built.load(); }
int64_t jit_cache_hits() { return g_cache_hits.load(); }

}  // namespace rse
