// rse_dispatch.hip -- the resident dispatcher of the synchronous small-stripe
// calls (rse_encode_now / rse_verify_now / rse_reconstruct_now, include/rse_hip.h).
//
// Why.  The reference's ReedSolomon::encode (core.rs:597-611) is a synchronous
// CPU call that returns in 0.06-14 us on its own bench's 1-16 KiB blocks
// (benches/bandwidth.rs:88-190).  A kernel launch plus the wait for it costs
// 12 us on MI355X before any work (tools/latency_probe.hip: empty kernel +
// hipStreamSynchronize 12.3 us, + a spin on a pinned word 6.1 us; rse_encode
// of 10+4 x 1 KiB + hipStreamSynchronize 18.5 us), while a round trip to a
// kernel that is already resident and polls pinned host memory is 2.7 us.
// So small calls go to one resident workgroup instead of a launch.
//
// Protocol (one request in flight per device; callers serialise on a mutex):
//  * the request is a run of 16-byte granules in pinned host memory, each
//    {tag, a, b}; the host writes the body, then granule 0, every granule
//    tagged with the request's sequence number;
//  * wave 0 of the resident workgroup reads the first 64 granules with one
//    wave-wide system-coherent load per poll (a PCIe read of 1 KiB: the whole
//    request for codecs up to ~24 coefficient rows x inputs); a request is
//    taken when granule 0 carries a new sequence number and every granule of
//    the request carries it too (a line the host had not written yet when it
//    was read shows the old tag: poll again);
//  * the workgroup builds the coefficients' v_perm tables in LDS, codes (or
//    checks) the shards, drains its stores, and stores {seq, verdict} into a
//    pinned ack word, which the host spins on;
//  * after RSE_OPT_DISPATCH_IDLE_US without a request the kernel stores
//    {last seq, EXIT} and ends, so it never holds the device (a
//    hipDeviceSynchronize waits at most that long for it) and always drains.
//    A host that finds EXIT without its sequence number relaunches; the new
//    kernel takes the pending request (it starts from the last sequence
//    number served).
//
// Memory ordering (MI355X_MICROARCH.md, inter-workgroup visibility).  The
// inputs come from kernels that completed before the call (the contract of
// the *_now entries: the caller has finished writing them), so their bytes
// were released at the end of those kernels.  The consumer side is the
// guide's valid form: one relaxed poll, then ONE agent-scope acquire per
// request on every coding workgroup's CU (its L1 invalidated; the table
// building overlaps the invalidate, which completes at an s_waitcnt vmcnt(0)
// before the workgroup barrier), then the loads.  Outputs are written with
// write-through (sc1) stores and drained (s_waitcnt vmcnt(0)) before the ack,
// so later kernels on any XCD read them from memory.  Only vector stores are
// used.
#include <hip/hip_runtime.h>

#include <atomic>
#include <algorithm>
#include <chrono>
#include <cstring>
#include <mutex>
#include <thread>

#include "rse_device.hpp"
#include "rse_dispatch.hpp"

namespace rse {
namespace {

constexpr int kDispThreads = 512;       // one workgroup, 8 waves (256 VGPRs: no spills)
constexpr int kMaxGranules = 256;       // 4 KiB of request
constexpr uint32_t kDispMaxIn = 64, kDispMaxOut = 64, kDispMaxCoef = 1024;
constexpr uint64_t kAckExit = 1ull << 32, kAckMismatch = 1ull << 33;
constexpr uint32_t kMaxDispWgs = 64, kAckStride = 8;  // one 64-byte line per workgroup's ack
constexpr uint32_t kOpCode = 0, kOpCheck = 1, kOpStop = 2;  // granule 0's a & 0xF

struct alignas(16) Granule {
  uint32_t tag, a;
  uint64_t b;
};

// 16-byte system-coherent loads of pinned host memory (PCIe reads that bypass
// L1 and L2), as vector loads: one request per granule, so a granule is read
// whole (a line the host is writing is seen before or after, never torn).
// The wait is tied to the loaded registers, so no use moves above it.
typedef unsigned dw4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ dw4 load_sys16_nowait(const Granule* g) {
  dw4 v;
  asm volatile("global_load_dwordx4 %0, %1, off sc0 sc1" : "=v"(v) : "v"(g) : "memory");
  return v;
}
__device__ __forceinline__ dw4 load_sys16_wait(const Granule* g) {  // one asm: load + wait
  dw4 v;
  asm volatile("global_load_dwordx4 %0, %1, off sc0 sc1\n\ts_waitcnt vmcnt(0)"
               : "=v"(v)
               : "v"(g)
               : "memory");
  return v;
}
__device__ __forceinline__ void wait_loads(dw4& a, dw4& b, dw4& c) {
  asm volatile("s_waitcnt vmcnt(0)" : "+v"(a), "+v"(b), "+v"(c)::"memory");
}

__device__ __forceinline__ uint64_t now_ticks() {  // 100 MHz constant clock
  return __builtin_amdgcn_s_memrealtime();
}

// Codes one request: items (vector v, output block ob) over the workgroup;
// OB outputs per item.  Pointers and tables are read from LDS (broadcast: the
// lanes of a wave share an output block).  Returns this thread's mismatch
// (check mode).
template <int OB>
__device__ bool code_items(const Granule* req, uint32_t n_in, uint32_t n_out, uint64_t n_vec,
                           bool check, const uint4* tq, const uint32_t* tt, uint32_t n_wg) {
  bool diff = false;
  const uint32_t n_ob = (n_out + OB - 1) / OB;
  const uint64_t items = n_vec * n_ob;
  for (uint64_t it = (uint64_t)blockIdx.x * kDispThreads + threadIdx.x; it < items;
       it += (uint64_t)n_wg * kDispThreads) {
    const uint32_t ob = (uint32_t)(it / n_vec);
    const uint64_t off = (it - (uint64_t)ob * n_vec) * 16u;
    const uint32_t o0 = ob * OB;
    uint4 acc[OB];
#pragma unroll
    for (int o = 0; o < OB; ++o) acc[o] = make_uint4(0u, 0u, 0u, 0u);
    for (uint32_t i0 = 0; i0 < n_in; i0 += 8) {
      uint4 x[8];
#pragma unroll
      for (int j = 0; j < 8; ++j)  // every load of the group in flight at once
        if (i0 + j < n_in)
          x[j] = ld16<true>(reinterpret_cast<const uint8_t*>(req[1 + i0 + j].b) + off);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        if (i0 + j >= n_in) break;
        const Sel s0 = make_sel(x[j].x), s1 = make_sel(x[j].y), s2 = make_sel(x[j].z),
                  s3 = make_sel(x[j].w);
#pragma unroll
        for (int o = 0; o < OB; ++o) {
          if (o0 + o >= n_out) break;
          const Gf8Tab t = read_tab(tq, tt, (int)((o0 + o) * n_in + i0 + j));
          acc[o].x = gf8_mac4(acc[o].x, t, s0);
          acc[o].y = gf8_mac4(acc[o].y, t, s1);
          acc[o].z = gf8_mac4(acc[o].z, t, s2);
          acc[o].w = gf8_mac4(acc[o].w, t, s3);
        }
      }
    }
#pragma unroll
    for (int o = 0; o < OB; ++o) {
      if (o0 + o >= n_out) break;
      uint8_t* p = reinterpret_cast<uint8_t*>(req[1 + n_in + o0 + o].b) + off;
      if (check) {
        const uint4 w = ld16<true>(p);
        diff |= (w.x != acc[o].x) | (w.y != acc[o].y) | (w.z != acc[o].z) | (w.w != acc[o].w);
      } else {
        const dw4 v = {acc[o].x, acc[o].y, acc[o].z, acc[o].w};
        asm volatile("global_store_dwordx4 %0, %1, off sc1" ::"v"(p), "v"(v) : "memory");
      }
    }
  }
  return diff;
}

// The resident workgroups.  ring: the request granules (device view of pinned
// host memory); acks: one pinned ack word per workgroup, kAckStride words
// apart.  seen: the last sequence number served before this launch.
// Workgroup 0 polls the first 64 granules every time (the whole of a small
// request in one PCIe read); the others poll granule 0 alone and read the
// request once its tag is new (a second round trip, but 16 bytes per poll).
// A request names how many workgroups code it (n_wg, the first n_wg); the
// others only take note of it.
__global__ __launch_bounds__(kDispThreads) void rse_dispatch_kernel(const Granule* ring,
                                                                    uint64_t* acks, uint32_t seen,
                                                                    uint64_t idle_ticks) {
  __shared__ Granule req[kMaxGranules];
  __shared__ uint4 tq[kDispMaxCoef];
  __shared__ uint32_t tt[kDispMaxCoef];
  __shared__ uint32_t s_state;  // 0 idle, 1 request in req[], 2 exit, 3 seen, not ours
  __shared__ uint32_t s_diff;
  const uint32_t tid = threadIdx.x, lane = tid & 63u, wave = tid >> 6;
  const bool lead = blockIdx.x == 0;
  uint64_t* ack = acks + (size_t)blockIdx.x * kAckStride;
  uint64_t last = now_ticks();
  uint64_t last_ack = seen;  // thread 0: the last ack stored (seq | mismatch)
  for (;;) {
    if (wave == 0) {
      uint32_t state = 0;
      const dw4 p0 = load_sys16_wait(ring + (lead ? lane : 0u));
      const uint32_t tag0 = __shfl(p0.x, 0);
      if (tag0 != seen) {
        // the request's granules lane, lane + 64, ...
        const dw4 g0 = lead ? p0 : load_sys16_wait(ring + lane);
        const uint32_t tag = __shfl(g0.x, 0);
        const uint32_t n_gran = (__shfl(g0.y, 0) >> 20) & 0xFFFu;
        if (tag == tag0 && n_gran >= 1 && n_gran <= (uint32_t)kMaxGranules) {
          bool ok = lane >= n_gran || g0.x == tag0;
          if (n_gran > 64u) {
            // granules 64..255: three more loads, all lanes (the ring holds
            // 256, so no lane's address is out of bounds), waited for
            // together; the loaded registers are used only inside this block
            // (no phi of an asm output that might be copied before the wait)
            dw4 m0 = load_sys16_nowait(ring + lane + 64u);
            dw4 m1 = load_sys16_nowait(ring + lane + 128u);
            dw4 m2 = load_sys16_nowait(ring + lane + 192u);
            wait_loads(m0, m1, m2);
            ok = ok && (lane + 64u >= n_gran || m0.x == tag0) &&
                 (lane + 128u >= n_gran || m1.x == tag0) && (lane + 192u >= n_gran || m2.x == tag0);
            if (__all(ok)) {  // every granule of the request is this request's
              dw4* q = reinterpret_cast<dw4*>(req);
              q[lane] = g0;
              if (lane + 64u < n_gran) q[lane + 64u] = m0;
              if (lane + 128u < n_gran) q[lane + 128u] = m1;
              if (lane + 192u < n_gran) q[lane + 192u] = m2;
              state = 1;
            }
          } else if (__all(ok)) {
            reinterpret_cast<dw4*>(req)[lane] = g0;
            state = 1;
          }
          if (state == 1) {
            seen = tag0;
            const uint32_t n_wg = (uint32_t)(__shfl(g0.w, 0) >> 16) & 0xFFu;  // b bits 48..55
            if ((__shfl(g0.y, 0) & 0xFu) == kOpStop) state = 2;  // a stop request: end now
            else if (blockIdx.x >= n_wg) state = 3;              // not one of its workgroups
            else __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");  // this CU's L1 invalidated
          }
        }
      }
      if (state == 0 && now_ticks() - last > idle_ticks) state = 2;
      if (lane == 0) {
        s_state = state;
        s_diff = 0;
      }
    }
    __syncthreads();
    const uint32_t state = s_state;
    if (state == 2) break;
    if (state != 1) {
      if (state == 3) last = now_ticks();  // the others are busy: not idle
      __syncthreads();  // s_state is rewritten by wave 0 only after everyone read it
      continue;
    }
    // the request: granule 0 {tag, op | n_in << 4 | n_out << 12 | n_gran << 20,
    // len | n_wg << 48 | outputs per work item << 56},
    // then n_in input and n_out output pointers, then the coefficients (12 per
    // granule, row-major by output, in a then b)
    const uint32_t hdr = req[0].a;
    const bool check = (hdr & 0xFu) == kOpCheck;
    const uint32_t n_in = (hdr >> 4) & 0xFFu, n_out = (hdr >> 12) & 0xFFu;
    const uint64_t len = req[0].b & ((1ull << 48) - 1);
    const uint32_t n_wg = (uint32_t)(req[0].b >> 48) & 0xFFu;
    const uint32_t n_coef = n_in * n_out;
    for (uint32_t c = tid; c < n_coef; c += kDispThreads) {
      const Granule& g = req[1 + n_in + n_out + c / 12u];
      const uint32_t byte = c % 12u;
      const uint32_t coef = byte < 4 ? (g.a >> (8 * byte)) & 0xFFu
                                     : (uint32_t)(g.b >> (8 * (byte - 4))) & 0xFFu;
      const Gf8Tab t = make_gf8_tab(coef);
      write_tab(tq, tt, (int)c, t);
    }
    // the acquire's invalidate has completed before any wave loads an input
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    const uint64_t n_vec = len / 16u;
    // outputs per item: enough items for the threads, at most 8
    const uint32_t ob = (uint32_t)(req[0].b >> 56) & 0xFu;
    bool diff;
    if (ob <= 1) diff = code_items<1>(req, n_in, n_out, n_vec, check, tq, tt, n_wg);
    else if (ob == 2) diff = code_items<2>(req, n_in, n_out, n_vec, check, tq, tt, n_wg);
    else if (ob <= 4) diff = code_items<4>(req, n_in, n_out, n_vec, check, tq, tt, n_wg);
    else diff = code_items<8>(req, n_in, n_out, n_vec, check, tq, tt, n_wg);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every store of this thread landed
    if (diff) atomicOr(&s_diff, 1u);
    __syncthreads();
    if (tid == 0) {
      last_ack = (uint64_t)seen | (s_diff ? kAckMismatch : 0ull);
      __hip_atomic_store(ack, last_ack, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
    last = now_ticks();
    __syncthreads();
  }
  // the exit ack keeps the last request served and its verdict: a host that
  // reads it late still finds its request served
  if (tid == 0) __hip_atomic_store(ack, last_ack | kAckExit, __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_SYSTEM);
}

// ------------------------------------------------------------------- host
struct Dispatcher {
  std::mutex mu;
  bool init = false, running = false;
  bool broken = false;  // a kernel that outlived a timed-out request: not used again
  hipStream_t st = nullptr;
  Granule* req = nullptr;  // pinned, mapped: host view
  Granule* dreq = nullptr;
  uint64_t* ack = nullptr;  // kMaxDispWgs ack words, kAckStride apart
  uint64_t* dack = nullptr;
  uint32_t seq = 0;     // the last request posted
  uint32_t served = 0;  // the last request acknowledged
  uint32_t n_wgs = 1;   // workgroups of the running kernel
};
constexpr int kDispDevs = 64;
Dispatcher& dispatcher(int dev) {
  static Dispatcher* d = new Dispatcher[kDispDevs];  // never destroyed (see rse_codec.cpp pool)
  return d[dev];
}
std::atomic<int64_t> g_dispatched{0}, g_dispatch_launches{0};

}  // namespace

hipError_t side_priority_stream(bool high, hipStream_t* q) {
  int least = 0, greatest = 0;
  if (hipDeviceGetStreamPriorityRange(&least, &greatest) == hipSuccess && least != greatest)
    return hipStreamCreateWithPriority(q, hipStreamNonBlocking, high ? greatest : least);
  (void)hipGetLastError();
  return hipStreamCreateWithFlags(q, hipStreamNonBlocking);
}

namespace {

hipError_t disp_init(Dispatcher& d) {
  if (d.init) return hipSuccess;
  // low priority: not on the hardware queues of the default-priority streams,
  // whose commands the resident kernel would otherwise hold up until it idles
  // out
  hipError_t e = side_priority_stream(false, &d.st);
  if (e == hipSuccess)
    e = hipHostMalloc(reinterpret_cast<void**>(&d.req), sizeof(Granule) * kMaxGranules + 64,
                      hipHostMallocMapped | hipHostMallocCoherent);
  if (e == hipSuccess)
    e = hipHostMalloc(reinterpret_cast<void**>(&d.ack), sizeof(uint64_t) * kAckStride * kMaxDispWgs,
                      hipHostMallocMapped | hipHostMallocCoherent);
  if (e == hipSuccess) e = hipHostGetDevicePointer(reinterpret_cast<void**>(&d.dreq), d.req, 0);
  if (e == hipSuccess) e = hipHostGetDevicePointer(reinterpret_cast<void**>(&d.dack), d.ack, 0);
  if (e != hipSuccess) return e;
  std::memset(d.req, 0, sizeof(Granule) * kMaxGranules);
  std::memset(d.ack, 0, sizeof(uint64_t) * kAckStride * kMaxDispWgs);
  d.init = true;
  return hipSuccess;
}

// A kernel that starts from the last request served (a posted one is new to
// it); the ack starts there too, never at a stale EXIT.
// at_least: the workgroups a pending request names (the option may have
// changed since it was posted).
hipError_t disp_launch(Dispatcher& d, uint32_t at_least = 1) {
  const int64_t g = get_option(45);  // RSE_OPT_DISPATCH_WORKGROUPS
  d.n_wgs = std::max<uint32_t>(at_least,
                               (uint32_t)(g < 1 ? 1 : g > (int64_t)kMaxDispWgs ? kMaxDispWgs : g));
  for (uint32_t w = 0; w < kMaxDispWgs; ++w)
    reinterpret_cast<volatile uint64_t*>(d.ack)[w * kAckStride] = (uint64_t)d.served;
  const int64_t idle_us = get_option(40);
  hipLaunchKernelGGL(rse_dispatch_kernel, dim3(d.n_wgs), dim3(kDispThreads), 0, d.st, d.dreq,
                     d.dack, d.served, (uint64_t)(idle_us < 1 ? 1 : idle_us) * 100u);
  const hipError_t e = hipGetLastError();
  if (e == hipSuccess) {
    d.running = true;
    ++g_dispatch_launches;
  }
  return e;
}

// Posts a stop request (the next sequence number, one granule): workgroups
// that had not taken the pending request never will, one that is coding it
// ends after it.  Called with d.mu held.
void post_stop(Dispatcher& d) {
  const uint32_t seq = d.seq + 1 == 0 ? 1 : d.seq + 1;
  volatile Granule* r = d.req;
  r[0].a = kOpStop | (1u << 20);  // one granule
  r[0].b = 0;
  std::atomic_thread_fence(std::memory_order_release);
  r[0].tag = seq;
  d.seq = seq;
}

// A request that timed out is taken back before the call fails: a stop is
// posted and the kernel is waited for (up to 2 s), so it cannot write the
// caller's outputs after the call has returned.  A kernel that does not end
// marks the dispatcher broken: later calls on the device take the launch
// path.  Called with d.mu held.
void retract(Dispatcher& d) {
  post_stop(d);
  const auto t0 = std::chrono::steady_clock::now();
  while (std::chrono::steady_clock::now() - t0 < std::chrono::seconds(2)) {
    const hipError_t q = hipStreamQuery(d.st);
    if (q != hipErrorNotReady) {
      d.running = false;
      d.served = d.seq;
      return;
    }
    std::this_thread::sleep_for(std::chrono::microseconds(100));
  }
  d.broken = true;
}

}  // namespace

bool dispatch_applies(int field, uint32_t n_in, uint32_t n_out, uint64_t len_bytes,
                      const uint8_t* const* in, uint8_t* const* out) {
  if (!get_option(39) || field != 8 || n_in == 0 || n_out == 0 || n_in > kDispMaxIn ||
      n_out > kDispMaxOut || n_in * n_out > kDispMaxCoef || len_bytes == 0 ||
      len_bytes % 16u != 0 || (int64_t)len_bytes > get_option(41))
    return false;
  const uint32_t n_gran = 1 + n_in + n_out + (n_in * n_out + 11) / 12;
  if (n_gran > (uint32_t)kMaxGranules) return false;
  for (uint32_t i = 0; i < n_in; ++i)
    if (!in[i] || (reinterpret_cast<uintptr_t>(in[i]) & 15u)) return false;
  for (uint32_t o = 0; o < n_out; ++o)
    if (!out[o] || (reinterpret_cast<uintptr_t>(out[o]) & 15u)) return false;
  return true;
}

// outputs = rows x inputs (check: compare with outputs, *mismatch set) on the
// resident workgroup of the current device; synchronous.  dispatch_applies
// must hold.  Returns a hipError_t.
hipError_t dispatch_run(const uint16_t* rows, uint32_t n_in, uint32_t n_out,
                        const uint8_t* const* in, uint8_t* const* out, uint64_t len_bytes,
                        bool check, bool* mismatch) {
  int dev = 0;
  hipError_t e = hipGetDevice(&dev);
  if (e != hipSuccess) return e;
  if (dev < 0 || dev >= kDispDevs) return hipErrorInvalidDevice;
  Dispatcher& d = dispatcher(dev);
  std::lock_guard<std::mutex> g(d.mu);
  if (d.broken) return hipErrorNotSupported;  // the caller takes the launch path
  if ((e = disp_init(d)) != hipSuccess) return e;
  const uint32_t seq = d.seq + 1 == 0 ? 1 : d.seq + 1;  // 0: the zeroed ring
  const uint32_t n_gran = 1 + n_in + n_out + (n_in * n_out + 11) / 12;
  // workgroups that code it: ~RSE_OPT_DISPATCH_LANE_UNITS (1) (16-byte vector,
  // output) units per lane, as
  // many as the running kernel has; outputs per work item: items (vectors x
  // output blocks) for their lanes
  const uint64_t n_vec = len_bytes / 16u;
  if (!d.running) d.n_wgs = (uint32_t)std::min<int64_t>(std::max<int64_t>(get_option(45), 1),
                                                          kMaxDispWgs);
  // (profiles/r05/s10/latency.log, 8 resident, 10+4: 4 KiB 6.6 us on one
  // workgroup against 7.3 on two; 8 / 16 KiB 8.0 / 8.3 us at one unit per
  // lane against 8.4 / 9.2 at two and 8.9 / 10.6 at four)
  const uint64_t units = n_vec * n_out;
  const uint64_t per_wg = (uint64_t)std::max<int64_t>(get_option(49), 1) * kDispThreads;
  const uint32_t n_wg =
      units <= 2u * kDispThreads
          ? 1u  // a request within 2 units per lane of one workgroup stays on it
          : (uint32_t)std::min<uint64_t>(d.n_wgs, (units + per_wg - 1) / per_wg);
  const uint64_t lanes = (uint64_t)n_wg * kDispThreads;
  uint32_t ob = 1;
  while (ob < 8 && n_vec * ((n_out + 2 * ob - 1) / (2 * ob)) >= lanes) ob *= 2;
  volatile Granule* r = d.req;
  for (uint32_t i = 0; i < n_in; ++i) {
    r[1 + i].a = 0;
    r[1 + i].b = reinterpret_cast<uint64_t>(in[i]);
  }
  for (uint32_t o = 0; o < n_out; ++o) {
    r[1 + n_in + o].a = 0;
    r[1 + n_in + o].b = reinterpret_cast<uint64_t>(out[o]);
  }
  const uint32_t nc = n_in * n_out, cg0 = 1 + n_in + n_out;
  for (uint32_t q = 0; q * 12 < nc; ++q) {
    uint8_t b[12] = {};
    for (uint32_t j = 0; j < 12 && q * 12 + j < nc; ++j) b[j] = (uint8_t)rows[q * 12 + j];
    uint32_t a;
    uint64_t w;
    std::memcpy(&a, b, 4);
    std::memcpy(&w, b + 4, 8);
    r[cg0 + q].a = a;
    r[cg0 + q].b = w;
  }
  for (uint32_t q = 1; q < n_gran; ++q) r[q].tag = seq;
  r[0].a = (check ? kOpCheck : kOpCode) | (n_in << 4) | (n_out << 12) | (n_gran << 20);
  r[0].b = len_bytes | ((uint64_t)n_wg << 48) | ((uint64_t)ob << 56);
  std::atomic_thread_fence(std::memory_order_release);
  r[0].tag = seq;  // the request is posted
  d.seq = seq;
  if (!d.running) {
    if ((e = disp_launch(d, n_wg)) != hipSuccess) return e;
  }
  // every coding workgroup's ack.  A workgroup that idled out before it saw
  // the request (EXIT without this seq): wait for the whole kernel to end and
  // launch again -- the new one serves the request in full (coding it twice
  // writes the same bytes: no request's inputs are its outputs).
  const volatile uint64_t* ack = d.ack;
  const auto t0 = std::chrono::steady_clock::now();
  bool mm = false;
  for (uint32_t w = 0; w < n_wg;) {
    for (uint64_t n = 1;; ++n) {
      const uint64_t a = ack[w * kAckStride];
      if ((uint32_t)a == seq) {  // served (an exit ack keeps the last request served)
        mm = mm || (a & kAckMismatch) != 0;
        ++w;
        break;
      }
      bool again = (a & kAckExit) != 0;
      if (!again) {
        __builtin_ia32_pause();
        if ((n & 4095u) != 0) continue;
        // a launch that failed, or a kernel that died, ends the wait
        const hipError_t q = hipStreamQuery(d.st);
        if (q != hipErrorNotReady && q != hipSuccess) return q;
        again = q == hipSuccess && ack[w * kAckStride] == a;  // ended without our ack
        if (std::chrono::steady_clock::now() - t0 > std::chrono::seconds(10)) {
          retract(d);
          return hipErrorLaunchTimeOut;
        }
        if (!again) continue;
      }
      if ((e = hipStreamSynchronize(d.st)) != hipSuccess) return e;
      d.running = false;
      if ((e = disp_launch(d, n_wg)) != hipSuccess) return e;
      w = 0;  // every workgroup again
      mm = false;
      break;
    }
  }
  d.served = seq;
  if (mismatch) *mismatch = mm;
  ++g_dispatched;
  return hipSuccess;
}

// Ends the resident kernel of every device this process started one on: a
// stop request (it would also end by itself after RSE_OPT_DISPATCH_IDLE_US).
void dispatch_stop_all() {
  for (int dev = 0; dev < kDispDevs; ++dev) {
    Dispatcher& d = dispatcher(dev);
    std::lock_guard<std::mutex> g(d.mu);
    if (!d.init || !d.running || d.broken) continue;
    int cur = 0;
    if (hipGetDevice(&cur) != hipSuccess) continue;
    if (cur != dev && hipSetDevice(dev) != hipSuccess) continue;
    post_stop(d);
    (void)hipStreamSynchronize(d.st);  // it takes the stop (or has idled out)
    d.served = d.seq;
    d.running = false;
    if (cur != dev) (void)hipSetDevice(cur);
  }
}

int64_t dispatch_count() { return g_dispatched.load(); }
int64_t dispatch_launch_count() { return g_dispatch_launches.load(); }

}  // namespace rse
