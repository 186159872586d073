// Floor of one synchronous small call on MI355X, by mechanism: what a drop-in
// caller of ReedSolomon::encode (core.rs:597-611) on 1 KiB shards waits for.
//   A  empty kernel launch + hipStreamSynchronize
//   B  empty kernel launch that stores a word of pinned host memory, host spins on it
//   C  rse_encode 10+4 x 1 KiB + hipStreamSynchronize
//   D  rse_encode 10+4 x 1 KiB enqueue only (no wait)
//   E  round trip to a resident kernel: host writes a sequence number into pinned
//      memory, one lane of the resident kernel polls it and stores it back
//   F  hipStreamQuery on an idle stream
//   G  rse_encode 10+4 x 1 KiB + hipStreamWriteValue32 of a pinned word, host spins
//   H  empty kernel + hipStreamWriteValue32, host spins
//   I  rse_encode_now 10+4 x 1 KiB (the resident dispatcher)
//   J  rse_encode_now by shard size: 1, 8, 32 dispatcher workgroups, and the launch path
//   K  rse_encode_now 4-64 KiB: 8 / 16 resident workgroups, 1 / 2 / 4 units per lane
//   L  rse_encode_now back to back, and each followed by hipDeviceSynchronize, by idle time
//   M  a kernel on another stream + its synchronisation between rse_encode_now calls
// argv[1] (optional): the letters of the cases to run.
// The resident kernel of E exits on a stop value or after a bounded number of
// polls, so it always drains.
//   hipcc --offload-arch=gfx950 -O2 -I include tools/latency_probe.hip \
//     -L reed-solomon-erasure_amd/reed_solomon_erasure -lrse_hip \
//     -Wl,-rpath,$PWD/reed-solomon-erasure_amd/reed_solomon_erasure -o tools/bin/latency_probe
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "rse_hip.h"

#define CK(x)                                                              \
  do {                                                                     \
    hipError_t e_ = (x);                                                   \
    if (e_ != hipSuccess) {                                                \
      std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      std::exit(2);                                                        \
    }                                                                      \
  } while (0)

__global__ void empty_kernel(uint32_t* word, uint32_t v) {
  if (word && threadIdx.x == 0 && blockIdx.x == 0)
    __hip_atomic_store(word, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

constexpr uint32_t kStop = 0xFFFFFFFFu;

// One lane polls db; every new value is stored back into ack.  Exits on kStop
// or after max_polls polls (each a PCIe round trip of ~1 us or more).
__global__ void responder(const uint32_t* db, uint32_t* ack, uint64_t max_polls) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  uint32_t seen = 0;
  for (uint64_t i = 0; i < max_polls; ++i) {
    const uint32_t s = __hip_atomic_load(db, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    if (s == kStop) break;
    if (s != seen) {
      seen = s;
      __hip_atomic_store(ack, s, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
  }
  __hip_atomic_store(ack, kStop, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

using clk = std::chrono::steady_clock;
double us_since(clk::time_point t0) {
  return std::chrono::duration<double, std::micro>(clk::now() - t0).count();
}

// Spins until *w == want; exits the probe after 2 s without it (no hang).
void spin(volatile uint32_t* w, uint32_t want, const char* what) {
  const auto lim = clk::now() + std::chrono::seconds(2);
  while (*w != want)
    if (clk::now() > lim) {
      std::printf("%s: the word never arrived\n", what);
      std::exit(6);
    }
}

struct Stat {
  std::vector<double> v;
  void report(const char* name) {
    std::sort(v.begin(), v.end());
    double s = 0;
    for (double x : v) s += x;
    std::printf("%-58s mean %7.2f  p50 %7.2f  p10 %7.2f  p90 %7.2f us (n=%zu)\n", name,
                s / v.size(), v[v.size() / 2], v[v.size() / 10], v[v.size() * 9 / 10], v.size());
  }
};

static const char* g_cases = nullptr;  // argv[1]: the case letters to run (all when absent)
bool want(char c) { return !g_cases || std::strchr(g_cases, c); }

int main(int argc, char** argv) {
  if (argc > 1) g_cases = argv[1];
  const int reps = 2000;
  hipStream_t st;
  CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
  uint32_t* hw = nullptr;  // [0] word for B, [16] doorbell, [32] ack (separate lines)
  CK(hipHostMalloc(reinterpret_cast<void**>(&hw), 4096, hipHostMallocCoherent | hipHostMallocMapped));
  volatile uint32_t* vw = hw;
  for (int i = 0; i < 1024; ++i) hw[i] = 0;
  uint32_t* dw = nullptr;
  CK(hipHostGetDevicePointer(reinterpret_cast<void**>(&dw), hw, 0));

  if (want('A')) {  // A
    Stat s;
    for (int i = 0; i < reps + 50; ++i) {
      const auto t0 = clk::now();
      hipLaunchKernelGGL(empty_kernel, dim3(1), dim3(64), 0, st, nullptr, 0u);
      CK(hipStreamSynchronize(st));
      if (i >= 50) s.v.push_back(us_since(t0));
    }
    s.report("A empty kernel + hipStreamSynchronize");
  }
  if (want('B')) {  // B
    Stat s;
    for (int i = 0; i < reps + 50; ++i) {
      const uint32_t want = (uint32_t)i + 1;
      const auto t0 = clk::now();
      hipLaunchKernelGGL(empty_kernel, dim3(1), dim3(64), 0, st, dw, want);
      spin(&vw[0], want, "B");
      if (i >= 50) s.v.push_back(us_since(t0));
    }
    CK(hipStreamSynchronize(st));
    s.report("B empty kernel, host spins on a pinned word");
  }
  if (want('H')) {  // H: empty kernel + stream memory write, host spins
    Stat s;
    for (int i = 0; i < reps + 50; ++i) {
      const uint32_t want = 0x20000u + (uint32_t)i;
      const auto t0 = clk::now();
      hipLaunchKernelGGL(empty_kernel, dim3(1), dim3(64), 0, st, nullptr, 0u);
      CK(hipStreamWriteValue32(st, dw + 64, want, 0));
      spin(&vw[64], want, "H");
      if (i >= 50) s.v.push_back(us_since(t0));
    }
    CK(hipStreamSynchronize(st));
    s.report("H empty kernel + hipStreamWriteValue32, host spins");
  }
  if (want('C')) {  // C, D
    rse_codec* c = nullptr;
    if (rse_codec_new(RSE_FIELD_GF8, 10, 4, &c)) return 3;
    const size_t L = 1024, T = 14;
    uint8_t* buf = nullptr;
    CK(hipMalloc(reinterpret_cast<void**>(&buf), T * L));
    CK(hipMemset(buf, 7, T * L));
    std::vector<void*> sh(T);
    std::vector<size_t> lens(T, L);
    for (size_t i = 0; i < T; ++i) sh[i] = buf + i * L;
    Stat s, d;
    for (int i = 0; i < reps + 50; ++i) {
      const auto t0 = clk::now();
      if (rse_encode(c, sh.data(), lens.data(), T, st)) return 4;
      CK(hipStreamSynchronize(st));
      if (i >= 50) s.v.push_back(us_since(t0));
    }
    s.report("C rse_encode 10+4 x 1 KiB + hipStreamSynchronize");
    {  // G: completion by a stream memory write, host spins
      Stat g;
      for (int i = 0; i < reps + 50; ++i) {
        const uint32_t want = 0x10000u + (uint32_t)i;
        const auto t0 = clk::now();
        if (rse_encode(c, sh.data(), lens.data(), T, st)) return 4;
        CK(hipStreamWriteValue32(st, dw + 48, want, 0));
        spin(&vw[48], want, "G");
        if (i >= 50) g.v.push_back(us_since(t0));
      }
      CK(hipStreamSynchronize(st));
      g.report("G rse_encode + hipStreamWriteValue32, host spins");
    }
    {  // I: the synchronous entry (resident dispatcher)
      Stat g;
      for (int i = 0; i < reps + 50; ++i) {
        const auto t0 = clk::now();
        if (rse_encode_now(c, sh.data(), lens.data(), T)) return 4;
        if (i >= 50) g.v.push_back(us_since(t0));
      }
      g.report("I rse_encode_now 10+4 x 1 KiB (returns when done)");
      std::printf("   dispatched %lld, dispatcher launches %lld\n",
                  (long long)rse_get_option(RSE_OPT_DISPATCHED),
                  (long long)rse_get_option(RSE_OPT_DISPATCH_LAUNCHES));
    }
    for (int i = 0; i < reps + 50; ++i) {
      const auto t0 = clk::now();
      if (rse_encode(c, sh.data(), lens.data(), T, st)) return 4;
      if (i >= 50) d.v.push_back(us_since(t0));
      if (i % 64 == 63) CK(hipStreamSynchronize(st));
    }
    CK(hipStreamSynchronize(st));
    d.report("D rse_encode 10+4 x 1 KiB, enqueue only");
    std::printf("   kernel: %s\n", rse_last_kernel());
    rse_codec_free(c);
    CK(hipFree(buf));
  }
  if (want('J')) {  // J: rse_encode_now by shard size and dispatcher workgroups, against the launch path
    rse_codec* c = nullptr;
    if (rse_codec_new(RSE_FIELD_GF8, 10, 4, &c)) return 3;
    const size_t T = 14, Lmax = 1u << 20;
    uint8_t* buf = nullptr;
    CK(hipMalloc(reinterpret_cast<void**>(&buf), T * Lmax));
    CK(hipMemset(buf, 7, T * Lmax));
    rse_set_option(RSE_OPT_DISPATCH_MAX_BYTES, (int64_t)Lmax);
    for (size_t L : {1024u, 4096u, 16384u, 65536u, 262144u, 1048576u}) {
      std::vector<void*> sh(T);
      std::vector<size_t> lens(T, L);
      for (size_t i = 0; i < T; ++i) sh[i] = buf + i * L;
      char name[96];
      for (int wgs : {1, 8, 32, 0}) {
        Stat g;
        if (wgs) {
          rse_set_option(RSE_OPT_DISPATCH, 1);
          rse_set_option(RSE_OPT_DISPATCH_WORKGROUPS, wgs);
          rse_dispatcher_stop();  // the next call launches with this many
        } else {
          rse_set_option(RSE_OPT_DISPATCH, 0);  // the launch path, waited for
        }
        const int n = L >= 262144 ? 300 : 1000;
        for (int i = 0; i < n + 20; ++i) {
          const auto t0 = clk::now();
          if (rse_encode_now(c, sh.data(), lens.data(), T)) return 4;
          if (i >= 20) g.v.push_back(us_since(t0));
        }
        if (wgs) std::snprintf(name, sizeof name, "J encode_now 10+4 x %zu KiB, %d workgroups", L >> 10, wgs);
        else std::snprintf(name, sizeof name, "J encode_now 10+4 x %zu KiB, launch path", L >> 10);
        g.report(name);
      }
    }
    rse_set_option(RSE_OPT_DISPATCH, 1);
    rse_set_option(RSE_OPT_DISPATCH_WORKGROUPS, 8);
    rse_set_option(RSE_OPT_DISPATCH_MAX_BYTES, 32768);
    rse_dispatcher_stop();
    rse_codec_free(c);
    CK(hipFree(buf));
  }
  if (want('K')) {  // K: workgroups per request (RSE_OPT_DISPATCH_LANE_UNITS) at 8 and 16 resident ones
    rse_codec* c = nullptr;
    if (rse_codec_new(RSE_FIELD_GF8, 10, 4, &c)) return 3;
    const size_t T = 14, Lmax = 1u << 16;
    uint8_t* buf = nullptr;
    CK(hipMalloc(reinterpret_cast<void**>(&buf), T * Lmax));
    CK(hipMemset(buf, 7, T * Lmax));
    rse_set_option(RSE_OPT_DISPATCH, 1);
    rse_set_option(RSE_OPT_DISPATCH_MAX_BYTES, (int64_t)Lmax);
    for (int wgs : {8, 16}) {
      rse_set_option(RSE_OPT_DISPATCH_WORKGROUPS, wgs);
      rse_dispatcher_stop();
      for (size_t L : {4096u, 8192u, 16384u, 32768u, 65536u}) {
        std::vector<void*> sh(T);
        std::vector<size_t> lens(T, L);
        for (size_t i = 0; i < T; ++i) sh[i] = buf + i * L;
        for (int u : {1, 2, 4}) {
          rse_set_option(RSE_OPT_DISPATCH_LANE_UNITS, u);
          Stat g;
          for (int i = 0; i < 1020; ++i) {
            const auto t0 = clk::now();
            if (rse_encode_now(c, sh.data(), lens.data(), T)) return 4;
            if (i >= 20) g.v.push_back(us_since(t0));
          }
          char name[96];
          std::snprintf(name, sizeof name, "K encode_now 10+4 x %zu KiB, %d resident, %d units/lane",
                        L >> 10, wgs, u);
          g.report(name);
        }
      }
    }
    rse_set_option(RSE_OPT_DISPATCH_LANE_UNITS, 2);
    rse_set_option(RSE_OPT_DISPATCH_WORKGROUPS, 8);
    rse_set_option(RSE_OPT_DISPATCH_MAX_BYTES, 65536);
    rse_dispatcher_stop();
    rse_codec_free(c);
    CK(hipFree(buf));
  }
  if (want('E')) {  // E
    hipStream_t rs;
    CK(hipStreamCreateWithFlags(&rs, hipStreamNonBlocking));
    volatile uint32_t* db = vw + 16;
    volatile uint32_t* ack = vw + 32;
    hipLaunchKernelGGL(responder, dim3(1), dim3(64), 0, rs, dw + 16, dw + 32, (uint64_t)20000000);
    CK(hipGetLastError());
    Stat s;
    bool ok = true;
    for (int i = 0; i < reps + 50 && ok; ++i) {
      const uint32_t want = (uint32_t)i + 1;
      const auto t0 = clk::now();
      *db = want;
      const auto lim = clk::now() + std::chrono::seconds(2);
      while (*ack != want) {
        if (*ack == kStop || clk::now() > lim) {
          ok = false;
          break;
        }
      }
      if (ok && i >= 50) s.v.push_back(us_since(t0));
    }
    *db = kStop;
    CK(hipStreamSynchronize(rs));
    if (!s.v.empty()) s.report("E round trip to a resident polling kernel");
    if (!ok) std::printf("E: responder did not answer\n");
    CK(hipStreamDestroy(rs));
  }
  if (want('F')) {  // F
    Stat s;
    for (int i = 0; i < reps; ++i) {
      const auto t0 = clk::now();
      const hipError_t q = hipStreamQuery(st);
      s.v.push_back(us_since(t0));
      if (q != hipSuccess) return 5;
    }
    s.report("F hipStreamQuery, idle stream");
  }
  if (want('L')) {  // L: encode_now then a device-wide synchronisation (torch.cuda.synchronize),
                    // by the dispatcher's idle time; M: a kernel on another stream between calls
    rse_codec* c = nullptr;
    if (rse_codec_new(RSE_FIELD_GF8, 10, 4, &c)) return 3;
    const size_t T = 14, L = 1024;
    uint8_t* buf = nullptr;
    CK(hipMalloc(reinterpret_cast<void**>(&buf), T * L));
    CK(hipMemset(buf, 7, T * L));
    std::vector<void*> sh(T);
    std::vector<size_t> lens(T, L);
    for (size_t i = 0; i < T; ++i) sh[i] = buf + i * L;
    hipStream_t other;
    CK(hipStreamCreateWithFlags(&other, hipStreamNonBlocking));
    for (int idle : {2000, 200, 50}) {
      rse_set_option(RSE_OPT_DISPATCH_IDLE_US, idle);
      rse_dispatcher_stop();
      char name[96];
      Stat a, b, m;
      for (int i = 0; i < 520; ++i) {
        const auto t0 = clk::now();
        if (rse_encode_now(c, sh.data(), lens.data(), T)) return 4;
        if (i >= 20) a.v.push_back(us_since(t0));
      }
      std::snprintf(name, sizeof name, "L encode_now 10+4 x 1 KiB back to back, idle %d us", idle);
      a.report(name);
      for (int i = 0; i < 220; ++i) {
        const auto t0 = clk::now();
        if (rse_encode_now(c, sh.data(), lens.data(), T)) return 4;
        CK(hipDeviceSynchronize());
        if (i >= 20) b.v.push_back(us_since(t0));
      }
      std::snprintf(name, sizeof name, "L encode_now + hipDeviceSynchronize, idle %d us", idle);
      b.report(name);
      for (int i = 0; i < 520; ++i) {
        if (rse_encode_now(c, sh.data(), lens.data(), T)) return 4;
        const auto t0 = clk::now();
        hipLaunchKernelGGL(empty_kernel, dim3(1), dim3(64), 0, other, nullptr, 0u);
        CK(hipStreamSynchronize(other));
        if (i >= 20) m.v.push_back(us_since(t0));
      }
      std::snprintf(name, sizeof name, "M other stream's kernel + sync after encode_now, idle %d", idle);
      m.report(name);
    }
    rse_set_option(RSE_OPT_DISPATCH_IDLE_US, 2000);
    rse_dispatcher_stop();
    CK(hipStreamDestroy(other));
    rse_codec_free(c);
    CK(hipFree(buf));
  }
  CK(hipHostFree(hw));
  CK(hipStreamDestroy(st));
  return 0;
}
