// Per-call latency of the C ABI with no binding layer in between -- what a
// Rust (or any FFI) caller of rse_verify / rse_encode sees: one 10+4 x 16 MiB
// stripe per call on device shards, synchronous verify, back-to-back encode.
//   hipcc --offload-arch=gfx950 -O2 -I include tools/capi_latency.cpp \
//     -L reed-solomon-erasure_amd/reed_solomon_erasure -lrse_hip -o /tmp/capi_latency
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "rse_hip.h"
#include "rse_hip_tune.h"

int main(int argc, char** argv) {
  setenv("RSE_TUNE", "1", 0);  // the tuning switches below (include/rse_hip_tune.h)
  const size_t k = 10, p = 4, L = 16u << 20, S = 8;
  if (argc > 1) {  // workgroups of the bit-sliced launches (RSE_OPT_GRID_X; 0 = default)
    const long g = std::atol(argv[1]);
    if (rse_set_option(RSE_OPT_GRID_X, g)) return 7;
    std::printf("grid %ld\n", g);
  }
  if (argc > 2) {  // RSE_OPT_SYNC_EVENT
    if (rse_set_option(RSE_OPT_SYNC_EVENT, std::atol(argv[2]))) return 8;
    std::printf("sync event %s\n", argv[2]);
  }
  if (argc > 3) {  // RSE_OPT_SPIN_WAIT
    if (rse_set_option(RSE_OPT_SPIN_WAIT, std::atol(argv[3]))) return 9;
    std::printf("spin wait %s\n", argv[3]);
  }
  rse_codec* c = nullptr;
  if (rse_codec_new(RSE_FIELD_GF8, k, p, &c)) return 1;
  uint8_t* buf = nullptr;
  if (hipMalloc(reinterpret_cast<void**>(&buf), S * (k + p) * L) != hipSuccess) return 2;
  std::vector<std::vector<void*>> sh(S, std::vector<void*>(k + p));
  std::vector<size_t> lens(k + p, L);
  for (size_t s = 0; s < S; ++s)
    for (size_t i = 0; i < k + p; ++i) {
      sh[s][i] = buf + (s * (k + p) + i) * L;
      if (i < k && rse_fill_splitmix(sh[s][i], L, 1, (s << 8) | i, nullptr)) return 3;
    }
  for (size_t s = 0; s < S; ++s)
    if (rse_encode(c, sh[s].data(), lens.data(), k + p, nullptr)) return 4;
  if (hipDeviceSynchronize() != hipSuccess) return 5;
  const double bytes = double((k + p) * L);
  for (int leg = 0; leg < 2; ++leg) {
    const int reps = 64;
    int ok = 1;
    for (int w = 0; w < 8; ++w)  // warm
      leg ? rse_encode(c, sh[w % S].data(), lens.data(), k + p, nullptr)
          : rse_verify(c, const_cast<const void* const*>(sh[w % S].data()), lens.data(), k + p,
                       &ok, nullptr);
    (void)hipDeviceSynchronize();
    const auto t0 = std::chrono::steady_clock::now();
    for (int r = 0; r < reps; ++r) {
      const int rc = leg ? rse_encode(c, sh[r % S].data(), lens.data(), k + p, nullptr)
                         : rse_verify(c, const_cast<const void* const*>(sh[r % S].data()),
                                      lens.data(), k + p, &ok, nullptr);
      if (rc || !ok) return 6;
    }
    (void)hipDeviceSynchronize();
    const double dt =
        std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() / reps;
    std::printf("%s (C ABI, one stripe per call): %.1f us per call, %.1f GB/s\n",
                leg ? "encode (asynchronous)" : "verify (synchronous)", dt * 1e6, bytes / dt / 1e9);
  }
  {  // the floor of any synchronous call: one tiny launch + stream synchronisation
    const int reps = 256;
    for (int w = 0; w < 16; ++w) {
      (void)rse_fill_splitmix(buf, 64, 1, 0, nullptr);
      (void)hipStreamSynchronize(nullptr);
    }
    const auto t0 = std::chrono::steady_clock::now();
    for (int r = 0; r < reps; ++r) {
      (void)rse_fill_splitmix(buf, 64, 1, 0, nullptr);
      (void)hipStreamSynchronize(nullptr);
    }
    const double dt =
        std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() / reps;
    std::printf("tiny launch + synchronize (the floor): %.1f us per call\n", dt * 1e6);
  }
  {  // the verify kernel alone: events around back-to-back verifies of one stripe
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    int ok = 1;
    const int reps = 32;
    (void)hipEventRecord(a, nullptr);
    for (int r = 0; r < reps; ++r)
      (void)rse_verify(c, const_cast<const void* const*>(sh[r % S].data()), lens.data(), k + p,
                       &ok, nullptr);
    (void)hipEventRecord(b, nullptr);
    (void)hipEventSynchronize(b);
    float ms = 0;
    (void)hipEventElapsedTime(&ms, a, b);
    std::printf("verify, device time between events (launch gaps included): %.1f us per call\n",
                ms * 1e3 / reps);
  }
  rse_codec_free(c);
  (void)hipFree(buf);
  return 0;
}
