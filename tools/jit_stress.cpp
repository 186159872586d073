// jit_stress.cpp -- host-side concurrency stress of librse_hip.so for the
// ThreadSanitizer build (tools/sanitize.sh); no GPU needed.
//
// Eight threads at once, each in a loop: create codecs (some shared with other
// threads, some their own), ask for their run-time specialised kernels (with
// and without waiting: the registry, the build queues, the rse_jitc helper
// processes, the on-disk cache), and plan reconstructs of many erasure
// patterns on the codecs they share (the mutex-guarded decode-matrix LRU of
// core.rs:697-731 and its eviction past 254 entries).  Without a device the
// reconstructs stop with RSE_ERR_DEVICE after planning, which is all the
// host-side state a reconstruct touches.  Then the process exits with builds
// still queued (the library's unload path).
#include <atomic>
#include <cstdio>
#include <cstdint>
#include <thread>
#include <vector>

#include "../include/rse_hip.h"

int main() {
  rse_codec* shared[3] = {};
  if (rse_codec_new(RSE_FIELD_GF8, 10, 4, &shared[0]) || rse_codec_new(RSE_FIELD_GF8, 12, 4, &shared[1]) ||
      rse_codec_new(RSE_FIELD_GF16, 6, 3, &shared[2])) {
    std::fprintf(stderr, "codec_new failed\n");
    return 1;
  }
  std::atomic<int> bad{0};
  std::vector<std::thread> th;
  for (int t = 0; t < 8; ++t)
    th.emplace_back([&, t] {
      for (int it = 0; it < 40; ++it) {
        rse_codec* own = nullptr;
        if (rse_codec_new(t % 2 ? RSE_FIELD_GF16 : RSE_FIELD_GF8, 3 + (t + it) % 5, 2 + it % 3, &own))
          ++bad;
        const int kind = rse_codec_kernel_kind(own, it % 10 == 0);
        if (kind < 0 || kind > RSE_KERNELS_SPECIALISE_FAILED) ++bad;
        rse_codec* c = shared[(t + it) % 3];
        const size_t k = rse_codec_data_shard_count(c), n = rse_codec_total_shard_count(c);
        std::vector<void*> ptrs(n);
        std::vector<size_t> lens(n, 65536);
        std::vector<uint8_t> present(n, 1);
        for (size_t i = 0; i < n; ++i) ptrs[i] = reinterpret_cast<void*>(uintptr_t(0x10000) * (i + 1));
        // a different erasure pattern per iteration: one or two shards lost
        present[(t * 7 + it) % n] = 0;
        if (it % 2) present[(t + it * 3) % n] = 0;
        const int rc = rse_reconstruct_data(c, ptrs.data(), lens.data(), present.data(), n, nullptr);
        if (rc != RSE_ERR_DEVICE && rc != RSE_OK) ++bad;
        (void)k;
        rse_codec_free(own);
      }
    });
  for (auto& x : th) x.join();
  // queue builds and leave without waiting for them
  rse_codec* late = nullptr;
  rse_codec_new(RSE_FIELD_GF8, 20, 6, &late);
  rse_codec_kernel_kind(late, 0);
  std::printf("jit_stress: %d unexpected statuses\n", bad.load());
  return bad.load() ? 1 : 0;
}
