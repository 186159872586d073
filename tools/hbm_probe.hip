// hbm_probe.hip -- memory-roofline probes for the encode access pattern.
//
// What bandwidth can MI355X sustain for "read 10 streams, write 4 streams" at
// 16 B/lane, independent of the GF arithmetic?  Reports GB/s (1e9) for:
//   copy     : 1 read + 1 write stream (the guide's float4-copy reference)
//   read14   : 14 read streams (verify's pattern)
//   xor10x4  : 10 reads, 4 writes, XOR/rotate only (encode's pattern, no tables)
// each with plain and non-temporal (nt) loads/stores.
//   hipcc --offload-arch=gfx950 -O3 tools/hbm_probe.hip -o /tmp/hbm_probe
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                 \
  do {                                                                        \
    hipError_t e = (x);                                                       \
    if (e != hipSuccess) {                                                    \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e)); \
      exit(1);                                                                \
    }                                                                         \
  } while (0)

typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
template <bool NT>
__device__ __forceinline__ uint4 ld(const uint4* p) {
  if constexpr (NT) {
    u32x4 v = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(p));
    return make_uint4(v.x, v.y, v.z, v.w);
  } else {
    return *p;
  }
}
template <bool NT>
__device__ __forceinline__ void st(uint4* p, uint4 v) {
  if constexpr (NT) {
    u32x4 w = {v.x, v.y, v.z, v.w};
    __builtin_nontemporal_store(w, reinterpret_cast<u32x4*>(p));
  } else {
    *p = v;
  }
}

template <bool NT>
__global__ __launch_bounds__(256) void copy_k(const uint4* __restrict__ a, uint4* __restrict__ b,
                                               size_t n) {
  for (size_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += gridDim.x * 256ull)
    st<NT>(b + i, ld<NT>(a + i));
}

// stripe layout: [stripe][14][vec]; grid.y = stripe
template <bool NT, int NR, int NW>
__global__ __launch_bounds__(256) void stream_k(uint4* base, size_t vec_per_shard,
                                                 size_t stripe_stride_vec) {
  uint4* s = base + blockIdx.y * stripe_stride_vec;
  for (size_t v = blockIdx.x * 256ull + threadIdx.x; v < vec_per_shard; v += gridDim.x * 256ull) {
    uint4 x[NR];
#pragma unroll
    for (int i = 0; i < NR; ++i) x[i] = ld<NT>(s + i * vec_per_shard + v);
    uint4 acc[NW > 0 ? NW : 1];
#pragma unroll
    for (int r = 0; r < (NW > 0 ? NW : 1); ++r) {
      acc[r] = make_uint4(r, r, r, r);
#pragma unroll
      for (int i = 0; i < NR; ++i) {
        acc[r].x ^= __builtin_rotateleft32(x[i].x, r + i);
        acc[r].y ^= __builtin_rotateleft32(x[i].y, r + i);
        acc[r].z ^= __builtin_rotateleft32(x[i].z, r + i);
        acc[r].w ^= __builtin_rotateleft32(x[i].w, r + i);
      }
    }
    if (NW > 0) {
#pragma unroll
      for (int r = 0; r < NW; ++r) st<NT>(s + (NR + r) * vec_per_shard + v, acc[r]);
    } else if ((acc[0].x ^ acc[0].y ^ acc[0].z ^ acc[0].w) == 0x12345678u) {
      s[v] = acc[0];  // keep the reads live
    }
  }
}

// all blocks sweep stripe 0, then stripe 1, ...: few open DRAM regions
template <bool NT, int NR, int NW>
__global__ __launch_bounds__(256) void seq_k(uint4* base, size_t vec_per_shard, size_t stripe_stride_vec,
                                             int stripes) {
  for (int st_i = 0; st_i < stripes; ++st_i) {
    uint4* s = base + st_i * stripe_stride_vec;
    for (size_t v = blockIdx.x * 256ull + threadIdx.x; v < vec_per_shard; v += gridDim.x * 256ull) {
      uint4 x[NR];
#pragma unroll
      for (int i = 0; i < NR; ++i) x[i] = ld<NT>(s + i * vec_per_shard + v);
#pragma unroll
      for (int r = 0; r < NW; ++r) {
        uint4 acc = make_uint4(r, r, r, r);
#pragma unroll
        for (int i = 0; i < NR; ++i) {
          acc.x ^= __builtin_rotateleft32(x[i].x, r + i);
          acc.y ^= __builtin_rotateleft32(x[i].y, r + i);
          acc.z ^= __builtin_rotateleft32(x[i].z, r + i);
          acc.w ^= __builtin_rotateleft32(x[i].w, r + i);
        }
        st<NT>(s + (NR + r) * vec_per_shard + v, acc);
      }
    }
  }
}

template <class F>
double time_ms(F f, int reps) {
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  f();
  CK(hipDeviceSynchronize());
  CK(hipEventRecord(a));
  for (int i = 0; i < reps; ++i) f();
  CK(hipEventRecord(b));
  CK(hipEventSynchronize(b));
  float ms;
  CK(hipEventElapsedTime(&ms, a, b));
  return ms / reps;
}

int main(int argc, char** argv) {
  const size_t shard = 16ull << 20, nvec = shard / 16;
  const int stripes = argc > 1 ? atoi(argv[1]) : 64;
  const size_t total = (size_t)stripes * 14 * shard;
  uint4* buf;
  CK(hipMalloc(&buf, total));
  CK(hipMemset(buf, 0x5A, total));
  const int reps = 5;
  for (int blocks_per_stripe : {2, 4, 8, 16, 32}) {
    dim3 g(blocks_per_stripe, stripes);
    auto run = [&](auto kern, const char* name, double bytes) {
      double ms = time_ms([&] { hipLaunchKernelGGL(kern, g, dim3(256), 0, 0, buf, nvec, 14 * nvec); },
                          reps);
      printf("%-10s bps=%-3d blocks=%-6d %8.1f GB/s  (%.3f ms)\n", name, blocks_per_stripe,
             blocks_per_stripe * stripes, bytes / ms / 1e6, ms);
    };
    run(stream_k<false, 10, 4>, "xor10x4", 14.0 * shard * stripes);
    run(stream_k<true, 10, 4>, "xor10x4nt", 14.0 * shard * stripes);
    run(stream_k<false, 14, 0>, "read14", 14.0 * shard * stripes);
    run(stream_k<true, 14, 0>, "read14nt", 14.0 * shard * stripes);
  }
  for (int blocks : {256, 512, 1024, 2048, 4096, 8192}) {
    double ms = time_ms([&] { hipLaunchKernelGGL((seq_k<false, 10, 4>), dim3(blocks), dim3(256), 0, 0,
                                                 buf, nvec, 14 * nvec, stripes); }, reps);
    double msn = time_ms([&] { hipLaunchKernelGGL((seq_k<true, 10, 4>), dim3(blocks), dim3(256), 0, 0,
                                                  buf, nvec, 14 * nvec, stripes); }, reps);
    const double bytes = 14.0 * shard * stripes;
    printf("seq10x4    blocks=%-6d %8.1f GB/s   nt %8.1f GB/s\n", blocks, bytes / ms / 1e6, bytes / msn / 1e6);
  }
  const size_t half = total / 16 / 2;  // uint4 count of each half
  for (int blocks : {1024, 2048, 4096, 8192}) {
    double ms = time_ms(
        [&] { hipLaunchKernelGGL(copy_k<false>, dim3(blocks), dim3(256), 0, 0, buf, buf + half, half); },
        reps);
    double msn = time_ms(
        [&] { hipLaunchKernelGGL(copy_k<true>, dim3(blocks), dim3(256), 0, 0, buf, buf + half, half); },
        reps);
    printf("copy       blocks=%-6d %8.1f GB/s   nt %8.1f GB/s\n", blocks, 2.0 * half * 16 / ms / 1e6,
           2.0 * half * 16 / msn / 1e6);
  }
  CK(hipFree(buf));
  return 0;
}
