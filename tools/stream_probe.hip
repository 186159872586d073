// stream_probe.hip -- which access pattern gets the most HBM bandwidth for
// encode's shape (read NR shards, write NW shards, 16 B per lane)?
//
// Sweeps, with trivial XOR arithmetic so only memory behaviour is measured:
//   U        vectors per lane per shard per step (bytes in flight per lane)
//   NTL/NTS  non-temporal loads / stores
//   CONTIG   each workgroup walks its own contiguous range (vs grid-stride)
//   blocks   grid size
// plus a plain copy for calibration (MI355X_MICROARCH.md: 6.29 TB/s float4 copy).
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/stream_probe.hip -o tools/stream_probe
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

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
__device__ __forceinline__ u32x4 ld(const u32x4* p) {
  if constexpr (NT) return __builtin_nontemporal_load(p);
  else return *p;
}
template <bool NT>
__device__ __forceinline__ void st(u32x4* p, u32x4 v) {
  if constexpr (NT) __builtin_nontemporal_store(v, p);
  else *p = v;
}

// Flat vector space over stripes: g -> (stripe g / nvec, vector g % nvec);
// shard i of a stripe starts at stripe * (NR + NW) * nvec + i * nvec.
template <int NR, int NW, int U, bool NTL, bool NTS, bool CONTIG>
__global__ __launch_bounds__(256) void enc_k(u32x4* base, uint64_t nvec, uint64_t stripes) {
  const uint64_t total = nvec * stripes;       // vectors per shard-row, all stripes
  const uint64_t step = 256ull * U;            // vectors per workgroup step
  const uint64_t nsteps = total / step;
  uint64_t s0, s1, sst;
  if (CONTIG) {
    const uint64_t per = (nsteps + gridDim.x - 1) / gridDim.x;
    s0 = blockIdx.x * per;
    s1 = s0 + per < nsteps ? s0 + per : nsteps;
    sst = 1;
  } else {
    s0 = blockIdx.x;
    s1 = nsteps;
    sst = gridDim.x;
  }
  for (uint64_t s = s0; s < s1; s += sst) {
    const uint64_t g = s * step;               // nvec is a multiple of step
    const uint64_t stripe = g / nvec, v0 = g - stripe * nvec + threadIdx.x;
    u32x4* sb = base + stripe * (NR + NW) * nvec + v0;
    u32x4 acc[NW][U];
#pragma unroll
    for (int r = 0; r < NW; ++r)
#pragma unroll
      for (int u = 0; u < U; ++u) acc[r][u] = (u32x4){(unsigned)r, 1u, 2u, 3u};
    u32x4 x[NR][U];
#pragma unroll
    for (int i = 0; i < NR; ++i)
#pragma unroll
      for (int u = 0; u < U; ++u) x[i][u] = ld<NTL>(sb + i * nvec + u * 256);
#pragma unroll
    for (int i = 0; i < NR; ++i)
#pragma unroll
      for (int r = 0; r < NW; ++r)
#pragma unroll
        for (int u = 0; u < U; ++u) acc[r][u] ^= (x[i][u] << (unsigned)((r + i) & 7));
#pragma unroll
    for (int r = 0; r < NW; ++r)
#pragma unroll
      for (int u = 0; u < U; ++u) st<NTS>(sb + (NR + r) * nvec + u * 256, acc[r][u]);
  }
}

template <int U, bool NT>
__global__ __launch_bounds__(256) void copy_k(const u32x4* __restrict__ a, u32x4* __restrict__ b,
                                               uint64_t n) {
  for (uint64_t i = (blockIdx.x * 256ull) * U + threadIdx.x; i < n; i += gridDim.x * 256ull * U) {
    u32x4 t[U];
#pragma unroll
    for (int u = 0; u < U; ++u) t[u] = ld<NT>(a + i + u * 256);
#pragma unroll
    for (int u = 0; u < U; ++u) st<NT>(b + i + u * 256, t[u]);
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
  CK(hipEventDestroy(a));
  CK(hipEventDestroy(b));
  return ms / reps;
}

u32x4* g_buf;
uint64_t g_nvec, g_stripes;

template <int U, bool NTL, bool NTS, bool CONTIG>
void run_enc(const char* tag) {
  for (int blocks : {1024, 2048, 4096, 8192}) {
    const double ms = time_ms(
        [&] {
          hipLaunchKernelGGL((enc_k<10, 4, U, NTL, NTS, CONTIG>), dim3(blocks), dim3(256), 0, 0,
                             g_buf, g_nvec, g_stripes);
        },
        5);
    const double bytes = 14.0 * 16 * g_nvec * g_stripes;
    printf("enc10x4 %-8s U=%d ntl=%d nts=%d contig=%d blocks=%-5d %8.1f GB/s\n", tag, U, NTL, NTS,
           CONTIG, blocks, bytes / ms / 1e6);
    fflush(stdout);
  }
}

template <int U, bool NT>
void run_copy() {
  const uint64_t n = 14 * g_nvec * g_stripes / 2;
  for (int blocks : {1024, 2048, 4096, 8192, 16384}) {
    const double ms = time_ms(
        [&] {
          hipLaunchKernelGGL((copy_k<U, NT>), dim3(blocks), dim3(256), 0, 0, g_buf, g_buf + n, n);
        },
        5);
    printf("copy U=%d nt=%d blocks=%-5d %8.1f GB/s\n", U, NT, blocks, 2.0 * 16 * n / ms / 1e6);
    fflush(stdout);
  }
}

// Pure streams: NR reads (kept live), NW writes, grid-stride, nt.
template <int NR, int NW>
__global__ __launch_bounds__(256) void rw_k(u32x4* base, uint64_t n) {
  u32x4 acc = {1u, 2u, 3u, 4u};
  for (uint64_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += gridDim.x * 256ull) {
#pragma unroll
    for (int r = 0; r < NR; ++r) acc ^= ld<true>(base + r * n + i);
#pragma unroll
    for (int w = 0; w < NW; ++w) st<true>(base + (NR + w) * n + i, acc + (unsigned)w);
  }
  if (NW == 0 && acc.x == 0x12345u) base[0] = acc;
}

void run_sizes() {
  for (uint64_t mib : {256ull, 1024ull, 4096ull, 8192ull}) {
    const uint64_t n = mib * 1048576 / 16 / 2;
    for (int blocks : {1024, 4096, 16384}) {
      const double ms = time_ms(
          [&] {
            hipLaunchKernelGGL((copy_k<1, true>), dim3(blocks), dim3(256), 0, 0, g_buf, g_buf + n, n);
          },
          10);
      printf("copy-size %5lu MiB blocks=%-5d %8.1f GB/s\n", mib, blocks, 2.0 * 16 * n / ms / 1e6);
      fflush(stdout);
    }
  }
  const uint64_t n = 256ull * 1048576;  // 4 GiB per stream
  for (int blocks : {1024, 4096}) {
    auto go = [&](auto kern, const char* name, int streams) {
      const double ms =
          time_ms([&] { hipLaunchKernelGGL(kern, dim3(blocks), dim3(256), 0, 0, g_buf, n); }, 3);
      printf("%-8s blocks=%-5d %8.1f GB/s\n", name, blocks, streams * 16.0 * n / ms / 1e6);
      fflush(stdout);
    };
    go(rw_k<1, 0>, "read1", 1);
    go(rw_k<2, 0>, "read2", 2);
    go(rw_k<0, 1>, "write1", 1);
    go(rw_k<0, 2>, "write2", 2);
    go(rw_k<1, 1>, "r1w1", 2);
    go(rw_k<2, 1>, "r2w1", 3);
    go(rw_k<3, 1>, "r3w1", 4);
  }
}

int main(int argc, char** argv) {
  g_stripes = argc > 1 ? atoi(argv[1]) : 64;
  g_nvec = (16ull << 20) / 16;
  const size_t total = g_stripes * 14 * (16ull << 20);
  CK(hipMalloc(&g_buf, total));
  CK(hipMemset(g_buf, 0x5A, total));
  printf("buffer %.1f GiB, %lu stripes of 10+4 x 16 MiB\n", total / 1073741824.0, g_stripes);
  if (argc > 2 && argv[2][0] == 's') {
    run_sizes();
    CK(hipFree(g_buf));
    return 0;
  }
  run_copy<1, false>();
  run_copy<1, true>();
  run_copy<4, false>();
  run_copy<4, true>();
  run_enc<1, true, true, false>("U1");
  run_enc<2, true, true, false>("U2");
  run_enc<4, true, true, false>("U4");
  run_enc<1, true, true, true>("U1c");
  run_enc<2, true, true, true>("U2c");
  run_enc<4, true, true, true>("U4c");
  run_enc<4, true, false, false>("U4ntl");
  run_enc<4, false, true, false>("U4nts");
  run_enc<4, false, false, false>("U4pl");
  CK(hipFree(g_buf));
  return 0;
}
