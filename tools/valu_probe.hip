// valu_probe.hip -- issue-rate probe: wave64 instructions per cycle per CU for
// v_perm_b32 vs v_xor_b32 (and mixes), 8 independent chains per lane so
// dependency latency is hidden; full occupancy.
//   hipcc --offload-arch=gfx950 -O3 tools/valu_probe.hip -o tools/valu_probe
#include <hip/hip_runtime.h>
#include <cstdio>

#define CHAINS 8
template <int KIND>
__global__ __launch_bounds__(256) void k(unsigned* out, unsigned seed, int iters) {
  unsigned x[CHAINS], t0 = seed * 0x9E3779B9u + threadIdx.x, t1 = t0 ^ 0x5bd1e995u;
#pragma unroll
  for (int c = 0; c < CHAINS; ++c) x[c] = t0 + c * 0x01010101u;
  for (int i = 0; i < iters; ++i) {
#pragma unroll
    for (int c = 0; c < CHAINS; ++c) {
      if (KIND == 0) x[c] = __builtin_amdgcn_perm(t0, t1, x[c] & 0x07070707u);  // perm + and
      if (KIND == 1) x[c] = (x[c] ^ t0) & t1;                                     // xor + and
      if (KIND == 2) x[c] = __builtin_amdgcn_perm(t0, t1, x[c]);                  // perm only
      if (KIND == 3) x[c] = (x[c] ^ t0) ^ (x[c] << 1);                            // xor, shl, xor
    }
  }
  unsigned r = 0;
#pragma unroll
  for (int c = 0; c < CHAINS; ++c) r ^= x[c];
  out[blockIdx.x * 256 + threadIdx.x] = r;
}

int main() {
  unsigned* out;
  hipMalloc(&out, 2048 * 256 * 4);
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  int dev;
  hipGetDevice(&dev);
  int clk_khz;
  hipDeviceGetAttribute(&clk_khz, hipDeviceAttributeClockRate, dev);
  const int iters = 4096, blocks = 2048;
  const char* names[] = {"perm+and", "xor+and", "perm", "xor+shl+xor"};
  const int insts[] = {2, 2, 1, 3};
  for (int kind = 0; kind < 4; ++kind) {
    auto launch = [&] {
      if (kind == 0) hipLaunchKernelGGL(k<0>, dim3(blocks), dim3(256), 0, 0, out, 1u, iters);
      if (kind == 1) hipLaunchKernelGGL(k<1>, dim3(blocks), dim3(256), 0, 0, out, 1u, iters);
      if (kind == 2) hipLaunchKernelGGL(k<2>, dim3(blocks), dim3(256), 0, 0, out, 1u, iters);
      if (kind == 3) hipLaunchKernelGGL(k<3>, dim3(blocks), dim3(256), 0, 0, out, 1u, iters);
    };
    launch();
    hipDeviceSynchronize();
    hipEventRecord(a);
    launch();
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms;
    hipEventElapsedTime(&ms, a, b);
    double wave_insts = (double)blocks * 4 * iters * CHAINS * insts[kind];
    double per_s = wave_insts / (ms * 1e-3);
    printf("%-12s %8.3f ms  %.3e wave-inst/s  = %.2f wave-inst/clk/CU at %d MHz nominal\n",
           names[kind], ms, per_s, per_s / 256 / (clk_khz * 1e3), clk_khz / 1000);
  }
  return 0;
}
