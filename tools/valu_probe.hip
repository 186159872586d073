// VALU issue-rate probe for gfx950: how many VALU instructions per cycle a
// SIMD retires for the instruction mixes of the bit-sliced kernels (v_bitop3
// with three sources, v_xor with two, v_bfi), at 1..8 waves per SIMD.  The
// chains are independent across 16 registers, so dependencies do not limit.
// Cycles are read with s_memtime inside the kernel (shader clock), so the
// rate is per clock, not per second.
//   hipcc --offload-arch=gfx950 -O3 tools/valu_probe.hip -o tools/bin/valu_probe
#include <hip/hip_runtime.h>

#include <cstdio>

constexpr int kIters = 4096;

template <int OP>
__global__ __launch_bounds__(256) void probe(uint32_t* out, uint64_t* cyc, uint32_t seed) {
  uint32_t r[16];
#pragma unroll
  for (int i = 0; i < 16; ++i) r[i] = seed * (threadIdx.x + i) + i;
  const uint64_t t0 = __builtin_amdgcn_s_memtime();
  for (int it = 0; it < kIters; ++it) {
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      if constexpr (OP == 0)  // v_bitop3: three sources (XOR3)
        asm volatile("v_bitop3_b32 %0, %0, %1, %2 bitop3:0x96" : "+v"(r[i]) : "v"(r[(i + 5) & 15]), "v"(r[(i + 10) & 15]));
      else if constexpr (OP == 1)  // v_xor: two sources
        asm volatile("v_xor_b32 %0, %0, %1" : "+v"(r[i]) : "v"(r[(i + 5) & 15]));
      else if constexpr (OP == 2)  // v_bfi: three sources
        asm volatile("v_bfi_b32 %0, %0, %1, %2" : "+v"(r[i]) : "v"(r[(i + 5) & 15]), "v"(r[(i + 10) & 15]));
      else if constexpr (OP == 3)  // v_bfi with the mask in an SGPR (the transposes' form)
        asm volatile("v_bfi_b32 %0, %1, %0, %2" : "+v"(r[i]) : "s"(seed), "v"(r[(i + 5) & 15]));
      else if constexpr (OP == 4)  // the same select as v_bitop3 (truth table 0xCA)
        asm volatile("v_bitop3_b32 %0, %1, %0, %2 bitop3:0xca" : "+v"(r[i]) : "s"(seed), "v"(r[(i + 5) & 15]));
      else  // shift (the transposes' other half)
        asm volatile("v_lshlrev_b32 %0, 4, %1" : "=v"(r[i]) : "v"(r[(i + 5) & 15]));
    }
  }
  const uint64_t t1 = __builtin_amdgcn_s_memtime();
  uint32_t x = 0;
#pragma unroll
  for (int i = 0; i < 16; ++i) x ^= r[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = x;
  if (threadIdx.x % 64 == 0) cyc[(blockIdx.x * blockDim.x + threadIdx.x) / 64] = t1 - t0;
}

int main() {
  int cus = 0;
  hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
  const char* names[6] = {"v_bitop3 (3 src)", "v_xor (2 src)", "v_bfi (3 src)",
                          "v_bfi (s mask)", "v_bitop3 0xca (s)", "v_lshlrev"};
  for (int op = 0; op < 6; ++op)
    for (int wps : {1, 2, 4, 8}) {  // waves per SIMD: 4 SIMDs, 256-lane groups of 4 waves
      const int blocks = cus * wps;
      uint32_t* out;
      uint64_t* cyc;
      hipMalloc(&out, (size_t)blocks * 256 * 4);
      hipMalloc(&cyc, (size_t)blocks * 4 * 8);
      auto k = op == 0 ? probe<0> : op == 1 ? probe<1> : op == 2 ? probe<2>
             : op == 3 ? probe<3> : op == 4 ? probe<4> : probe<5>;
      hipLaunchKernelGGL(k, dim3(blocks), dim3(256), 0, 0, out, cyc, 3u);
      hipEvent_t a, b;
      hipEventCreate(&a);
      hipEventCreate(&b);
      hipEventRecord(a);
      hipLaunchKernelGGL(k, dim3(blocks), dim3(256), 0, 0, out, cyc, 5u);
      hipEventRecord(b);
      hipEventSynchronize(b);
      float ms = 0;
      hipEventElapsedTime(&ms, a, b);
      uint64_t* h = new uint64_t[blocks * 4];
      hipMemcpy(h, cyc, (size_t)blocks * 4 * 8, hipMemcpyDeviceToHost);
      double mean = 0;
      for (int i = 0; i < blocks * 4; ++i) mean += (double)h[i];
      mean /= blocks * 4;
      const double insts = (double)kIters * 16;  // per wave
      // per SIMD: wps waves side by side; s_memtime counts shader clocks
      const double per_ns = insts * blocks * 4 / (cus * 4.0) / (ms * 1e6);
      std::printf("%-18s %d waves/SIMD: %.3f ms, %.3f VALU instr/ns per SIMD, %.0f clocks per "
                  "wave -> %.3f instr/clock per SIMD, clock %.2f GHz\n",
                  names[op], wps, ms, per_ns, mean, insts * wps / mean, mean / (ms * 1e6));
      delete[] h;
      hipFree(out);
      hipFree(cyc);
    }
  return 0;
}
