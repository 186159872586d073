// rse_sub_ext.hpp -- a variant of the narrow modules' 1 / 2 KiB-shard body
// (rse_bitslice_core.hpp bitslice_body with SUB) that run-time modules include
// only when RSE_OPT_SUB_DEPTH asks for it (rse_jit.cpp make_source appends
// this text after the core's, so the other modules keep their cache keys).
//
// bitslice_body keeps one input's loads in flight per wave.  With 1 / 2 KiB
// shards a launch of a few thousand stripes gives each wave one 4 KiB chunk,
// so the launch is k dependent HBM round trips long (16+16 x 1 KiB
// reconstruct_one: 4.35 TB/s at 8192 stripes against 5.19 at 65536,
// profiles/r05/s21/).  Here D inputs are in flight (a ring of D + 1 slots,
// indexed at compile time so it stays in VGPRs).
#pragma once

namespace rse {

template <class C, int D, int I, uint32_t S>
__device__ __forceinline__ void code_inputs_ring(uint32_t (&acc)[C::p * 16],
                                                 u32x4 (&buf)[D + 1][4], const CodeArgs& a,
                                                 uint64_t off) {
  if constexpr (I < C::k) {
    if constexpr (I + D < C::k) load4<true, S>(buf[(I + D) % (D + 1)], a.in[I + D] + off);
    __builtin_amdgcn_sched_barrier(0);  // the loads stay ahead of the network
    uint32_t pl[16];
    slice<typename C::Field>(buf[I % (D + 1)], pl);
    mac_input<C, I, false>(acc, pl, make_int_seq<C::p * 16>{});
#pragma unroll
    for (int q = 0; q < C::p * 16; ++q) asm volatile("" : "+v"(acc[q]));
    code_inputs_ring<C, D, I + 1, S>(acc, buf, a, off);
  }
}

// bitslice_body<C, NT = true, ..., W4 = true, ..., SUB> with D inputs in flight.
template <class C, int D, uint32_t SUB>
__device__ __forceinline__ void bitslice_body_sub_deep(const CodeArgs& a, uint64_t) {
  static_assert(SUB == 1024u || SUB == 2048u, "1 or 2 KiB shards");
  constexpr uint32_t S = SUB / 4u;
  constexpr uint32_t SPC = 4096u / SUB, LPS = 64u / SPC;  // stripes / chunk, lanes / stripe
  const uint64_t total = (a.n_stripes + SPC - 1) / SPC;
  const uint64_t steps = (total + 3) / 4;
  const uint32_t sub = threadIdx.x >> 6;  // wave-uniform
  const uint32_t lane = threadIdx.x & 63u;
  const uint32_t lane_off = (lane % LPS) * 16u;
  const uint32_t mode = a.mode;
  bool diff = false;
  for (uint64_t idx = blockIdx.x; idx < steps; idx += gridDim.x) {
    const uint64_t c = idx * 4 + sub;
    if (c >= total) continue;  // the last step's spare waves
    uint64_t stripe = c * SPC + lane / LPS;
    const bool ok = stripe < a.n_stripes;
    if (!ok) stripe = a.n_stripes - 1;  // loaded, never stored
    const uint64_t off = stripe * a.stripe_stride + lane_off;
    uint32_t acc[C::p * 16];
    u32x4 buf[D + 1][4];
#pragma unroll
    for (int j = 0; j < D; ++j)
      if (j < C::k) load4<true, S>(buf[j], a.in[j] + off);
    code_inputs_ring<C, D, 0, S>(acc, buf, a, off);
    store_outputs<C, true, false, S, 0, CodeArgs, false>(acc, a, off, mode, diff, ok);
    if (a.per_stripe && diff) {  // verify_flat: this lane's stripe
      flag_mismatch(a.mismatch + c * SPC + lane / LPS);
      diff = false;
    }
  }
  if (mode != kStore && diff) flag_mismatch(a.mismatch);
}

}  // namespace rse
