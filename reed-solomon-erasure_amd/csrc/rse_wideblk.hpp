// rse_wideblk.hpp -- wide codecs past one wide module's argument block
// (rse_jit.cpp "wide modules over input blocks"), for the host codec.  Kept
// out of rse_kernels.hpp, whose text is part of every run-time module's source.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

namespace rse {

// Whether a p x k matrix runs as a chain of wide modules over input blocks
// (RSE_OPT_WIDE_BLOCK_INPUTS > 0, k + 2p past the one-module limit, p within
// a wide module's); *n_blocks = the chain's length.  jit_register_blocks and
// jit_blocks_status then register / report those modules instead of the
// 8 x 32 kJitBlock ones.
bool wide_blocks_plan(uint32_t k, uint32_t p, uint32_t* n_blocks);
// out = rows x in (store mode) through the chain, every whole 4 KiB chunk of
// the shards (or the whole 1 / 2 KiB shards); *done = the bytes per shard
// coded, 0 if a module is not built yet (nothing launched).
hipError_t launch_wide_blocks(int field, uint32_t k, uint32_t p, const uint16_t* rows,
                              const uint8_t* const* in, uint8_t* const* out, uint64_t len,
                              uint64_t stripe_stride, uint32_t n_stripes, hipStream_t stream,
                              uint64_t* done);

}  // namespace rse
