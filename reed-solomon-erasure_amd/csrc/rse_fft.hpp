// rse_fft.hpp -- the additive-FFT kernels of GF(2^8) codecs with k = p = 16,
// 32 or 64 (rse_fft.hip): encode / verify (the codec's parity rows) and every
// data shard rebuilt from the parity shards (the same rows: the parity block
// is its own inverse), bit-exact with the coefficient networks.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace rse {

constexpr int kFftMax = 64;

// Kernel arguments: stripe 0's k input, k output and k compare pointers (the
// other stripes stripe_stride bytes further).
struct FftArgs {
  uint64_t stripe_stride;
  uint64_t cols_per_stripe;  // whole 2 KiB columns per shard (1 KiB shards: 0)
  uint32_t* mismatch;        // check modes
  uint32_t n_stripes;
  uint32_t mode;             // CodeMode
  uint32_t per_stripe;       // check modes: mismatch[stripe]
  uint32_t pad;
  const uint8_t* in[kFftMax];
  uint8_t* out[kFftMax];
  const uint8_t* cmp[kFftMax];
};

// rows[p x k] are the parity rows of the GF(2^8) k+k codec (k = p = 16, 32,
// 64) -- which are also their own inverse -- and RSE_OPT_FFT is on.
bool fft_applies(int field, uint32_t k, uint32_t p, const uint16_t* rows);
// Codes the whole 2 KiB columns of every shard (1 KiB shards: all of them) of
// n_stripes stripes when fft_applies; *done = bytes per shard
// coded, 0 if nothing was launched.
hipError_t launch_fft(int field, uint32_t k, uint32_t p, const uint16_t* rows,
                      const uint8_t* const* in, uint8_t* const* out, const uint8_t* const* cmp,
                      uint64_t len, uint64_t stripe_stride, uint32_t n_stripes, uint32_t mode,
                      uint32_t* mismatch, bool per_stripe, hipStream_t stream, uint64_t* done);

}  // namespace rse
