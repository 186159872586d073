// Prints the Horner-mixing basis of rse_kernels.hpp (z, the GF(2^16) taps,
// to_b and from_b masks, and horner_coords of a few constants) for
// tests/test_horner_basis.py, which checks them against the oracle's field.
#define RSE_JIT 1
#define __host__
#define __device__
#include <cstdint>
#include <cstdio>
#include <initializer_list>
using std::uint16_t;
using std::uint32_t;
using std::uint64_t;
using std::uint8_t;
using std::int32_t;
#include "rse_kernels.hpp"

int main() {
  using namespace rse;
  std::printf("z %u taps16 %u taps8 %u\n", kHornerZ16, kHornerTaps16, kHornerTaps8);
  std::printf("to_b");
  for (int i = 0; i < 16; ++i) std::printf(" %u", kHornerBasis16.to_b[i]);
  std::printf("\nfrom_b");
  for (int i = 0; i < 16; ++i) std::printf(" %u", kHornerBasis16.from_b[i]);
  std::printf("\ncoords");
  for (uint32_t c : {1u, 2u, 0x100u, 0x4815u, 0xFFFFu, 0x1234u, 0xBEEFu})
    std::printf(" %u:%u", c, horner_coords(16, c));
  std::printf("\n");
  return 0;
}
