#!/bin/bash
# Instruction histogram of the compiled codecs' default encode kernels, built
# alone from rse_bitslice_core.hpp (seconds, vs minutes for rse_bitslice.o):
#   tools/isa_probe.sh [extra hipcc flags]
# Prints VGPR/spill counts and the top instructions per kernel; the assembly
# is left in /tmp/rse_isa_probe/.
set -e
REPO="$(cd "$(dirname "$0")/.." && pwd)"
PKG="$REPO/reed-solomon-erasure_amd"
OUT=/tmp/rse_isa_probe
mkdir -p "$OUT"
cat > "$OUT/probe.hip" <<'EOF'
#include "rse_bitslice_core.hpp"
namespace rse {
namespace {
#include "rse_bs_tables.inc"
template <class C, bool SB>
__global__ __launch_bounds__(kBsBlock, C::p > 4 ? 2 : 3) void probe_kernel(
    const CodeArgs a, uint64_t chunks_per_stripe) {
  bitslice_body<C, true, SB, false>(a, chunks_per_stripe);
}
template <class C, int NS>
__global__ __launch_bounds__(kBsBlock, NS > 4 ? 2 : 3) void rprobe(const BsReconArgs a,
                                                                  uint64_t chunks_per_stripe) {
  bitslice_recon_body<C, true, NS, kReconMixDefault>(a, chunks_per_stripe);
}
template <class C>
__global__ __launch_bounds__(kBsBlock, 3) void pprobe(const BsReconArgs a, uint64_t chunks_per_stripe) {
  bitslice_recon_pair_body<C, true, 2>(a, chunks_per_stripe);
}
}  // namespace
void* probe_fns[] = {(void*)probe_kernel<Bs16_20_8, false>, (void*)probe_kernel<Bs8_10_4, true>, (void*)rprobe<Bs16_20_8, 8>, (void*)rprobe<Bs16_20_8, 4>, (void*)rprobe<Bs8_10_4, 4>, (void*)pprobe<Bs16_20_8>};
}  // namespace rse
EOF
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 --offload-device-only -I"$PKG/csrc" \
  -I"$PKG/build" "$@" -S "$OUT/probe.hip" -o "$OUT/probe.s"
grep -E "^\s+\.(name|vgpr_count|vgpr_spill_count):" "$OUT/probe.s" |
  awk '/\.name:/{n=$2} /\.vgpr_count:/{v=$2} /\.vgpr_spill_count:/{print "vgpr", v, "spill", $2, n}'
awk '/^_Z[^ ]*:/{k=substr($1, 1, 60)} /^\t[sv]_[a-z0-9_]+/{c[k" "$1]++} END{for (x in c) print c[x], x}' \
  "$OUT/probe.s" | sort -k2,2 -k1,1nr | awk '{if (n[$2]++ < 16) print}'
