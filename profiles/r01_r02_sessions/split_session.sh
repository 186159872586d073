#!/bin/bash
# One-module kernels with the outputs split over waves (RSE_OPT_WIDE_SPLIT 4:
# two waves of 4 outputs sharing each input chunk, 3 waves/SIMD) against the
# single-wave run-time specialised kernels (8 outputs per wave, 2 waves/SIMD),
# separate processes.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
T="python -u tools/tune.py --rounds 5 --nt-only --shapes 0:0 --bitslice 1"
bash tools/gpu_session.sh \
 "s8_16_12_8:300:$T --field 16 --k 12 --p 8 --shard-mib 4 --stripes 256" \
 "s4_16_12_8:300:$T --wide-split 4 --field 16 --k 12 --p 8 --shard-mib 4 --stripes 256" \
 "s8_16_24_8:300:$T --field 16 --k 24 --p 8 --shard-mib 4 --stripes 128" \
 "s4_16_24_8:300:$T --wide-split 4 --field 16 --k 24 --p 8 --shard-mib 4 --stripes 128" \
 "s8_16_40_12:300:$T --field 16 --k 40 --p 12 --shard-mib 1 --stripes 64" \
 "s4_16_40_12:300:$T --wide-split 4 --field 16 --k 40 --p 12 --shard-mib 1 --stripes 64" \
 "s8_8_50_20:300:$T --k 50 --p 20 --shard-mib 1 --stripes 64" \
 "s4_8_50_20:300:$T --wide-split 4 --k 50 --p 20 --shard-mib 1 --stripes 64"
