#!/bin/bash
# Encode variant 10 (4 waves/SIMD, GF(2^8) p <= 4) against the default (1) and
# plain (0) at 1..512 stripes of 10+4 x 16 MiB and 10+2 x 1 MiB.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
T="python -u tools/tune.py --rounds 7 --nt-only --shapes 0:0 --variant-list 1,0,10"
bash tools/gpu_session.sh \
 "s1:200:$T --stripes 1" \
 "s2:200:$T --stripes 2" \
 "s4:200:$T --stripes 4" \
 "s64:200:$T --stripes 64" \
 "s512:300:$T --stripes 512 --rounds 3" \
 "p2:200:$T --k 10 --p 2 --shard-mib 1 --stripes 2048" \
 "p2s1:200:$T --k 10 --p 2 --shard-mib 1 --stripes 1"
