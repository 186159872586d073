#!/bin/bash
# Wide codecs (k > 32 or p > 8): table kernels with input/output chunking.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
T="python -u tools/tune.py --rounds 2 --nt-only --shapes 0:0"
bash tools/gpu_session.sh \
 "w8_50_20:300:$T --k 50 --p 20 --shard-mib 1 --stripes 64" \
 "w8_10_16:300:$T --k 10 --p 16 --shard-mib 1 --stripes 256" \
 "w16_100_30:300:$T --field 16 --k 100 --p 30 --shard-mib 1 --stripes 32" \
 "w16_200_56:300:$T --field 16 --k 200 --p 56 --shard-kib 256 --stripes 32"
