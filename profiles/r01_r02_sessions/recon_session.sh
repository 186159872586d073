#!/bin/bash
# Reconstruct A/B: decode-pattern kernels (patterns=1) vs bit-sliced syndrome
# kernels (patterns=0, bitslice=1) vs table kernels (bitslice=0).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
T="python -u tools/tune.py --op reconstruct --rounds 3 --nt-only --bitslice 1,0 --patterns 1,0"
bash tools/gpu_session.sh \
 "rec_10_4_e2:300:$T --k 10 --p 4 --stripes 128 --shapes 4096:1,8192:1 --erase 0,1" \
 "rec_10_4_e1:300:$T --k 10 --p 4 --stripes 128 --shapes 4096:1,8192:1 --erase 3" \
 "rec_20_8_e8:300:$T --field 16 --k 20 --p 8 --shard-mib 4 --stripes 256 --shapes 4096:1,8192:1 --erase 0,1,2,3,4,5,6,7" \
 "rec_20_8_e4:300:$T --field 16 --k 20 --p 8 --shard-mib 4 --stripes 256 --shapes 4096:1,8192:1 --erase 0,1,2,3" \
 "enc_10_2:300:python -u tools/tune.py --k 10 --p 2 --stripes 128 --rounds 3 --shapes 4096:1 --nt-only"
