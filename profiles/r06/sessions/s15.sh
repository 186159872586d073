#!/bin/bash
# Round 6, session 15: output groups past 64 parity rows -- the wide-codec GPU
# tests, then GF(2^8) 128+128 encode rates on the group modules, and 4+66
# against its round-5 8 x 32 block modules (RSE_OPT_WIDE_BLOCK_INPUTS 0).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}" || exit 1
export TMPDIR=/tmp
T="python -u -m pytest -x -q -m gpu --timeout 300 --timeout-method thread"
bash tools/gpu_session.sh \
 "wide_tests:600:$T tests/test_gpu_parity.py -k 'wide'" \
 "g128_1m:200:python3 -u tools/tune.py --k 128 --p 128 --shard-mib 1 --stripes 128 --nt-only --shapes 0:0 --rounds 5" \
 "g128_1k:200:python3 -u tools/tune.py --k 128 --p 128 --shard-kib 1 --stripes 1024 --nt-only --shapes 0:0 --rounds 5" \
 "g466_groups:200:python3 -u tools/tune.py --k 4 --p 66 --shard-mib 1 --stripes 256 --nt-only --shapes 0:0 --rounds 5" \
 "g466_blocks:300:python3 -u tools/tune.py --k 4 --p 66 --shard-mib 1 --stripes 256 --nt-only --shapes 0:0 --rounds 5 --set 46=0"
