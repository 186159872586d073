#!/bin/bash
# Round 6, session 21: FFT kernels exchanging one plane quad at a time (half
# the LDS: two workgroups per CU at 64+64) -- tests, then same-process A/Bs.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}" || exit 1
export TMPDIR=/tmp
T="python -u -m pytest -x -q -m gpu --timeout 120 --timeout-method thread"
A="--nt-only --shapes 0:0 --rounds 9 --ab 55=0,1"
bash tools/gpu_session.sh \
 "fft_tests:300:$T tests/test_gpu_fft.py" \
 "ab64:200:python3 -u tools/tune.py --k 64 --p 64 --shard-kib 1 --stripes 2048 $A" \
 "ab32:200:python3 -u tools/tune.py --k 32 --p 32 --shard-kib 1 --stripes 4096 $A" \
 "ab16:200:python3 -u tools/tune.py --k 16 --p 16 --shard-kib 1 --stripes 8192 $A" \
 "ab64m:200:python3 -u tools/tune.py --k 64 --p 64 --shard-mib 1 --stripes 64 $A"
