#!/bin/bash
# Common-subexpression budget (RSE_OPT_JIT_CSE) of run-time specialised
# GF(2^16) networks; one process per budget (modules are cached per process).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
T="python -u tools/tune.py --field 16 --shard-mib 4 --rounds 3 --nt-only"
bash tools/gpu_session.sh \
 "e12_8_b0:300:$T --k 12 --p 8 --stripes 256 --shapes 8192:1 --jit-cse 0" \
 "e12_8_b8:300:$T --k 12 --p 8 --stripes 256 --shapes 8192:1 --jit-cse 8" \
 "e12_8_b16:300:$T --k 12 --p 8 --stripes 256 --shapes 8192:1 --jit-cse 16" \
 "e10_4_b0:300:$T --k 10 --p 4 --stripes 256 --shapes 4096:1,8192:1 --jit-cse 0" \
 "e10_4_b16:300:$T --k 10 --p 4 --stripes 256 --shapes 4096:1,8192:1 --jit-cse 16" \
 "e24_8_b0:300:$T --k 24 --p 8 --stripes 256 --shapes 8192:1 --jit-cse 0" \
 "e24_8_b16:300:$T --k 24 --p 8 --stripes 256 --shapes 8192:1 --jit-cse 16"
