#!/bin/bash
# Round 5, session 21: reconstruct of one lost data shard, 16+16 x 1 KiB (the
# reference bench's reconstruct_one): 8192 stripes per launch as the bench
# matrix runs it, against 65536 -- whether the short launch, not the kernel's
# rate, is what reads low.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}" || exit 1
export TMPDIR=/tmp
TR="python3 tools/tune.py --op reconstruct --erase 0 --k 16 --p 16 --shard-kib 1 --rounds 9 --nt-only --shapes 0:0"
bash tools/gpu_session.sh \
 "r16:300:for i in 1 2; do $TR --stripes 8192 && $TR --stripes 65536 || exit 1; done"
