#!/bin/bash
# reconstruct_batch on the bit-sliced per-stripe path vs the table planner path.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
B="python -u tools/tune.py --op batch --rounds 3 --nt-only --bitslice 1,0 --shapes 4096:1,8192:1"
bash tools/gpu_session.sh \
 "pytest:900:python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread" \
 "batch_10_4:300:$B --k 10 --p 4 --stripes 128 --erase 0,1" \
 "batch_20_8:300:$B --field 16 --k 20 --p 8 --shard-mib 4 --stripes 256 --erase 0,1,2,3"
