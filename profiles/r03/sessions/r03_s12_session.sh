#!/bin/bash
# 10+2 x 1 MiB (BASELINE configs[1]) over bit-sliced variants and grids, one
# process (same placement for every configuration).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
bash tools/gpu_session.sh \
 "t102:600:python3 -u tools/tune.py --rounds 3 --nt-only --k 10 --p 2 --shard-mib 1 --stripes 2048 --variant-list 0,1,2,5,7,8 --shapes 0:0,2048:0,8192:0,16384:0" \
 "t104:600:python3 -u tools/tune.py --rounds 3 --nt-only --k 10 --p 4 --shard-mib 16 --stripes 256 --variant-list 0,1,2,5,7,8 --shapes 0:0,2048:0,8192:0"
grep -A30 "GB/s" gpurun_out/t102.log | head -30
grep -A20 "GB/s" gpurun_out/t104.log | head -20
