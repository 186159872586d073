#!/bin/bash
# Round 6, session 12: the batch reconstruct's 4 KiB-per-wave kernel by grid
# size (workgroups of 4 waves; 16384 = one stripe per wave, the default).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}" || exit 1
export TMPDIR=/tmp
B="python3 -u tools/tune.py --op batch --batch-parity --field 16 --k 20 --p 8 --shard-kib 4 --stripes 65536 --erase 0,1,2,3 --nt-only"
bash tools/gpu_session.sh \
 "grid:300:$B --shapes 0:0,1024:0,2048:0,4096:0,8192:0,16384:0 --rounds 7" \
 "grid_data:300:python3 -u tools/tune.py --op batch --field 16 --k 20 --p 8 --shard-kib 4 --stripes 65536 --erase 0,1,2,3 --nt-only --shapes 0:0,1024:0,2048:0,4096:0,8192:0 --rounds 7"
