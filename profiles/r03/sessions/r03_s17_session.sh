#!/bin/bash
# First-use (syndrome) reconstruct of the compiled 10+4 codec: workgroups x
# inputs in flight, 2 and 4 lost data shards (decode-pattern kernels off);
# 10+2 x 1 MiB encode: the new default grid (16384 at <= 2 outputs) against 4096.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
T="python3 -u tools/tune.py --rounds 5 --nt-only --op reconstruct --patterns 0 --k 10 --p 4 --shard-mib 16 --stripes 256 --shapes 4096:0,8192:0,16384:0,32768:0 --recon-depth 1,2"
bash tools/gpu_session.sh "r2:600:$T --erase 0,1" "r4:600:$T --erase 0,1,2,3" \
 "e102:600:python3 -u tools/tune.py --rounds 7 --nt-only --k 10 --p 2 --shard-mib 1 --stripes 2048 --variant-list 5 --shapes 0:0,4096:0"
for f in r2 r4 e102; do grep -A8 "GB/s" gpurun_out/$f.log | head -9; done
