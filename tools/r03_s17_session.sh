#!/bin/bash
# First-use (syndrome) reconstruct of the compiled 10+4 codec: workgroups x
# inputs in flight, 2 and 4 lost data shards (decode-pattern kernels off).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
T="python3 -u tools/tune.py --rounds 5 --nt-only --op reconstruct --patterns 0 --k 10 --p 4 --shard-mib 16 --stripes 256 --shapes 4096:0,8192:0,16384:0,32768:0 --recon-depth 1,2"
bash tools/gpu_session.sh "r2:600:$T --erase 0,1" "r4:600:$T --erase 0,1,2,3"
for f in r2 r4; do grep -A8 "GB/s" gpurun_out/$f.log | head -9; done
