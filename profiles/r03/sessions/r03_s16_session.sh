#!/bin/bash
# Inputs in flight beyond the defaults: GF(2^16) 20+8 encode variants 0 / 5
# (two inputs in flight) / 1; syndrome reconstruct depth 1..3 for 10+4 (2 lost)
# and GF(2^16) 20+8 (4 lost), one process each.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
T="python3 -u tools/tune.py --rounds 5 --nt-only --shapes 0:0"
bash tools/gpu_session.sh \
 "e16:600:$T --field 16 --k 20 --p 8 --shard-mib 4 --stripes 256 --variant-list 0,5,1" \
 "r104:600:$T --op reconstruct --k 10 --p 4 --shard-mib 16 --stripes 256 --erase 0,1 --recon-depth 1,2,3" \
 "r16_4:600:$T --op reconstruct --field 16 --k 20 --p 8 --shard-mib 4 --stripes 256 --erase 0,1,2,3 --recon-depth 1,2,3"
for f in e16 r104 r16_4; do grep -A4 "GB/s" gpurun_out/$f.log | head -5; done
