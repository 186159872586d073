#!/bin/bash
# Headline shape (10+4 x 16 MiB, 512 stripes): default variant 1 against
# variant 5 (two inputs in flight) and 7 (XCD order), in two processes.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
H="python3 -u tools/tune.py --rounds 5 --nt-only --k 10 --p 4 --shard-mib 16 --stripes 512 --variant-list 1,5,7 --shapes 0:0,8192:0"
bash tools/gpu_session.sh "h1:600:$H" "h2:600:$H" \
 "t102:600:python3 -u tools/tune.py --rounds 5 --nt-only --k 10 --p 2 --shard-mib 1 --stripes 2048 --variant-list 1,2,5 --shapes 0:0,16384:0"
for f in h1 h2 t102; do grep -A8 "GB/s" gpurun_out/$f.log | head -8; done
