#!/bin/bash
# Small shards (benches/bandwidth.rs uses 1-16 KiB) through the flat API:
# many stripes per launch; launch shapes of the table kernels (0:0 = the
# library's automatic shape).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
T="python -u tools/tune.py --k 10 --p 4 --rounds 3 --nt-only"
bash tools/gpu_session.sh \
 "kib1:300:$T --shard-kib 1 --stripes 262144 --shapes 0:0,0:1,16:0,4:0,64:0,1:0" \
 "kib4:300:$T --shard-kib 4 --stripes 65536 --shapes 0:0,0:1,16:0,4:0,64:0,1:0" \
 "kib16:300:$T --shard-kib 16 --stripes 16384 --shapes 0:0,2048:1,4096:1 --bitslice 1,0" \
 "mib16_table:300:$T --shard-mib 16 --stripes 128 --shapes 0:0,0:1,2048:1 --bitslice 0" \
 "gf16_kib2:300:$T --field 16 --k 20 --p 8 --shard-kib 2 --stripes 32768 --shapes 0:0,0:1,16:0"
