#!/bin/bash
# 4 KiB per-wave bit-sliced chunks: parity tests, then small-shard throughput.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
T="python -u tools/tune.py --rounds 3 --nt-only --shapes 0:0 --bitslice 1,0"
bash tools/gpu_session.sh \
 "pytest:1200:python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread" \
 "kib4:300:$T --k 10 --p 4 --shard-kib 4 --stripes 65536" \
 "kib8:300:$T --k 10 --p 4 --shard-kib 8 --stripes 32768" \
 "kib12:300:$T --k 10 --p 4 --shard-kib 12 --stripes 16384" \
 "g16_kib4:300:$T --field 16 --k 20 --p 8 --shard-kib 4 --stripes 16384" \
 "jit_kib4:300:$T --k 6 --p 3 --shard-kib 4 --stripes 65536" \
 "mib16:300:python -u tools/tune.py --rounds 3 --nt-only --shapes 0:0 --k 10 --p 4 --stripes 448"
