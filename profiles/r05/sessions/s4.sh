#!/bin/bash
# Round 5, session 4: dispatcher tests and the N-rank rehearsals after their
# fixes; RSE_OPT_WIDE_GRID (launch in multiples of the resident workgroups) in
# one process per codec; GF(2^16) 1000+24 at 128 stripes; the bench.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}" || exit 1
export TMPDIR=/tmp
TU="python3 tools/tune.py --rounds 15 --nt-only --shapes 0:0 --ab 44=0,1,2,4"
bash tools/gpu_session.sh \
 "dispatch:300:python3 -u -m pytest tests/test_gpu_dispatch.py -x -q --timeout 120 --timeout-method thread" \
 "ranks:600:python3 -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread -k rehearsal" \
 "g64:200:$TU --k 64 --p 64 --shard-kib 1 --stripes 2048" \
 "g32:200:$TU --k 32 --p 32 --shard-kib 1 --stripes 4096" \
 "g16x16:200:$TU --k 16 --p 16 --shard-kib 1 --stripes 8192" \
 "g50k:200:$TU --k 50 --p 20 --shard-kib 1 --stripes 3744" \
 "g50m:200:$TU --k 50 --p 20 --shard-mib 1 --stripes 128" \
 "g40m:200:$TU --field 16 --k 40 --p 12 --shard-mib 1 --stripes 128" \
 "g100m:200:$TU --field 16 --k 100 --p 30 --shard-mib 1 --stripes 128" \
 "g1000:300:python3 tools/tune.py --rounds 10 --nt-only --shapes 0:0 --field 16 --k 1000 --p 24 --shard-kib 64 --stripes 128" \
 "bench:600:python3 -u bench.py"
