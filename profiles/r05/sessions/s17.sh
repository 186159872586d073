#!/bin/bash
# Round 5, session 17: the GF(2^16) 1000+24 chain at 3 outputs per wave and 4
# waves per SIMD (RSE_OPT_WIDE_SPLIT 4 + RSE_OPT_WIDE_OCCUPANCY 4: 8-wave
# workgroups of <= 128 VGPRs, two per CU) against the default (4 waves of 6
# outputs, ~240 VGPRs), alternating processes.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}" || exit 1
export TMPDIR=/tmp
TU="python3 tools/tune.py --rounds 9 --nt-only --shapes 0:0"
G16="--field 16 --k 1000 --p 24 --shard-kib 64 --stripes 128"
bash tools/gpu_session.sh \
 "g16o4:400:for i in 1 2; do $TU $G16 && $TU $G16 --set 18=4 --set 20=4 || exit 1; done"
