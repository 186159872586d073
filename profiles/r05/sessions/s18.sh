#!/bin/bash
# Round 5, session 18: the GF(2^16) 1000+24 chain at 2 outputs per wave
# (RSE_OPT_WIDE_SPLIT 2: 16-wave workgroups, <= 128 VGPRs by construction, 4
# waves per SIMD) against the default (4 waves of 6 outputs), alternating.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}" || exit 1
export TMPDIR=/tmp
TU="python3 tools/tune.py --rounds 9 --nt-only --shapes 0:0"
G16="--field 16 --k 1000 --p 24 --shard-kib 64 --stripes 128"
bash tools/gpu_session.sh \
 "g16s2:400:for i in 1 2; do $TU $G16 && $TU $G16 --set 18=2 || exit 1; done"
