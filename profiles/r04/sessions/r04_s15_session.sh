#!/bin/bash
# Round 4, session 15: GF(2^16) 100+30 (subfield, GF(2^8) wide module)
# variants, each module built for its options (--set): default, networks per
# input instead of input pairs (29=0), 3 waves per SIMD (20=3).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
export RSE_JIT_CACHE_DIR=$PWD/jitcache
T16="python3 -u tools/tune.py --nt-only --field 16 --shapes 0:0 --k 100 --p 30 --rounds 3 --shard-mib 1 --stripes 128"
bash tools/gpu_session.sh \
 "w100_def:300:$T16" \
 "w100_nopairs:300:$T16 --set 29=0" \
 "w100_occ3:300:$T16 --set 20=3" \
 "w100_def2:300:$T16"
