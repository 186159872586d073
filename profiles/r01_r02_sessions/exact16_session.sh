#!/bin/bash
# GF(2^16) exact-decomposition networks: the compiled 20+8 codec (variant 0,
# its network now from factor16) against variant 9 (no temporaries) in one
# process; run-time GF(2^16) codecs with RSE_OPT_JIT_EXACT 1 (default) against
# 0 (pair/triple greedy), one process each; then the full GPU suite.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
P="python -u -m pytest -x -q --timeout 300 --timeout-method thread"
T="python -u tools/tune.py --rounds 5 --nt-only --shapes 0:0 --bitslice 1"
E16="--field 16 --k 20 --p 8 --shard-mib 4 --stripes 256"
W16="--field 16 --k 40 --p 12 --shard-mib 1 --stripes 64"
N16="--field 16 --k 12 --p 8 --shard-mib 4 --stripes 64"
R="--op reconstruct --patterns 0"
bash tools/gpu_session.sh \
 "e16:300:$T $E16 --variant-list 0,9" \
 "r16_e8:300:$T $E16 $R --erase 0,1,2,3,4,5,6,7" \
 "r16_e4:300:$T $E16 $R --erase 0,1,2,3" \
 "w40_exact:300:$T $W16" \
 "w40_greedy:300:$T $W16 --set 23=0" \
 "n12_exact:300:$T $N16" \
 "n12_greedy:300:$T $N16 --set 23=0" \
 "pytest:900:$P tests -m gpu"
