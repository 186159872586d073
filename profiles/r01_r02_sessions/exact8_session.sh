#!/bin/bash
# GF(2^8) run-time networks: exact-decomposition temporaries (RSE_OPT_JIT_EXACT8
# 1, default) against the pair/triple greedy (0), and no temporaries (JIT_CSE
# 0: round 2's narrow GF(2^8) codecs), one process per configuration.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
P="python -u -m pytest -x -q --timeout 900 --timeout-method thread"
T="python -u tools/tune.py --rounds 5 --nt-only --shapes 0:0 --bitslice 1"
W8="--k 50 --p 20 --shard-mib 1 --stripes 64"
W10="--k 10 --p 16 --shard-mib 1 --stripes 256"
N12="--k 12 --p 8 --shard-mib 4 --stripes 64"
bash tools/gpu_session.sh \
 "pytest:900:$P tests/test_gpu_parity.py -k 'wide or jit or JIT'" \
 "w50_exact:300:$T $W8" \
 "w50_greedy:300:$T $W8 --set 23=0" \
 "w10_exact:300:$T $W10" \
 "w10_greedy:300:$T $W10 --set 23=0" \
 "n12_exact:300:$T $N12" \
 "n12_none:300:$T $N12 --set 13=0"
