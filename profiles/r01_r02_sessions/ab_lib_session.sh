#!/bin/bash
# Same-box A/B of two builds of the library (RSE_LIB_PATH): the current
# in-tree librse_hip.so against tools/bin/librse_hip_prev.so, alternating
# processes, for the headline encode and GF(2^16) 20+8 encode.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
PREV="RSE_LIB_PATH=$PWD/tools/bin/librse_hip_prev.so"
H="python -u tools/tune.py --rounds 3 --nt-only --shapes 0:0 --stripes 512"
G="python -u tools/tune.py --rounds 3 --nt-only --shapes 0:0 --field 16 --k 20 --p 8 --shard-mib 4 --stripes 256"
bash tools/gpu_session.sh \
 "h_new1:120:$H" "h_prev1:120:env $PREV $H" "h_new2:120:$H" "h_prev2:120:env $PREV $H" \
 "g_new1:120:$G" "g_prev1:120:env $PREV $G" "g_new2:120:$G" "g_prev2:120:env $PREV $G"
