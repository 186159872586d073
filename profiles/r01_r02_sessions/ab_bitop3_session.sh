#!/bin/bash
# Same-box A/B: transposes on v_bitop3 (in-tree build) against v_bfi
# (tools/bin/librse_hip_prev.so), alternating processes; plus the VALU probe and
# the slicing parity tests on the new build.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export RSE_JIT_CACHE_DIR="$PWD/jitcache"
PREV="RSE_LIB_PATH=$PWD/tools/bin/librse_hip_prev.so"
H="python -u tools/tune.py --rounds 3 --nt-only --shapes 0:0 --stripes 512"
G="python -u tools/tune.py --rounds 3 --nt-only --shapes 0:0 --field 16 --k 20 --p 8 --shard-mib 4 --stripes 256"
R8="$G --op reconstruct --erase 0,1,2,3,4,5,6,7 --patterns 0"
W="python -u tools/tune.py --rounds 3 --nt-only --shapes 0:0 --k 50 --p 20 --shard-mib 1 --stripes 128"
W16="python -u tools/tune.py --rounds 3 --nt-only --shapes 0:0 --field 16 --k 40 --p 12 --shard-mib 1 --stripes 128"
bash tools/gpu_session.sh \
 "valu:120:./tools/bin/valu_probe" \
 "parity:300:python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 240 --timeout-method thread -k 'bitslice_matches or reconstruct_every_mixing or wide_codec_kernels'" \
 "h_new1:120:$H" "h_prev1:120:env $PREV $H" "h_new2:120:$H" "h_prev2:120:env $PREV $H" \
 "g_new1:120:$G" "g_prev1:120:env $PREV $G" "g_new2:120:$G" "g_prev2:120:env $PREV $G" \
 "r8_new1:120:$R8" "r8_prev1:120:env $PREV $R8" "r8_new2:120:$R8" "r8_prev2:120:env $PREV $R8" \
 "w_new1:120:$W" "w_prev1:120:env $PREV $W" "w_new2:120:$W" "w_prev2:120:env $PREV $W" \
 "w16_new1:120:$W16" "w16_prev1:120:env $PREV $W16"
