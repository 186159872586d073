#!/bin/bash
# Horner nibble dispatch as an opaque binary tree of uniform branches, and the
# pair kernel back to 141 VGPRs without the prefetch state: the in-tree
# library against tools/bin/librse_hip_prev.so (before both), alternating
# processes; parity first.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
PREV="RSE_LIB_PATH=$PWD/tools/bin/librse_hip_prev.so"
T16="python3 -u tools/tune.py --rounds 3 --nt-only --field 16 --k 20 --p 8 --shapes 0:0 --shard-mib 4 --stripes 128"
R8="$T16 --op reconstruct --patterns 0 --erase 0,1,2,3,4,5,6,7 --recon-mix 3 --ab 28=1,0"
R4="$T16 --op reconstruct --patterns 0 --erase 0,1,2,3 --recon-mix 3"
B8="$T16 --op batch --erase 0,1,2,3,4,5,6,7"
R8_10="python3 -u tools/tune.py --rounds 3 --nt-only --shapes 0:0 --k 10 --p 4 --stripes 128 --op reconstruct --patterns 0 --erase 0,1,2,3"
bash tools/gpu_session.sh \
 "pytest:600:python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py -m gpu -k 'wave_pairs or every_mixing or reconstruct'" || exit $?
grep -q " passed" gpurun_out/pytest.log && ! grep -q -E "[0-9]+ failed" gpurun_out/pytest.log || exit 1
bash tools/gpu_session.sh \
 "r8_new1:200:$R8" "r8_prev1:200:env $PREV $R8" "r8_new2:200:$R8" "r8_prev2:200:env $PREV $R8" \
 "r4_new1:200:$R4" "r4_prev1:200:env $PREV $R4" \
 "b8_new1:200:$B8" "b8_prev1:200:env $PREV $B8" \
 "g4_new1:200:$R8_10" "g4_prev1:200:env $PREV $R8_10"
grep -H median gpurun_out/r8_*.log gpurun_out/r4_*.log gpurun_out/b8_*.log gpurun_out/g4_*.log
