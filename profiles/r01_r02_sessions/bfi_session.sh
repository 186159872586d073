#!/bin/bash
# A/B on one box: the library with explicit v_bfi transposes (in-tree) against
# the previous commit's build (build-prev/, RSE_LIB_PATH), configuration by
# configuration, after the GPU tests of the bit-sliced kernels.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
P="python -u -m pytest -x -q --timeout 600 --timeout-method thread"
T="python -u tools/tune.py --rounds 5 --nt-only --shapes 0:0 --bitslice 1"
PREV="RSE_LIB_PATH=$PWD/build-prev/librse_hip.so"
steps=("pytest_bs:900:$P tests/test_gpu_parity.py -k 'bitslice or kernel_variants or specialised or wide or reconstruct'")
add() {  # name secs args
  steps+=("$1_new:$2:$T $3" "$1_prev:$2:$PREV $T $3")
}
add e16_20_8 300 "--field 16 --k 20 --p 8 --shard-mib 4 --stripes 256"
add e8_10_4 300 "--k 10 --p 4 --stripes 128"
add e16_12_8 300 "--field 16 --k 12 --p 8 --shard-mib 4 --stripes 256"
add w8_50_20 400 "--k 50 --p 20 --shard-mib 1 --stripes 64"
add w16_40_12 400 "--field 16 --k 40 --p 12 --shard-mib 1 --stripes 64"
add r16_e8 300 "--op reconstruct --patterns 0 --field 16 --k 20 --p 8 --shard-mib 4 --stripes 256 --erase 0,1,2,3,4,5,6,7"
add r16_e4 300 "--op reconstruct --patterns 0 --field 16 --k 20 --p 8 --shard-mib 4 --stripes 256 --erase 0,1,2,3"
bash tools/gpu_session.sh "${steps[@]}"
