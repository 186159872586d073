#!/bin/bash
# Round 6, session 20: GF(2^16) 1000+24 x 64 KiB, 512 stripes: chains of 8
# blocks (RSE_OPT_WIDE_BLOCK_INPUTS 128, default) against 3 (400), each set at
# codec creation, alternating processes; then the chain tests.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}" || exit 1
export TMPDIR=/tmp
B="python3 -u tools/tune.py --field 16 --k 1000 --p 24 --shard-kib 64 --stripes 512 --nt-only --shapes 0:0 --rounds 5"
T="python -u -m pytest -x -v -m gpu --timeout 300 --timeout-method thread"
bash tools/gpu_session.sh \
 "b128a:200:$B --set 46=128" "b400a:200:$B --set 46=400" \
 "b128b:200:$B --set 46=128" "b400b:200:$B --set 46=400" \
 "chain_tests:400:$T tests/test_gpu_parity.py -k 'block_chain'"
