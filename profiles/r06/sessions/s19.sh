#!/bin/bash
# Round 6, session 19: GF(2^16) 1000+24 on chains of 3 blocks of 333-334
# inputs (RSE_OPT_WIDE_BLOCK_INPUTS 400) against 8 of 125: the chain tests,
# then a same-process A/B at the bench's 512 stripes x 64 KiB.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}" || exit 1
export TMPDIR=/tmp
T="python -u -m pytest -x -v -m gpu --timeout 300 --timeout-method thread"
bash tools/gpu_session.sh \
 "chain_tests:400:$T tests/test_gpu_parity.py -k 'block_chain'" \
 "ab:400:python3 -u tools/tune.py --field 16 --k 1000 --p 24 --shard-kib 64 --stripes 512 --nt-only --shapes 0:0 --rounds 5 --ab 46=128,400"
