#!/bin/bash
# Round 6, session 13: the batch reconstruct's 4 KiB chunks at 8 sigma rows on
# wave pairs (RSE_OPT_RECON_W4_PAIRS): correctness against the oracle, the
# batch GPU tests, then a same-process A/B of 0 / 1 / 2 and the bench's leg.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}" || exit 1
export TMPDIR=/tmp
T="python -u -m pytest -x -q -m gpu --timeout 120 --timeout-method thread"
B="python3 -u tools/tune.py --op batch --field 16 --k 20 --p 8 --shard-kib 4 --stripes 65536 --erase 0,1,2,3 --nt-only --shapes 0:0"
bash tools/gpu_session.sh \
 "w4p_tests:300:$T tests/test_gpu_parity.py -k 'wave_pairs or reconstruct_batch'" \
 "ab_parity:300:$B --batch-parity --rounds 9 --ab 54=0,1,2" \
 "ab_data:300:$B --rounds 9 --ab 54=0,1,2"
