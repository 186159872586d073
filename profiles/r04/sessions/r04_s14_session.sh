#!/bin/bash
# Round 4, session 14: the syndrome reconstruct over 4 KiB chunks (first use
# of a pattern on 4-16 KiB shards and on the 4 KiB chunks past 16 KiB ones):
# tests, the whole suite, and its rate against the table kernels.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
export RSE_JIT_CACHE_DIR=$PWD/jitcache
T="python3 -u tools/tune.py --nt-only --shapes 0:0 --op reconstruct --patterns 0 --bitslice 1,0"
bash tools/gpu_session.sh \
 "first:400:python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py -m gpu -k 'syndrome_reconstruct_4k or bitslice_reconstruct_every or wave_pairs'" || exit $?
grep -q " passed" gpurun_out/first.log && ! grep -q -E "[0-9]+ failed" gpurun_out/first.log || exit 1
bash tools/gpu_session.sh \
 "suite:900:python3 -u -m pytest -q --timeout 300 --timeout-method thread tests -m gpu" \
 "r8k_10_4:300:$T --field 8 --k 10 --p 4 --shard-kib 8 --stripes 16384 --rounds 3 --erase 0,1" \
 "r4k_20_8:300:$T --field 16 --k 20 --p 8 --shard-kib 4 --stripes 16384 --rounds 3 --erase 0,1,2,3" \
 "r12k_6_3:300:$T --field 8 --k 6 --p 3 --shard-kib 12 --stripes 16384 --rounds 3 --erase 0,4,7"
