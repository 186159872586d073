#!/bin/bash
# Round 4, session 8: the GF(2^16) subfield route measured -- GF(2^16) 20+8
# 8-erasure reconstruct variants and depth on the GF(2^8) kernels, 100+30 and
# 40+12 wide codecs in GF(2^8) against their GF(2^16) kernels
# (RSE_OPT_SUBFIELD 0) -- and the tests that failed in session 7 (pattern
# budget, compiled kind).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
export RSE_JIT_CACHE_DIR=$PWD/jitcache
T16="python3 -u tools/tune.py --nt-only --field 16 --shapes 0:0"
bash tools/gpu_session.sh \
 "tests:600:python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py -m gpu -k 'run_time_specialised or decode_pattern or wide_reconstruct_pattern or wide_codec'" || exit $?
grep -q " passed" gpurun_out/tests.log && ! grep -q -E "[0-9]+ failed" gpurun_out/tests.log || exit 1
bash tools/gpu_session.sh \
 "r8ab:300:$T16 --k 20 --p 8 --rounds 5 --shard-mib 4 --stripes 256 --op reconstruct --patterns 0 --erase 0,1,2,3,4,5,6,7 --recon-mix 3 --ab 28=1,2,3,7" \
 "r8depth:300:$T16 --k 20 --p 8 --rounds 3 --shard-mib 4 --stripes 256 --op reconstruct --patterns 0 --erase 0,1,2,3,4,5,6,7 --recon-mix 3 --set 28=0 --recon-depth 1,2,3" \
 "w100:300:$T16 --k 100 --p 30 --rounds 3 --shard-mib 1 --stripes 128" \
 "w100_gf16:400:$T16 --k 100 --p 30 --rounds 3 --shard-mib 1 --stripes 128 --set 34=0" \
 "w40:300:$T16 --k 40 --p 12 --rounds 3 --shard-mib 1 --stripes 128" \
 "w40_gf16:300:$T16 --k 40 --p 12 --rounds 3 --shard-mib 1 --stripes 128 --set 34=0" \
 "b4k_e8:300:$T16 --k 20 --p 8 --rounds 3 --shard-kib 4 --stripes 65536 --op batch --erase 0,1,2,3,4,5,6,7 --ab 28=1,7"
