#!/bin/bash
# Round 4, session 9: the field-dependent wave-pair default (GF(2^8): two
# pairs per workgroup) -- the pair tests, the 8-erasure A/Bs at 128 / 256
# stripes and in reconstruct_batch, a kernel trace of the 4 KiB batch (the
# 8-lane planner's time), and the bench.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
export RSE_JIT_CACHE_DIR=$PWD/jitcache
T16="python3 -u tools/tune.py --nt-only --field 16 --k 20 --p 8 --shapes 0:0"
bash tools/gpu_session.sh \
 "tests:600:python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_capi.py -m gpu -k 'wave_pairs or batch or every_mixing or bitslice_reconstruct_every'" || exit $?
grep -q " passed" gpurun_out/tests.log && ! grep -q -E "[0-9]+ failed" gpurun_out/tests.log || exit 1
bash tools/gpu_session.sh \
 "r8ab128:300:$T16 --rounds 5 --shard-mib 4 --stripes 128 --op reconstruct --patterns 0 --erase 0,1,2,3,4,5,6,7 --recon-mix 3 --ab 28=8,1,2" \
 "r8ab256:300:$T16 --rounds 5 --shard-mib 4 --stripes 256 --op reconstruct --patterns 0 --erase 0,1,2,3,4,5,6,7 --recon-mix 3 --ab 28=8,1,2" \
 "b4k_e8:300:$T16 --rounds 3 --shard-kib 4 --stripes 65536 --op batch --erase 0,1,2,3,4,5,6,7 --ab 28=8,1" \
 "b4k_trace:200:rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/b4k_trace -o t -- python3 tools/batch_probe.py --erasures 4 --calls 10 --device-flags" \
 "bench:400:python3 -u bench.py"
