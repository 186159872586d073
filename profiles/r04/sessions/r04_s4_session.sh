#!/bin/bash
# Round 4, session 4: the depth-2 pair variant (RSE_OPT_RECON_PAIRS 7) and
# run-time codecs' verify completion word -- parity tests first; then the
# 8-erasure A/B, reconstruct_batch with the host trims (planner workspace
# kept per lease, runs scan cut short), its runtime trace, and the bench.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
export RSE_JIT_CACHE_DIR=$PWD/jitcache
T16="python3 -u tools/tune.py --nt-only --field 16 --k 20 --p 8 --shapes 0:0"
bash tools/gpu_session.sh \
 "tests:500:python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_bench_checks.py tests/test_gpu_parity.py tests/test_gpu_host_paths.py -m gpu -k 'bench or wave_pairs or batch or every_mixing or jit_verify or verify'" || exit $?
grep -q " passed" gpurun_out/tests.log && ! grep -q -E "[0-9]+ failed" gpurun_out/tests.log || exit 1
bash tools/gpu_session.sh \
 "r8ab:300:$T16 --rounds 5 --shard-mib 4 --stripes 128 --op reconstruct --patterns 0 --erase 0,1,2,3,4,5,6,7 --recon-mix 3 --ab 28=1,3,7" \
 "r8ab256:300:$T16 --rounds 3 --shard-mib 4 --stripes 256 --op reconstruct --patterns 0 --erase 0,1,2,3,4,5,6,7 --recon-mix 3 --ab 28=1,7" \
 "b4k_e4:300:$T16 --rounds 3 --shard-kib 4 --stripes 65536 --op batch --erase 0,1,2,3" \
 "b4k_e8:300:$T16 --rounds 3 --shard-kib 4 --stripes 65536 --op batch --erase 0,1,2,3,4,5,6,7 --ab 28=1,7" \
 "b4k_rt:200:rocprofv3 --runtime-trace --kernel-trace --stats --output-format csv -d gpurun_out/b4k_rt -o t -- python3 tools/tune.py --rounds 2 --nt-only --shapes 0:0 --field 16 --k 20 --p 8 --shard-kib 4 --stripes 65536 --op batch --erase 0,1,2,3" \
 "bench:400:python3 -u bench.py"
