#!/bin/bash
# Round 4, session 7: 1 / 2 KiB shards on the bit-sliced kernels (SUB chunks),
# the batch planner and device flags (session 6's list), and the reference
# bench matrix with prebuilt run-time modules.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
export RSE_JIT_CACHE_DIR=$PWD/jitcache
bash tools/gpu_session.sh \
 "sub:400:python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py -m gpu -k 'sub_chunk'" || exit $?
grep -q " passed" gpurun_out/sub.log && ! grep -q -E "[0-9]+ failed" gpurun_out/sub.log || exit 1
bash tools/gpu_session.sh \
 "tests:500:python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_host_paths.py tests/test_bench_checks.py -m gpu -k 'batch or wave_pairs or bench or host_direct or flat or verify'" \
 "matrix:400:python3 -u tools/ref_matrix.py" \
 "probe_e4:200:python3 -u tools/batch_probe.py --erasures 4 --calls 20" \
 "probe_e4d:200:python3 -u tools/batch_probe.py --erasures 4 --calls 20 --device-flags" \
 "probe_e8d:200:python3 -u tools/batch_probe.py --erasures 8 --calls 20 --device-flags"
