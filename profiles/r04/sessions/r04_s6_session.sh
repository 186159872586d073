#!/bin/bash
# Round 4, session 6: the cooperative batch planner (8 lanes per stripe) and
# device-resident flags for reconstruct_batch: the batch tests, then per-call
# timing with host and device flags, and a kernel + runtime trace.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
export RSE_JIT_CACHE_DIR=$PWD/jitcache
bash tools/gpu_session.sh \
 "tests:500:python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_host_paths.py tests/test_bench_checks.py -m gpu -k 'batch or wave_pairs or bench or host_direct'" || exit $?
grep -q " passed" gpurun_out/tests.log && ! grep -q -E "[0-9]+ failed" gpurun_out/tests.log || exit 1
bash tools/gpu_session.sh \
 "probe_e4:200:python3 -u tools/batch_probe.py --erasures 4 --calls 20" \
 "probe_e4d:200:python3 -u tools/batch_probe.py --erasures 4 --calls 20 --device-flags" \
 "probe_e8:200:python3 -u tools/batch_probe.py --erasures 8 --calls 20" \
 "probe_e8d:200:python3 -u tools/batch_probe.py --erasures 8 --calls 20 --device-flags" \
 "probe_4m:200:python3 -u tools/batch_probe.py --erasures 4 --calls 10 --shard-kib 4096 --stripes 128" \
 "rt_e4d:200:rocprofv3 --runtime-trace --kernel-trace --stats --output-format csv -d gpurun_out/rt_e4d -o t -- python3 tools/batch_probe.py --erasures 4 --calls 5 --device-flags"
