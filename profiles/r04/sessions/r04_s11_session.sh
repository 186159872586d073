#!/bin/bash
# Round 4, session 11: the batch scan's atomics per workgroup, the wide launch
# shape taken from the module (session 10's launch failure under a changed
# RSE_OPT_WIDE_SPLIT), and 100+30 at 4 outputs per wave built for it (--set).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
export RSE_JIT_CACHE_DIR=$PWD/jitcache
T16="python3 -u tools/tune.py --nt-only --field 16 --shapes 0:0"
bash tools/gpu_session.sh \
 "tests:600:python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_host_paths.py -m gpu -k 'batch or wide_launch or sub_chunk'" || exit $?
grep -q " passed" gpurun_out/tests.log && ! grep -q -E "[0-9]+ failed" gpurun_out/tests.log || exit 1
bash tools/gpu_session.sh \
 "b4k_trace:200:rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/b4k_trace -o t -- python3 tools/batch_probe.py --erasures 4 --calls 10 --device-flags" \
 "probe_e4d:200:python3 -u tools/batch_probe.py --erasures 4 --calls 20 --device-flags" \
 "probe_e8d:200:python3 -u tools/batch_probe.py --erasures 8 --calls 20 --device-flags" \
 "w100_def:300:$T16 --k 100 --p 30 --rounds 3 --shard-mib 1 --stripes 128" \
 "w100_split4:300:$T16 --k 100 --p 30 --rounds 3 --shard-mib 1 --stripes 128 --set 18=4"
