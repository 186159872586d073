#!/bin/bash
# Round 4, session 5: the whole GPU suite (depth-2 pair kernel now the
# default, host calls' direct path), reconstruct_batch per call, the bench.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
export RSE_JIT_CACHE_DIR=$PWD/jitcache
bash tools/gpu_session.sh \
 "tests:900:python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests -m gpu" || exit $?
grep -q " passed" gpurun_out/tests.log && ! grep -q -E "[0-9]+ failed" gpurun_out/tests.log || exit 1
bash tools/gpu_session.sh \
 "probe_e4:200:python3 -u tools/batch_probe.py --erasures 4 --calls 20" \
 "probe_e8:200:python3 -u tools/batch_probe.py --erasures 8 --calls 20" \
 "bench:400:python3 -u bench.py"
