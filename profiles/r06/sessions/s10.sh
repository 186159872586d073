#!/bin/bash
# Round 6, session 10: host pipeline with outputs stored in place (no D2H
# copies, RSE_OPT_HOST_ZC_OUT): host-path tests, the bench-sequence probe
# with zc on/off, then the full bench.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}" || exit 1
export TMPDIR=/tmp
T="python -u -m pytest -x -q -m gpu --timeout 120 --timeout-method thread"
bash tools/gpu_session.sh \
 "host_tests:600:$T tests/test_gpu_host_paths.py" \
 "probe:400:python3 -u tools/e2e_bench_probe.py" \
 "bench:900:python -u bench.py"
