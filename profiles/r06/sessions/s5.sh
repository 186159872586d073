#!/bin/bash
# Round 6, session 5: dispatcher on a low-priority stream, pipeline D2H at high
# priority: the dispatcher and host-path tests, the queue probe, and what the
# dispatcher's idle time costs device-synchronising / other-stream callers.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}" || exit 1
export TMPDIR=/tmp
T="python -u -m pytest -x -q -m gpu --timeout 120 --timeout-method thread"
bash tools/gpu_session.sh \
 "dispatch_tests:300:$T tests/test_gpu_dispatch.py" \
 "queue_probe:300:python3 -u tools/queue_probe.py" \
 "sync_probe:300:python3 -u tools/dispatch_sync_probe.py" \
 "host_tests:700:$T tests/test_gpu_host_paths.py"
