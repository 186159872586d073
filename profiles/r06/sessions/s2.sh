#!/bin/bash
# Round 6, session 2: pinned host stripes coded in place (zero-copy) against the
# pipeline and the copy engines; the dispatcher with one agent acquire per
# request (its tests, then its latency and the device-sync / other-stream
# patterns by idle time).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}" || exit 1
export TMPDIR=/tmp
bash tools/gpu_session.sh \
 "zerocopy:300:python3 -u tools/zerocopy_probe.py" \
 "dispatch_tests:300:python -u -m pytest tests/test_gpu_dispatch.py -x -q -m gpu --timeout 120 --timeout-method thread" \
 "latency:300:./tools/bin/latency_probe ICL"
