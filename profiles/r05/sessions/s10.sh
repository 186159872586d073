#!/bin/bash
# Round 5, session 10: how many resident workgroups a synchronous request
# should take (RSE_OPT_DISPATCH_LANE_UNITS 1 / 2 / 4 at 8 and 16 resident
# workgroups, 4-64 KiB 10+4 shards: latency probe case K), and the dispatcher
# tests.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}" || exit 1
export TMPDIR=/tmp
bash tools/gpu_session.sh \
 "latency:300:./tools/bin/latency_probe" \
 "dispatch:300:python3 -u -m pytest tests/test_gpu_dispatch.py -x -q --timeout 120 --timeout-method thread"
