#!/bin/bash
# Round 5, sessions 4+5 in one call (no box was free for session 4 alone),
# after the multi-workgroup dispatcher: its tests and the latency sweep first.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}" || exit 1
export TMPDIR=/tmp
bash tools/gpu_session.sh "latency:200:./tools/bin/latency_probe" || exit $?
bash profiles/r05/sessions/s4.sh || exit $?
bash profiles/r05/sessions/s5.sh
