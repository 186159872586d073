#!/bin/bash
# Round 6, session 8: the default bench (every leg) on the round's library.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}" || exit 1
export TMPDIR=/tmp
bash tools/gpu_session.sh "bench:900:python -u bench.py"
