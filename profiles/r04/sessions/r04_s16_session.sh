#!/bin/bash
# Round 4, session 16: the bench with its reconstruct_batch leg.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
bash tools/gpu_session.sh "bench:500:python3 -u bench.py"
