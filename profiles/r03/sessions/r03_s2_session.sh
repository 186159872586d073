#!/bin/bash
# GPU suite at HEAD (wave pairs default, run-time pair modules), wide
# occupancy A/B, then the bench.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
bash tools/gpu_session.sh \
 "pytest:900:python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread" || exit $?
bash tools/wide_occ_session.sh || exit $?
bash tools/gpu_session.sh "bench:600:python3 -u bench.py"
