#!/bin/bash
# The whole GPU suite and the smoke test at HEAD.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
bash tools/gpu_session.sh \
 "smoke:300:python3 -c 'import __graft_entry__ as g; g.smoke()'" \
 "pytest:900:python3 -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread --durations=40"
