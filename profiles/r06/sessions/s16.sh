#!/bin/bash
# Round 6, session 16: the wide-codec tests again after the module budget fix.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}" || exit 1
export TMPDIR=/tmp
T="python -u -m pytest -x -q -m gpu --timeout 300 --timeout-method thread"
bash tools/gpu_session.sh "wide_tests:600:$T tests/test_gpu_parity.py -k 'wide'"
