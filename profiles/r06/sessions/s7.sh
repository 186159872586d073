#!/bin/bash
# Round 6, session 7: the whole GPU suite and smoke() on the round's library
# with the tree's prebuilt JIT cache (tools/prebuild_all.sh, 64 min on 8 cores).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}" || exit 1
export TMPDIR=/tmp
bash tools/gpu_session.sh \
 "suite:1000:python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread --maxfail=10 --durations=25 -p no:cacheprovider" \
 "smoke:120:python -u -c 'import __graft_entry__ as g; g.smoke()'"
