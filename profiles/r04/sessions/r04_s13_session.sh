#!/bin/bash
# Round 4, session 13: decode-pattern kernels for 4-16 KiB shards.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
export RSE_JIT_CACHE_DIR=$PWD/jitcache
bash tools/gpu_session.sh \
 "tests:600:python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_host_paths.py -m gpu -k 'pattern or reconstruct'"
