#!/bin/bash
# Round 6, session 18: the GPU suite on an EMPTY JIT cache (VERDICT r05 item
# 5): every run-time module built on the box while the tests run; per-test
# limit 170 s so a test waiting on a build ends (and prints) within gpurun's
# 3-minute silence limit.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}" || exit 1
export TMPDIR=/tmp
mkdir -p /tmp/rse_empty_cache gpurun_out/s18
export RSE_JIT_CACHE_DIR=/tmp/rse_empty_cache RSE_TEST_JIT_BUDGET_S=60
bash tools/gpu_session.sh \
 "cold_suite:1100:python -u -m pytest tests -m gpu -v --timeout 170 --timeout-method thread -p no:cacheprovider --durations=30"
