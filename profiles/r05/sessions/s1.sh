#!/bin/bash
# Round 5, session 1: the new/changed tests, then the default bench (compact line).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}" || exit 1
export TMPDIR=/tmp
bash tools/gpu_session.sh \
 "tests:400:python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k 'parity_only or flags_must_sit or bench_legs or wave_pairs or per_stripe_patterns or timing_splits'" \
 "bench:600:python3 -u bench.py"
