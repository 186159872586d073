#!/bin/bash
# Round 6, session 17: the default bench with the host legs timed over 10 calls.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}" || exit 1
export TMPDIR=/tmp
bash tools/gpu_session.sh "bench:600:python -u bench.py --full-out gpurun_out/s17/bench_full_n1.json"
