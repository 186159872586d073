#!/bin/bash
# Headline profile: rocprofv3 kernel trace + stats of the bench command, then
# the PMC traffic passes (separate runs, one counter each).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
bash tools/gpu_session.sh \
 "trace:600:rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_trace -o bench -- python3 bench.py --no-cpu --steps 10" \
 "pmc:900:python3 tools/pmc_traffic.py --tag r01final --steps 5"
