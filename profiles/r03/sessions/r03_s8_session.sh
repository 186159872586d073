#!/bin/bash
# GPU suite and bench at HEAD (paired wide networks, one wave pair per
# workgroup, short-launch grid), then a headline kernel trace.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
bash tools/gpu_session.sh \
 "pytest:900:python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread" \
 "bench:600:python3 -u bench.py" \
 "trace:400:rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/trace -o bench -- python3 bench.py --no-cpu --no-extras --steps 10"
