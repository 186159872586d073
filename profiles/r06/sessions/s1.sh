#!/bin/bash
# Round 6, session 1: the pinned-host flat encode leg --
# the same rse_encode_host_flat call after each step of a bench-like process,
# plus variants at the slow point; then the same under a copy/kernel trace.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}" || exit 1
export TMPDIR=/tmp
bash tools/gpu_session.sh \
 "probe:400:python3 -u tools/e2e_probe.py" \
 "probe_trace:500:rocprofv3 --memory-copy-trace --kernel-trace --output-format csv -d gpurun_out/e2e_trace -o e2e -- python3 -u tools/e2e_probe.py"
