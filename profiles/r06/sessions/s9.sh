#!/bin/bash
# Round 6, session 9: the bench's slow pinned-host flat encode leg inside the
# bench's own sequence, variants at that point, then the same under a
# memory-copy + kernel trace (which engine / queue each copy takes, overlap).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}" || exit 1
export TMPDIR=/tmp
bash tools/gpu_session.sh \
 "zerocopy:300:python3 -u tools/zerocopy_probe.py" \
 "probe:400:python3 -u tools/e2e_bench_probe.py" \
 "probe_trace:500:rocprofv3 --memory-copy-trace --kernel-trace --output-format csv -d gpurun_out/e2e_trace -o e2e -- python3 -u tools/e2e_bench_probe.py"
