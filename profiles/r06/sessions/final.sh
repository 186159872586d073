#!/bin/bash
# Round 6, final library: the whole GPU suite and smoke(); the default bench;
# the bench's headline under a kernel trace (per-dispatch rows of the
# 512-stripe launches); the PMC traffic file of the same library.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out/final
bash tools/gpu_session.sh \
 "suite:900:python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread --maxfail=10 -p no:cacheprovider" \
 "smoke:120:python -u -c 'import __graft_entry__ as g; g.smoke()'" \
 "bench:600:python -u bench.py --full-out gpurun_out/final/bench_full_n1.json" \
 "trace:300:rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/final/trace -o b -- python3 -u bench.py --no-cpu --no-extras" \
 "pmc:300:python3 -u tools/pmc_traffic.py --tag r06final"
