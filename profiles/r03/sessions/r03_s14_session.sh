#!/bin/bash
# Python verify overhead breakdown; PMC traffic of the headline kernel (now
# bitslice_deep_kernel, variant 5), stamped from BUILD_INFO.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
bash tools/gpu_session.sh \
 "pyv:300:python3 -u tools/pyverify_overhead.py" \
 "pmc_traffic:600:python3 tools/pmc_traffic.py --tag r03final --steps 5"
