#!/bin/bash
# Round-4 final evidence at HEAD: smoke, GPU suite, bench, rocprofv3 kernel
# trace of the headline bench, PMC traffic of the headline kernel (stamped from
# BUILD_INFO).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
export RSE_JIT_CACHE_DIR=$PWD/jitcache
bash tools/gpu_session.sh \
 "smoke:300:python3 -c 'import __graft_entry__ as g; g.smoke()'" \
 "pytest:900:python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread" \
 "bench:600:python3 -u bench.py" \
 "trace:400:rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/trace -o bench -- python3 bench.py --no-cpu --no-extras --steps 10" \
 "pmc_traffic:600:python3 tools/pmc_traffic.py --tag r04final2 --steps 5"
