#!/bin/bash
# Round 5, session 11: the headline kernel's HBM traffic with this library
# (tools/pmc_traffic.py: FETCH_SIZE and WRITE_SIZE passes of the bench), then
# the default bench under a rocprofv3 kernel trace (its summary beside the
# bench line's HIP-event launch time).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}" || exit 1
export TMPDIR=/tmp
bash tools/gpu_session.sh \
 "traffic:400:python3 tools/pmc_traffic.py --tag r05final && cp profiles/r05final_pmc_traffic.json gpurun_out/" \
 "benchprof:600:rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/benchprof -o b -- python3 -u bench.py --full-out gpurun_out/bench_full_n1.json"
