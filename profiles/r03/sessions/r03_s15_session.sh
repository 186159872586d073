#!/bin/bash
# Completion word (RSE_OPT_SPIN_WAIT): parity tests of verify, then per-call
# verify latency through the C ABI with it on / off (alternating processes)
# and the Python per-call breakdown.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
CAPI="hipcc --offload-arch=gfx950 -O2 -I include tools/capi_latency.cpp -L reed-solomon-erasure_amd/reed_solomon_erasure -lrse_hip -Wl,-rpath,$PWD/reed-solomon-erasure_amd/reed_solomon_erasure -o /tmp/capi_latency"
bash tools/gpu_session.sh \
 "tverify:300:python3 -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k 'verify or smoke' --timeout 120 --timeout-method thread" \
 "capi_build:180:$CAPI" \
 "spin1a:120:/tmp/capi_latency 0 0 1" \
 "spin0a:120:/tmp/capi_latency 0 0 0" \
 "spin1b:120:/tmp/capi_latency 0 0 1" \
 "spin0b:120:/tmp/capi_latency 0 0 0" \
 "pyv:300:python3 -u tools/pyverify_overhead.py"
