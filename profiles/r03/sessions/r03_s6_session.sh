#!/bin/bash
# Per-call latency with the balanced grid of short launches (default) and
# explicit workgroup counts; the GPU suite's bit-sliced tests; the bench.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
CAPI="hipcc --offload-arch=gfx950 -O2 -I include tools/capi_latency.cpp -L reed-solomon-erasure_amd/reed_solomon_erasure -lrse_hip -Wl,-rpath,$PWD/reed-solomon-erasure_amd/reed_solomon_erasure -o /tmp/capi_latency"
bash tools/gpu_session.sh \
 "capi_build:180:$CAPI" \
 "capi_auto:120:/tmp/capi_latency 0" \
 "capi256:120:/tmp/capi_latency 256" \
 "capi384:120:/tmp/capi_latency 384" \
 "capi512:120:/tmp/capi_latency 512" \
 "capi640:120:/tmp/capi_latency 640" \
 "capi768:120:/tmp/capi_latency 768" \
 "capi1024:120:/tmp/capi_latency 1024" \
 "capi_auto2:120:/tmp/capi_latency 0" \
 "pytest:900:python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread" \
 "bench:600:python3 -u bench.py"
for f in gpurun_out/capi*.log; do echo "$f $(grep -h -E 'verify \(sync|encode \(async' $f | tr '\n' ' ')"; done
