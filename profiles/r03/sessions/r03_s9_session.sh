#!/bin/bash
# Per-call verify: stream synchronisation vs an event recorded after the
# kernels (RSE_OPT_SYNC_EVENT), alternating.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
CAPI="hipcc --offload-arch=gfx950 -O2 -I include tools/capi_latency.cpp -L reed-solomon-erasure_amd/reed_solomon_erasure -lrse_hip -Wl,-rpath,$PWD/reed-solomon-erasure_amd/reed_solomon_erasure -o /tmp/capi_latency"
bash tools/gpu_session.sh \
 "capi_build:180:$CAPI" \
 "stream1:120:/tmp/capi_latency 0 0" \
 "event1:120:/tmp/capi_latency 0 1" \
 "stream2:120:/tmp/capi_latency 0 0" \
 "event2:120:/tmp/capi_latency 0 1" \
 "stream3:120:/tmp/capi_latency 0 0" \
 "event3:120:/tmp/capi_latency 0 1"
for f in gpurun_out/stream*.log gpurun_out/event*.log; do echo "$f $(grep -h 'verify (sync' $f)"; done
