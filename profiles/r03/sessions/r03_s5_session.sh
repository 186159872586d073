#!/bin/bash
# Pair kernels with the next unit's first input prefetched during the mixing
# (RSE_OPT_RECON_PAIRS 3) against the default (1); per-call verify over the
# workgroup count; reconstruct_batch at round 2's 256 stripes.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
T16="python3 -u tools/tune.py --rounds 5 --nt-only --field 16 --k 20 --p 8 --shapes 0:0"
B="python -u tools/tune.py --op batch --rounds 5 --nt-only --bitslice 1 --shapes 0:0"
CAPI="hipcc --offload-arch=gfx950 -O2 -I include tools/capi_latency.cpp -L reed-solomon-erasure_amd/reed_solomon_erasure -lrse_hip -Wl,-rpath,$PWD/reed-solomon-erasure_amd/reed_solomon_erasure -o /tmp/capi_latency"
bash tools/gpu_session.sh \
 "pytest_pairs:300:python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py -m gpu -k wave_pairs" || exit $?
grep -q " passed" gpurun_out/pytest_pairs.log && ! grep -q -E "[0-9]+ failed" gpurun_out/pytest_pairs.log || exit 1
bash tools/gpu_session.sh \
 "r8_pf:300:$T16 --shard-mib 4 --stripes 128 --op reconstruct --patterns 0 --erase 0,1,2,3,4,5,6,7 --recon-mix 3 --ab 28=1,3" \
 "b8_pf:300:$T16 --shard-mib 4 --stripes 128 --op batch --erase 0,1,2,3,4,5,6,7 --ab 28=1,3" \
 "b16_e4:200:$B --field 16 --k 20 --p 8 --shard-mib 4 --stripes 256 --erase 0,1,2,3" \
 "b16_e8:200:$B --field 16 --k 20 --p 8 --shard-mib 4 --stripes 256 --erase 0,1,2,3,4,5,6,7" \
 "capi_build:180:$CAPI" \
 "capi0:120:/tmp/capi_latency 0" \
 "capi512:120:/tmp/capi_latency 512" \
 "capi768:120:/tmp/capi_latency 768" \
 "capi2048:120:/tmp/capi_latency 2048"
