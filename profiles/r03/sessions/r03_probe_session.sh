#!/bin/bash
# Round-3 probes: wave-pair reconstruct parity and A/B, GF(2^16) 20+8
# 8-erasure reconstruct over mixing mode / inputs in flight, reconstruct_batch
# at 4 KiB x 65536 (kernel trace), per-kernel clocks, C-ABI verify latency.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
T16="python3 -u tools/tune.py --rounds 3 --nt-only --field 16 --k 20 --p 8 --shard-mib 4 --stripes 128 --patterns 0"
bash tools/gpu_session.sh \
 "pytest_pairs:600:python3 -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_parity.py -m gpu -k 'wave_pairs or every_mixing or batch or full_size'" || exit $?
grep -q " passed" gpurun_out/pytest_pairs.log && ! grep -q -E "[0-9]+ failed" gpurun_out/pytest_pairs.log || exit 1
bash tools/gpu_session.sh \
 "r8_pairs:300:$T16 --op reconstruct --erase 0,1,2,3,4,5,6,7 --shapes 0:0 --recon-mix 3 --ab 28=0,1" \
 "b8_pairs:300:$T16 --op batch --erase 0,1,2,3,4,5,6,7 --shapes 0:0 --recon-mix 3 --ab 28=0,1" \
 "r8_depth:300:$T16 --op reconstruct --erase 0,1,2,3,4,5,6,7 --shapes 0:0 --recon-mix 2 --recon-depth 1,2,3 --ab 28=0" \
 "r8_grid:300:$T16 --op reconstruct --erase 0,1,2,3,4,5,6,7 --shapes 4096:0,8192:0,16384:0,32768:0 --recon-mix 3 --ab 28=1" \
 "r4:300:$T16 --op reconstruct --erase 0,1,2,3 --shapes 0:0 --recon-mix 3" \
 "batch_trace:300:rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/batch_trace -o b -- python3 tools/tune.py --rounds 2 --nt-only --shapes 0:0 --field 16 --k 20 --p 8 --shard-kib 4 --stripes 65536 --op batch --erase 0,1,2,3" \
 "capi:180:hipcc --offload-arch=gfx950 -O2 -I include tools/capi_latency.cpp -L reed-solomon-erasure_amd/reed_solomon_erasure -lrse_hip -Wl,-rpath,$PWD/reed-solomon-erasure_amd/reed_solomon_erasure -o /tmp/capi_latency && /tmp/capi_latency" \
 "clock:900:bash tools/clock_session.sh"
