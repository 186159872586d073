#!/bin/bash
# Round 6, session 3: first GPU run of the additive-FFT kernels (k = p = 16 / 32
# / 64) and of the dispatcher with one agent acquire per request; FFT kernel
# rates on the reference bench's 1 KiB shapes; the pinned-host e2e probe.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}" || exit 1
export TMPDIR=/tmp
T="python -u -m pytest -x -q -m gpu --timeout 120 --timeout-method thread"
bash tools/gpu_session.sh \
 "fft_tests:300:$T tests/test_gpu_fft.py" \
 "dispatch_tests:300:$T tests/test_gpu_dispatch.py" \
 "fft64_enc:120:python3 -u tools/tune.py --k 64 --p 64 --shard-kib 1 --stripes 2048 --nt-only --shapes 0:0,512:0,1024:0,2048:0 --rounds 5" \
 "fft32_enc:120:python3 -u tools/tune.py --k 32 --p 32 --shard-kib 1 --stripes 4096 --nt-only --shapes 0:0,512:0,1024:0,2048:0 --rounds 5" \
 "fft16_enc:120:python3 -u tools/tune.py --k 16 --p 16 --shard-kib 1 --stripes 8192 --nt-only --shapes 0:0,512:0,1024:0,2048:0 --rounds 5" \
 "fft64_all:120:python3 -u tools/tune.py --op reconstruct --k 64 --p 64 --shard-kib 1 --stripes 2048 --nt-only --shapes 0:0,1024:0 --erase $(seq -s, 0 63) --rounds 5" \
 "e2e_probe:400:python3 -u tools/e2e_probe.py"
