#!/bin/bash
# Round 6, session 4: FFT kernels with one direction (the parity block is its
# own inverse), the dispatcher's fresh-input test at 64 KiB x 8 workgroups,
# and the host pipeline's streams against hardware-queue sharing.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}" || exit 1
export TMPDIR=/tmp
T="python -u -m pytest -x -q -m gpu --timeout 120 --timeout-method thread"
bash tools/gpu_session.sh \
 "fft_tests:300:$T tests/test_gpu_fft.py" \
 "dispatch_tests:300:$T tests/test_gpu_dispatch.py" \
 "queue_probe:300:python3 -u tools/queue_probe.py"
