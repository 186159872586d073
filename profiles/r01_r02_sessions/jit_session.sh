#!/bin/bash
# GPU session for the run-time specialised (hiprtc) bit-sliced kernels: the
# parity suite, then table vs specialised throughput on codecs that are not
# compiled into the library.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
bash tools/gpu_session.sh \
 "pytest:900:python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread" \
 "tune_gf8_12_4:300:python -u tools/tune.py --k 12 --p 4 --stripes 64 --rounds 3 --bitslice 1,0 --shapes 4096:1 --nt-only" \
 "tune_gf16_10_4:300:python -u tools/tune.py --field 16 --k 10 --p 4 --stripes 64 --rounds 3 --bitslice 1,0 --shapes 4096:1 --nt-only" \
 "tune_gf8_6_3:300:python -u tools/tune.py --k 6 --p 3 --stripes 64 --rounds 3 --bitslice 1,0 --shapes 4096:1 --nt-only" \
 "tune_gf16_12_8_rec:300:python -u tools/tune.py --field 16 --k 12 --p 8 --stripes 32 --rounds 3 --bitslice 1,0 --shapes 8192:1 --nt-only --op reconstruct --erase 0,1,2,3"
