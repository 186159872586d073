#!/bin/bash
# A/B of the bit-sliced encode variants, incl. 2/3 inputs in flight (5, 6).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
bash tools/gpu_session.sh \
 "pytest_bs:600:python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread -k 'bitslice_kernel_variants or decode_pattern'" \
 "tune_10_4:300:python -u tools/tune.py --k 10 --p 4 --stripes 128 --rounds 3 --variants 7 --shapes 4096:1,8192:1 --nt-only" \
 "tune_10_2:300:python -u tools/tune.py --k 10 --p 2 --stripes 128 --rounds 3 --variants 7 --shapes 4096:1,8192:1 --nt-only" \
 "tune_20_8:300:python -u tools/tune.py --field 16 --k 20 --p 8 --shard-mib 4 --stripes 256 --rounds 3 --variants 7 --shapes 4096:1,8192:1 --nt-only"
