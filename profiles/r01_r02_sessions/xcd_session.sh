#!/bin/bash
# XCD-aware chunk order (variant 7) vs the default (1).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
bash tools/gpu_session.sh \
 "pytest_v:600:python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread -k bitslice_kernel_variants" \
 "t10_4:300:python -u tools/tune.py --k 10 --p 4 --stripes 448 --rounds 3 --variants 8 --shapes 4096:1,8192:1 --nt-only" \
 "t20_8:300:python -u tools/tune.py --field 16 --k 20 --p 8 --shard-mib 4 --stripes 256 --rounds 3 --variants 8 --shapes 4096:1,8192:1 --nt-only"
