#!/bin/bash
# Store cache policy: write-through sc1 (variant 8, nt=0: sc1, nt=1: sc1 nt) vs nt (1).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
bash tools/gpu_session.sh \
 "pytest_v:600:python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread -k bitslice_kernel_variants" \
 "t10_4:300:python -u tools/tune.py --k 10 --p 4 --stripes 448 --rounds 4 --variants 9 --shapes 4096:1 " \
 "t20_8:300:python -u tools/tune.py --field 16 --k 20 --p 8 --shard-mib 4 --stripes 256 --rounds 3 --variants 9 --shapes 8192:1"
