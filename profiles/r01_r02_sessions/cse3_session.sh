#!/bin/bash
# Same-process A/B: compiled GF(2^16) 20+8 networks with shared subexpressions
# (variants 0, 1) vs without (9).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
bash tools/gpu_session.sh \
 "pytest_v:600:python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread -k bitslice_kernel_variants" \
 "t20_8:300:python -u tools/tune.py --field 16 --k 20 --p 8 --shard-mib 4 --stripes 256 --rounds 5 --variants 10 --shapes 4096:1,8192:1 --nt-only"
