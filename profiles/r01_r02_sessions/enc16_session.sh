#!/bin/bash
# GF(2^16) encode after the network generator change: compiled 20+8 (default
# variant vs variant 9 = no shared subexpressions), run-time 12+8, and the
# GPU tests that cover the bit-sliced kernels and the host paths.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
P="python -u -m pytest -x -q --timeout 600 --timeout-method thread"
bash tools/gpu_session.sh \
 "pytest_bs:900:$P tests/test_gpu_parity.py -k 'bitslice or kernel_variants or specialised or wide'" \
 "pytest_host:600:$P tests/test_gpu_host_paths.py" \
 "e16_20_8:300:python -u tools/tune.py --field 16 --k 20 --p 8 --shard-mib 4 --stripes 256 --rounds 5 --nt-only --shapes 0:0,4096:1 --variants 10" \
 "e16_12_8:300:python -u tools/tune.py --field 16 --k 12 --p 8 --shard-mib 4 --stripes 256 --rounds 5 --nt-only --shapes 0:0" \
 "w16_40_12:400:python -u tools/tune.py --rounds 5 --nt-only --shapes 0:0 --bitslice 1 --field 16 --k 40 --p 12 --shard-mib 1 --stripes 64" \
 "w8_50_20:400:python -u tools/tune.py --rounds 5 --nt-only --shapes 0:0 --bitslice 1 --k 50 --p 20 --shard-mib 1 --stripes 64"
