#!/bin/bash
# Round 5, session 24: the compiled codecs' 1 / 2 KiB kernels with 4 inputs in
# flight (bitslice_sub_deep_kernel, RSE_OPT_SUB_DEPTH > 1) -- the sub-chunk
# parity tests, smoke, and 10+4 / 10+2 x 1 KiB against depth 1.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}" || exit 1
export TMPDIR=/tmp
PY="python -u -m pytest -x -q --timeout 300 --timeout-method thread"
TU="python3 tools/tune.py --rounds 9 --nt-only --shapes 0:0"
E104="--k 10 --p 4 --shard-kib 1 --stripes 16384"
bash tools/gpu_session.sh \
 "tests:600:$PY tests/test_gpu_parity.py -k 'sub_chunk'" \
 "smoke:120:python3 -c 'import __graft_entry__ as g; g.smoke()'" \
 "c104:300:for i in 1 2; do $TU $E104 && $TU $E104 --set 50=1 || exit 1; done"
