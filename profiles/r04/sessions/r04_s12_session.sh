#!/bin/bash
# Round 4, session 12: the whole GPU suite at the round's code (1 / 2 KiB
# kernels in both wide bodies), then the reference bench matrix.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
export RSE_JIT_CACHE_DIR=$PWD/jitcache
bash tools/gpu_session.sh \
 "first:400:python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py -m gpu -k 'sub_chunk or wide_launch'" || exit $?
grep -q " passed" gpurun_out/first.log && ! grep -q -E "[0-9]+ failed" gpurun_out/first.log || exit 1
bash tools/gpu_session.sh \
 "suite:900:python3 -u -m pytest -q --timeout 300 --timeout-method thread tests -m gpu" \
 "matrix:400:python3 -u tools/ref_matrix.py --no-crossover"
