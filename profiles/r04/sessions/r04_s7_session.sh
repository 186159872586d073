#!/bin/bash
# Round 4, session 7: 1 / 2 KiB shards on the bit-sliced kernels (SUB chunks),
# GF(2^16) codecs of <= 256 shards in the GF(2^8) subfield, the batch planner
# and device flags; then the whole GPU suite, the bench and the reference
# bench matrix with prebuilt run-time modules.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
export RSE_JIT_CACHE_DIR=$PWD/jitcache
bash tools/gpu_session.sh \
 "first:400:python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py -m gpu -k 'sub_chunk or wave_pairs or bitslice_reconstruct_every'" || exit $?
grep -q " passed" gpurun_out/first.log && ! grep -q -E "[0-9]+ failed" gpurun_out/first.log || exit 1
bash tools/gpu_session.sh \
 "suite:900:python3 -u -m pytest -q --timeout 300 --timeout-method thread tests -m gpu" \
 "bench:400:python3 -u bench.py" \
 "matrix:400:python3 -u tools/ref_matrix.py --no-crossover" \
 "probe_e4d:200:python3 -u tools/batch_probe.py --erasures 4 --calls 20 --device-flags" \
 "probe_e8d:200:python3 -u tools/batch_probe.py --erasures 8 --calls 20 --device-flags"
