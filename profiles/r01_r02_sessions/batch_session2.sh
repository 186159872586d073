#!/bin/bash
# reconstruct_batch with contiguous chunk runs per workgroup: parity tests of
# the batch paths, then per-stripe random patterns (GF(2^16) 4 and 8 erasures,
# GF(2^8) 4).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
B="python -u tools/tune.py --op batch --rounds 5 --nt-only --bitslice 1 --shapes 0:0"
bash tools/gpu_session.sh \
 "pytest:600:python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_host_paths.py -x -q --timeout 300 --timeout-method thread -k batch" \
 "b16_e4:200:$B --field 16 --k 20 --p 8 --shard-mib 4 --stripes 256 --erase 0,1,2,3" \
 "b16_e8:200:$B --field 16 --k 20 --p 8 --shard-mib 4 --stripes 256 --erase 0,1,2,3,4,5,6,7" \
 "b8_e4:200:$B --k 10 --p 4 --stripes 128 --erase 0,1,2,3"
