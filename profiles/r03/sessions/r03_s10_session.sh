#!/bin/bash
# reconstruct_batch after the pinned flag upload and the norm inverse: batch
# parity tests, the 4 KiB x 65536 rates and kernel trace.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
T16="python3 -u tools/tune.py --rounds 5 --nt-only --field 16 --k 20 --p 8 --shapes 0:0"
bash tools/gpu_session.sh \
 "pytest_batch:600:python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_host_paths.py -m gpu -k 'batch'" || exit $?
grep -q " passed" gpurun_out/pytest_batch.log && ! grep -q -E "[0-9]+ failed" gpurun_out/pytest_batch.log || exit 1
bash tools/gpu_session.sh \
 "b4k_e4:300:$T16 --shard-kib 4 --stripes 65536 --op batch --erase 0,1,2,3" \
 "b4k_e8:300:$T16 --shard-kib 4 --stripes 65536 --op batch --erase 0,1,2,3,4,5,6,7" \
 "b4m_e4:300:$T16 --shard-mib 4 --stripes 256 --op batch --erase 0,1,2,3" \
 "trace_b4k:300:rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/trace_b4k -o b -- python3 tools/tune.py --rounds 2 --nt-only --shapes 0:0 --field 16 --k 20 --p 8 --shard-kib 4 --stripes 65536 --op batch --erase 0,1,2,3"
grep -h median gpurun_out/b4*.log
