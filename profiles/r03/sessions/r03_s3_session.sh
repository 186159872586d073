#!/bin/bash
# Device validation of reconstruct_batch and the pair kernels' default grid:
# parity, batch rates (4 KiB x 65536 and 4 MiB x 128, 4 and 8 erasures), the
# 8-erasure reconstruct, its kernel trace and SQ counter passes (pairs vs one
# wave per column).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
T16="python3 -u tools/tune.py --rounds 3 --nt-only --field 16 --k 20 --p 8 --shapes 0:0"
R8="python3 tools/tune.py --rounds 1 --nt-only --shapes 0:0 --field 16 --k 20 --p 8 --shard-mib 4 --stripes 128 --op reconstruct --erase 0,1,2,3,4,5,6,7 --patterns 0 --recon-mix 3"
bash tools/gpu_session.sh "dbg:120:python3 -u tools/dbg_runs.py"
bash tools/gpu_session.sh \
 "pytest_batch:600:python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_host_paths.py -m gpu -k 'batch or wave_pairs or every_mixing'" || exit $?
grep -q " passed" gpurun_out/pytest_batch.log && ! grep -q -E "[0-9]+ failed" gpurun_out/pytest_batch.log || exit 1
bash tools/gpu_session.sh \
 "b4k_e4:300:$T16 --shard-kib 4 --stripes 65536 --op batch --erase 0,1,2,3" \
 "b4k_e8:300:$T16 --shard-kib 4 --stripes 65536 --op batch --erase 0,1,2,3,4,5,6,7" \
 "b4m_e4:300:$T16 --shard-mib 4 --stripes 128 --op batch --erase 0,1,2,3" \
 "b4m_e8:300:$T16 --shard-mib 4 --stripes 128 --op batch --erase 0,1,2,3,4,5,6,7 --ab 28=0,1,2" \
 "r8:300:$T16 --shard-mib 4 --stripes 128 --op reconstruct --patterns 0 --erase 0,1,2,3,4,5,6,7 --recon-mix 3 --ab 28=0,1,2" \
 "trace_r8:300:rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/trace_r8 -o r -- $R8" \
 "trace_b4k:300:rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/trace_b4k -o b -- python3 tools/tune.py --rounds 2 --nt-only --shapes 0:0 --field 16 --k 20 --p 8 --shard-kib 4 --stripes 65536 --op batch --erase 0,1,2,3" \
 "pmc_pairs:500:bash tools/pmc_kernel_session.sh pairs8 bitslice_recon_pair_kernel $R8" \
 "pmc_pairs1:500:bash tools/pmc_kernel_session.sh pairs8p1 bitslice_recon_pair_kernel $R8 --set 28=2" \
 "pmc_onewave:500:bash tools/pmc_kernel_session.sh onewave8 bitslice_recon_kernel $R8 --set 28=0"
