#!/bin/bash
# Round 5, session 3: the dispatcher tests (poll fix); launch-grid and
# temporaries A/Bs of the half-chunk wide modules (64+64, 32+32 x 1 KiB);
# PMC of GF(2^16) proper (1000+24 block modules); the whole GPU suite.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}" || exit 1
export TMPDIR=/tmp
TU="python3 tools/tune.py --rounds 20 --nt-only"
W64="--k 64 --p 64 --shard-kib 1 --stripes 2048"
W32="--k 32 --p 32 --shard-kib 1 --stripes 4096"
G16="--field 16 --k 1000 --p 24 --shard-kib 64 --stripes 32"
C1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_WAVES GRBM_GUI_ACTIVE"
P="rocprofv3 --kernel-include-regex rse_jit --output-format csv"
PT="python3 tools/tune.py --rounds 2 --shapes 0:0 --nt-only"
bash tools/gpu_session.sh \
 "dispatch:600:python3 -u -m pytest tests/test_gpu_dispatch.py -x -q --timeout 120 --timeout-method thread" \
 "grid64:300:$TU $W64 --shapes 0:0,256:0,512:0,2048:0" \
 "grid32:300:$TU $W32 --shapes 0:0,256:0,512:0,2048:0" \
 "cse64:300:$TU $W64 --shapes 0:0,256:0 --set 13=16" \
 "cse32:300:$TU $W32 --shapes 0:0,256:0 --set 13=16" \
 "g16:300:$TU $G16 --shapes 0:0" \
 "pmcg16_1:120:timeout -s KILL 110 $P --pmc $C1 -d gpurun_out/pmcg16_1 -o p -- $PT $G16" \
 "pmcg16_f:120:timeout -s KILL 110 $P --pmc FETCH_SIZE -d gpurun_out/pmcg16_f -o p -- $PT $G16" \
 "pmcg16_w:120:timeout -s KILL 110 $P --pmc WRITE_SIZE -d gpurun_out/pmcg16_w -o p -- $PT $G16" \
 "traceg16:120:timeout -s KILL 110 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/traceg16 -o t -- $PT $G16" \
 "suite:1000:python3 -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread --durations=20"
