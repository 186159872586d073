#!/bin/bash
# Round 5, session 16: counters of the 64+64 x 1 KiB module as it now runs by
# default (4 outputs per wave, 16 waves, launches of resident workgroups):
# VALU issue and waits, and HBM traffic (FETCH_SIZE, WRITE_SIZE passes).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}" || exit 1
export TMPDIR=/tmp
W64="--k 64 --p 64 --shard-kib 1 --stripes 2048"
C1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_WAVES GRBM_GUI_ACTIVE"
P="rocprofv3 --kernel-include-regex rse_jit --output-format csv"
PT="python3 tools/tune.py --rounds 2 --shapes 0:0 --nt-only"
bash tools/gpu_session.sh \
 "pmc64_1:120:timeout -s KILL 110 $P --pmc $C1 -d gpurun_out/pmc64_1 -o p -- $PT $W64" \
 "pmc64_f:120:timeout -s KILL 110 $P --pmc FETCH_SIZE -d gpurun_out/pmc64_f -o p -- $PT $W64" \
 "pmc64_w:120:timeout -s KILL 110 $P --pmc WRITE_SIZE -d gpurun_out/pmc64_w -o p -- $PT $W64" \
 "trace64:120:timeout -s KILL 110 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/trace64 -o t -- $PT $W64"
