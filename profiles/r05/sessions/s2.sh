#!/bin/bash
# Round 5, session 2: the latency floor of a synchronous small call; GF(2^8)
# wide codecs on half chunks (RSE_OPT_WIDE_HALF): their tests, a same-box A/B
# against full chunks (alternating processes: the option shapes the module),
# PMC passes of the reference's widest bench shape; then the bench.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}" || exit 1
export TMPDIR=/tmp
TU="python3 tools/tune.py --rounds 20 --shapes 0:0 --nt-only"
W64="--k 64 --p 64 --shard-kib 1 --stripes 2048"
W32="--k 32 --p 32 --shard-kib 1 --stripes 4096"
W50="--k 50 --p 20 --shard-kib 1 --stripes 3744"
W50M="--k 50 --p 20 --shard-mib 1 --stripes 128"
C1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_WAVES GRBM_GUI_ACTIVE"
C2="SQ_IFETCH SQ_INSTS_SALU SQ_INSTS_LDS SQ_ACTIVE_INST_LDS SQ_INSTS_BRANCH SQ_WAIT_INST_LDS SQ_WAVE_CYCLES SQ_WAVES"
P="rocprofv3 --kernel-include-regex rse_jit_wide --output-format csv"
PT="python3 tools/tune.py --rounds 2 --shapes 0:0 --nt-only"
bash tools/gpu_session.sh \
 "latency:120:./tools/bin/latency_probe" \
 "dispatch:600:python3 -u -m pytest tests/test_gpu_dispatch.py -x -q --timeout 120 --timeout-method thread" \
 "tests:900:python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k 'wide or sub_chunk'" \
 "ab64:400:for i in 1 2; do $TU $W64 --set 38=0 && $TU $W64 || exit 1; done" \
 "ab32:400:for i in 1 2; do $TU $W32 --set 38=0 && $TU $W32 || exit 1; done" \
 "ab50:400:for i in 1 2; do $TU $W50 --set 38=0 && $TU $W50 || exit 1; done" \
 "ab50m:400:for i in 1 2; do $TU $W50M --set 38=0 && $TU $W50M || exit 1; done" \
 "pmc64h_1:90:timeout -s KILL 80 $P --pmc $C1 -d gpurun_out/pmc64h_1 -o p -- $PT $W64" \
 "pmc64h_2:90:timeout -s KILL 80 $P --pmc $C2 -d gpurun_out/pmc64h_2 -o p -- $PT $W64" \
 "pmc64h_f:90:timeout -s KILL 80 $P --pmc FETCH_SIZE -d gpurun_out/pmc64h_f -o p -- $PT $W64" \
 "pmc64h_w:90:timeout -s KILL 80 $P --pmc WRITE_SIZE -d gpurun_out/pmc64h_w -o p -- $PT $W64" \
 "pmc64f_1:90:timeout -s KILL 80 $P --pmc $C1 -d gpurun_out/pmc64f_1 -o p -- $PT $W64 --set 38=0" \
 "pmc64f_f:90:timeout -s KILL 80 $P --pmc FETCH_SIZE -d gpurun_out/pmc64f_f -o p -- $PT $W64 --set 38=0" \
 "pmc64f_w:90:timeout -s KILL 80 $P --pmc WRITE_SIZE -d gpurun_out/pmc64f_w -o p -- $PT $W64 --set 38=0" \
 "pmc32h_1:90:timeout -s KILL 80 $P --pmc $C1 -d gpurun_out/pmc32h_1 -o p -- $PT $W32" \
 "bench:600:python3 -u bench.py"
