#!/bin/bash
# Round 5, session 5: 4 outputs per wave (RSE_OPT_WIDE_SPLIT 4: 64+64 in 16
# waves, 32+32 and 50+20 in 8, ~115 VGPRs -> 4 waves per SIMD) against the
# default 8 (~170 VGPRs, 2 waves per SIMD), alternating processes, each with
# the launch-grid A/B; GF(2^16) proper PMC (its files were lost in session 3).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}" || exit 1
export TMPDIR=/tmp
TU="python3 tools/tune.py --rounds 15 --nt-only --shapes 0:0 --ab 44=0,1,2"
W64="--k 64 --p 64 --shard-kib 1 --stripes 2048"
W32="--k 32 --p 32 --shard-kib 1 --stripes 4096"
W50="--k 50 --p 20 --shard-kib 1 --stripes 3744"
W50M="--k 50 --p 20 --shard-mib 1 --stripes 128"
G16="--field 16 --k 1000 --p 24 --shard-kib 64 --stripes 128"
C1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_WAVES GRBM_GUI_ACTIVE"
P="rocprofv3 --kernel-include-regex rse_jit --output-format csv"
PT="python3 tools/tune.py --rounds 2 --shapes 0:0 --nt-only"
bash tools/gpu_session.sh \
 "s64:300:for i in 1 2; do $TU $W64 --set 18=4 && $TU $W64 || exit 1; done" \
 "s32:300:for i in 1 2; do $TU $W32 --set 18=4 && $TU $W32 || exit 1; done" \
 "s50:300:for i in 1 2; do $TU $W50 --set 18=4 && $TU $W50 || exit 1; done" \
 "s50m:300:for i in 1 2; do $TU $W50M --set 18=4 && $TU $W50M || exit 1; done" \
 "pmc64s_1:120:timeout -s KILL 110 $P --pmc $C1 -d gpurun_out/pmc64s_1 -o p -- $PT $W64 --set 18=4" \
 "pmcg16_1:120:timeout -s KILL 110 $P --pmc $C1 -d gpurun_out/pmcg16_1 -o p -- $PT $G16" \
 "pmcg16_f:120:timeout -s KILL 110 $P --pmc FETCH_SIZE -d gpurun_out/pmcg16_f -o p -- $PT $G16" \
 "pmcg16_w:120:timeout -s KILL 110 $P --pmc WRITE_SIZE -d gpurun_out/pmcg16_w -o p -- $PT $G16" \
 "traceg16:120:timeout -s KILL 110 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/traceg16 -o t -- $PT $G16"
