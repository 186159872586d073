#!/bin/bash
# Round 5, session 6: GF(2^16) 1000+24 on the chain of wide modules over input
# blocks (RSE_OPT_WIDE_BLOCK_INPUTS 128) against the 8 x 32 block modules
# (46=0), with PMC traffic and a kernel trace of the chain; 64+64 / 32+32 x
# 1 KiB at 4 waves per SIMD (RSE_OPT_WIDE_OCCUPANCY 4: <= 128 VGPRs, two
# 8-wave workgroups per CU) with fewer temporaries (RSE_OPT_JIT_CSE 16 / 8).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}" || exit 1
export TMPDIR=/tmp
PY="python -u -m pytest -x -v --timeout 300 --timeout-method thread"
TU="python3 tools/tune.py --rounds 9 --nt-only --shapes 0:0"
G16="--field 16 --k 1000 --p 24 --shard-kib 64 --stripes 128"
W64="--k 64 --p 64 --shard-kib 1 --stripes 2048"
W32="--k 32 --p 32 --shard-kib 1 --stripes 4096"
C1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_WAVES GRBM_GUI_ACTIVE"
P="rocprofv3 --kernel-include-regex rse_jit --output-format csv"
PT="python3 tools/tune.py --rounds 2 --shapes 0:0 --nt-only"
[ "$1" = occ ] || bash tools/gpu_session.sh \
 "chain:600:$PY tests/test_gpu_parity.py -k 'wide_block_chain or wide_codec_kernels' && $PY tests/test_gpu_host_paths.py -k beyond_256" \
 "g1000:400:for i in 1 2; do $TU $G16 && $TU $G16 --set 46=0 || exit 1; done" \
 "pmcc_1:120:timeout -s KILL 110 $P --pmc $C1 -d gpurun_out/pmcc_1 -o p -- $PT $G16" \
 "pmcc_f:120:timeout -s KILL 110 $P --pmc FETCH_SIZE -d gpurun_out/pmcc_f -o p -- $PT $G16" \
 "pmcc_w:120:timeout -s KILL 110 $P --pmc WRITE_SIZE -d gpurun_out/pmcc_w -o p -- $PT $G16" \
 "tracec:120:timeout -s KILL 110 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/tracec -o t -- $PT $G16"


# (second call) 64+64 / 32+32 x 1 KiB: RSE_OPT_WIDE_OCCUPANCY 4 (<= 128 VGPRs; the
# modules spill 98-761 VGPRs) and the tune build's barrier-free modules (47=1,
# WRONG bytes: what the per-round barriers cost)
if [ "$1" = occ ]; then
TL="env RSE_LIB_PATH=reed-solomon-erasure_amd/build-tune/librse_hip.so $TU"
bash tools/gpu_session.sh \
 "o64:400:for i in 1 2; do $TU $W64 && $TU $W64 --set 20=4 && $TU $W64 --set 20=4 --set 13=16 && $TL $W64 --set 47=1 || exit 1; done" \
 "o32:400:for i in 1 2; do $TU $W32 && $TU $W32 --set 20=4 --set 13=8 && $TL $W32 --set 47=1 || exit 1; done"
fi
if [ "$1" = nosync ]; then
TL="env RSE_LIB_PATH=reed-solomon-erasure_amd/build-tune/librse_hip.so $TU"
bash tools/gpu_session.sh \
 "n64:400:for i in 1 2; do $TU $W64 && $TL $W64 --set 47=1 || exit 1; done" \
 "n32:400:for i in 1 2; do $TU $W32 && $TL $W32 --set 47=1 || exit 1; done"
fi
