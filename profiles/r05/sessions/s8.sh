#!/bin/bash
# Round 5, session 8: wide modules with the next LDS slot's reads issued
# before the current slot's network (RSE_OPT_WIDE_LDS_PIPE 1, the default)
# against without (48=0): parity of the wide tests, 64+64 / 32+32 / 50+20 x
# 1 KiB and 50+20 x 1 MiB A/Bs, the GF(2^16) 1000+24 chain; instruction-cache
# and LDS counters of 64+64 against 16+16 x 1 KiB.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}" || exit 1
export TMPDIR=/tmp
PY="python -u -m pytest -x -v --timeout 300 --timeout-method thread"
TU="python3 tools/tune.py --rounds 9 --nt-only --shapes 0:0"
G16="--field 16 --k 1000 --p 24 --shard-kib 64 --stripes 128"
W64="--k 64 --p 64 --shard-kib 1 --stripes 2048"
W32="--k 32 --p 32 --shard-kib 1 --stripes 4096"
W16="--k 16 --p 16 --shard-kib 1 --stripes 8192"
W50="--k 50 --p 20 --shard-kib 1 --stripes 3744"
W50M="--k 50 --p 20 --shard-mib 1 --stripes 128"
CI="SQC_ICACHE_REQ SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQ_IFETCH SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_INSTS_VALU GRBM_GUI_ACTIVE"
CL="SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_WAIT_ANY SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VALU GRBM_GUI_ACTIVE"
P="rocprofv3 --kernel-include-regex rse_jit --output-format csv"
PT="python3 tools/tune.py --rounds 2 --shapes 0:0 --nt-only"
if [ "$1" = a ]; then
bash tools/gpu_session.sh \
 "tests:600:$PY tests/test_gpu_parity.py -k 'wide_codec or wide_sixteen or wide_full or sub_chunk'" \
 "q64:300:$TU $W64 && $TU $W32 && $TU $W50" \
 "ic64:120:timeout -s KILL 110 $P --pmc $CI -d gpurun_out/ic64 -o p -- $PT $W64" \
 "ic16:120:timeout -s KILL 110 $P --pmc $CI -d gpurun_out/ic16 -o p -- $PT $W16" \
 "lds64:120:timeout -s KILL 110 $P --pmc $CL -d gpurun_out/lds64 -o p -- $PT $W64"
exit
fi
bash tools/gpu_session.sh \
 "p64:300:for i in 1 2; do $TU $W64 && $TU $W64 --set 48=0 || exit 1; done" \
 "p32:300:for i in 1 2; do $TU $W32 && $TU $W32 --set 48=0 || exit 1; done" \
 "p50:300:for i in 1 2; do $TU $W50 && $TU $W50 --set 48=0 || exit 1; done" \
 "p50m:300:for i in 1 2; do $TU $W50M && $TU $W50M --set 48=0 || exit 1; done" \
 "g16:300:$TU $G16" \
 "smoke:300:python3 -c 'import __graft_entry__ as g; g.smoke()'"
