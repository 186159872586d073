#!/bin/bash
# VALU vs wait cycles (SQ counters, one PMC pass per configuration) of the
# GF(2^16) encode kernels after the round-2 network generator: compiled 20+8
# default (variant 0), 20+8 without shared subexpressions (variant 9), and the
# run-time specialised 12+8.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
C="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_WAVES"
T="python3 tools/tune.py --field 16 --p 8 --shard-mib 4 --rounds 1 --shapes 0:0 --nt-only"
bash tools/gpu_session.sh \
 "pmc16_v0:150:timeout -s KILL 140 rocprofv3 --pmc $C --kernel-include-regex 'bitslice_kernel|rse_jit_encode' --output-format csv -d gpurun_out/pmc16_v0 -o p -- $T --k 20 --stripes 128" \
 "pmc16_v9:150:timeout -s KILL 140 rocprofv3 --pmc $C --kernel-include-regex 'bitslice_kernel|rse_jit_encode' --output-format csv -d gpurun_out/pmc16_v9 -o p -- $T --k 20 --stripes 128 --variants 10" \
 "pmc16_12:150:timeout -s KILL 140 rocprofv3 --pmc $C --kernel-include-regex 'bitslice_kernel|rse_jit_encode' --output-format csv -d gpurun_out/pmc16_12 -o p -- $T --k 12 --stripes 128"
