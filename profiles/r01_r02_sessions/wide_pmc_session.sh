#!/bin/bash
# Where the wide codecs' time goes: SQ counters of the one-module kernels
# (rse_jit_wide) for GF(2^8) 50+20 and GF(2^16) 40+12, with the compiled
# GF(2^16) 20+8 encode kernel as the reference point.  A plain run first fills
# the JIT disk cache, so the profiled processes load modules and spawn no
# compiler.  Two counter passes, each within the per-block limits.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
C1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_WAVES"
C2="SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_SALU SQ_ACTIVE_INST_SCA SQ_INSTS_VMEM_RD SQ_WAVES"
T="python3 tools/tune.py --rounds 1 --shapes 0:0 --nt-only --bitslice 1"
W8="--k 50 --p 20 --shard-mib 1 --stripes 64"
W16="--field 16 --k 40 --p 12 --shard-mib 1 --stripes 64"
E16="--field 16 --k 20 --p 8 --shard-mib 4 --stripes 128"
K="--kernel-include-regex 'rse_jit_wide|bitslice_kernel'"
bash tools/gpu_session.sh \
 "warm:400:$T $W8 && $T $W16" \
 "w8_c1:150:timeout -s KILL 140 rocprofv3 --pmc $C1 $K --output-format csv -d gpurun_out/w8_c1 -o p -- $T $W8" \
 "w8_c2:150:timeout -s KILL 140 rocprofv3 --pmc $C2 $K --output-format csv -d gpurun_out/w8_c2 -o p -- $T $W8" \
 "w16_c1:150:timeout -s KILL 140 rocprofv3 --pmc $C1 $K --output-format csv -d gpurun_out/w16_c1 -o p -- $T $W16" \
 "w16_c2:150:timeout -s KILL 140 rocprofv3 --pmc $C2 $K --output-format csv -d gpurun_out/w16_c2 -o p -- $T $W16" \
 "e16_c1:150:timeout -s KILL 140 rocprofv3 --pmc $C1 $K --output-format csv -d gpurun_out/e16_c1 -o p -- $T $E16" \
 "e16_c2:150:timeout -s KILL 140 rocprofv3 --pmc $C2 $K --output-format csv -d gpurun_out/e16_c2 -o p -- $T $E16"
