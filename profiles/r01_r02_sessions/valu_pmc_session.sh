#!/bin/bash
# VALU vs wait cycles of the bit-sliced encode kernels (GF(2^8) 10+4, GF(2^16)
# 20+8), one PMC pass each (SQ block only, 8 counters).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
C="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_WAVES"
bash tools/gpu_session.sh \
 "list:60:rocprofv3 -L > gpurun_out/counters.txt 2>&1; grep -c SQ_ gpurun_out/counters.txt" \
 "pmc8:120:timeout -s KILL 110 rocprofv3 --pmc $C --kernel-include-regex bitslice_kernel --output-format csv -d gpurun_out/pmc_valu8 -o p -- python3 tools/tune.py --k 10 --p 4 --stripes 64 --rounds 1 --shapes 4096:1 --nt-only" \
 "pmc16:120:timeout -s KILL 110 rocprofv3 --pmc $C --kernel-include-regex bitslice_kernel --output-format csv -d gpurun_out/pmc_valu16 -o p -- python3 tools/tune.py --field 16 --k 20 --p 8 --shard-mib 4 --stripes 128 --rounds 1 --shapes 8192:1 --nt-only"
