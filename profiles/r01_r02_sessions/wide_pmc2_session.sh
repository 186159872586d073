#!/bin/bash
# Where a wide codec's wave cycles go (GF(2^8) 50+20 x 1 MiB, 64 stripes, the
# one-module kernel): VALU, LDS, waits, LDS bank conflicts; one SQ pass.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
C="SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_WAIT_ANY SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU SQ_WAVES"
T="python3 tools/tune.py --rounds 1 --nt-only --shapes 0:0 --bitslice 1 --k 50 --p 20 --shard-mib 1 --stripes 64"
bash tools/gpu_session.sh \
 "pmcw:200:timeout -s KILL 190 rocprofv3 --pmc $C --kernel-include-regex rse_jit_wide --output-format csv -d gpurun_out/pmc_w50 -o p -- $T"
