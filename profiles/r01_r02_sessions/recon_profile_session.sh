#!/bin/bash
# Evidence for the Horner-mixing syndrome reconstruct (GF(2^16) 20+8 x 4 MiB,
# 256 stripes, first uses of an erasure pattern): rocprofv3 kernel trace +
# stats, then one VALU PMC pass per erasure count (SQ block, 8 counters), then
# the bench (duplex PCIe leg).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
C="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_WAVES"
T="python3 tools/tune.py --op reconstruct --rounds 2 --nt-only --bitslice 1 --patterns 0 --shapes 0:0 --field 16 --k 20 --p 8 --shard-mib 4 --stripes 256"
R="--kernel-include-regex bitslice_recon_kernel --output-format csv"
bash tools/gpu_session.sh \
 "trace8:200:timeout -s KILL 190 rocprofv3 --kernel-trace --stats $R -d gpurun_out/recon_trace8 -o t -- $T --erase 0,1,2,3,4,5,6,7" \
 "trace4:200:timeout -s KILL 190 rocprofv3 --kernel-trace --stats $R -d gpurun_out/recon_trace4 -o t -- $T --erase 0,1,2,3" \
 "pmc8:200:timeout -s KILL 190 rocprofv3 --pmc $C $R -d gpurun_out/recon_pmc8 -o p -- $T --erase 0,1,2,3,4,5,6,7 --recon-mix 2,1" \
 "pmc4:200:timeout -s KILL 190 rocprofv3 --pmc $C $R -d gpurun_out/recon_pmc4 -o p -- $T --erase 0,1,2,3 --recon-mix 2,1" \
 "bench:400:python3 -u bench.py"
