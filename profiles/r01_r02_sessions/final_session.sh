#!/bin/bash
# Round-2 (second session) evidence: VALU PMC of the GF(2^16) 20+8 encode
# kernel with the factor16 network, rocprofv3 trace + stats of the headline
# bench, then the full bench.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
C="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_WAVES"
bash tools/gpu_session.sh \
 "pmc16:150:timeout -s KILL 140 rocprofv3 --pmc $C --kernel-include-regex bitslice_kernel --output-format csv -d gpurun_out/pmc_valu16 -o p -- python3 tools/tune.py --field 16 --k 20 --p 8 --shard-mib 4 --stripes 128 --rounds 1 --shapes 0:0 --nt-only" \
 "trace:400:rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/trace -o bench -- python3 bench.py --no-cpu --no-extras --steps 10" \
 "bench:600:python3 -u bench.py"
