#!/bin/bash
# Round-2 evidence: rocprofv3 kernel trace + stats of the headline bench, the
# PMC traffic of the headline kernel (tools/pmc_traffic.py, which attaches
# the kernel id and commit), the HBM traffic of the one-module wide kernels
# (FETCH_SIZE / WRITE_SIZE in separate passes), then the full bench.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
W="--kernel-include-regex rse_jit_wide --output-format csv"
T="python3 tools/tune.py --rounds 1 --nt-only --shapes 0:0 --bitslice 1 --shard-mib 1 --stripes 64"
bash tools/gpu_session.sh \
 "trace:400:rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r02_trace -o bench -- python3 bench.py --no-cpu --no-extras --steps 10" \
 "pmc:600:python3 tools/pmc_traffic.py --tag r02 --steps 5" \
 "wf50:200:timeout -s KILL 190 rocprofv3 --pmc FETCH_SIZE $W -d gpurun_out/wide_f50 -o p -- $T --k 50 --p 20" \
 "ww50:200:timeout -s KILL 190 rocprofv3 --pmc WRITE_SIZE $W -d gpurun_out/wide_w50 -o p -- $T --k 50 --p 20" \
 "wf40:200:timeout -s KILL 190 rocprofv3 --pmc FETCH_SIZE $W -d gpurun_out/wide_f40 -o p -- $T --field 16 --k 40 --p 12" \
 "ww40:200:timeout -s KILL 190 rocprofv3 --pmc WRITE_SIZE $W -d gpurun_out/wide_w40 -o p -- $T --field 16 --k 40 --p 12" \
 "bench:600:python3 -u bench.py"
