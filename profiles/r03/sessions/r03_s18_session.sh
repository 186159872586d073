#!/bin/bash
# After the grid defaults (GF(2^8) encode 16384 workgroups at <= 2 outputs,
# GF(2^8) syndrome reconstruct 32768): GPU suite, bench, one-process A/B of
# the reconstruct default against the old 8192.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
T="python3 -u tools/tune.py --rounds 5 --nt-only --op reconstruct --patterns 0 --k 10 --p 4 --shard-mib 16 --stripes 256 --shapes 0:0,8192:0"
bash tools/gpu_session.sh \
 "pytest:900:python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread" \
 "r4:300:$T --erase 0,1,2,3" \
 "bench:600:python3 -u bench.py"
grep -A3 "GB/s" gpurun_out/r4.log | head -4
