#!/bin/bash
# Round-3 evidence at HEAD: GPU suite, rocprofv3 kernel trace + stats of the
# headline bench, PMC traffic of the headline kernel (stamped from BUILD_INFO),
# SQ counter passes of the GF(2^16) 8-erasure reconstruct and the 50+20 wide
# kernel, then the full bench.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
export RSE_JIT_CACHE_DIR=$PWD/jitcache
T16="python3 tools/tune.py --rounds 1 --nt-only --shapes 0:0 --field 16 --k 20 --p 8 --shard-mib 4 --stripes 128"
bash tools/gpu_session.sh \
 "pytest:900:python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread" \
 "trace:400:rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/trace -o bench -- python3 bench.py --no-cpu --no-extras --steps 10" \
 "pmc_traffic:600:python3 tools/pmc_traffic.py --tag r03 --steps 5" \
 "pmc_recon8:500:bash tools/pmc_kernel_session.sh recon8 bitslice_recon_kernel $T16 --op reconstruct --erase 0,1,2,3,4,5,6,7 --patterns 0" \
 "pmc_wide50:500:bash tools/pmc_kernel_session.sh wide50 rse_jit_wide python3 tools/tune.py --rounds 1 --nt-only --shapes 0:0 --k 50 --p 20 --shard-mib 1 --stripes 64" \
 "bench:600:python3 -u bench.py"
