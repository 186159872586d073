#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
bash tools/gpu_session.sh \
 "pytest:900:python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread" \
 "t20_8:300:python -u tools/tune.py --field 16 --k 20 --p 8 --shard-mib 4 --stripes 256 --rounds 3 --variants 2 --shapes 4096:1,8192:1 --nt-only" \
 "r20_8:300:python -u tools/tune.py --op reconstruct --field 16 --k 20 --p 8 --shard-mib 4 --stripes 256 --rounds 3 --shapes 8192:1 --nt-only --patterns 0 --erase 0,1,2,3" \
 "bench:600:python -u bench.py"
