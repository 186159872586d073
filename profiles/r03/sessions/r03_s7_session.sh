#!/bin/bash
# Wide GF(2^8) modules over paired inputs (RSE_OPT_WIDE_PAIRS 1, default)
# against one input at a time (0): wide parity tests, then alternating
# processes (the option applies when a module is built).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
W8="python3 -u tools/tune.py --rounds 5 --nt-only --shapes 0:0 --k 50 --p 20 --shard-mib 1 --stripes 128"
W10="python3 -u tools/tune.py --rounds 5 --nt-only --shapes 0:0 --k 10 --p 16 --shard-mib 1 --stripes 256"
W33="python3 -u tools/tune.py --rounds 5 --nt-only --shapes 0:0 --k 33 --p 9 --shard-mib 1 --stripes 256"
bash tools/gpu_session.sh \
 "pytest_wide:900:python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py -m gpu -k 'wide or full_size'" || exit $?
grep -q " passed" gpurun_out/pytest_wide.log && ! grep -q -E "[0-9]+ failed" gpurun_out/pytest_wide.log || exit 1
bash tools/gpu_session.sh \
 "w8_pairs:300:$W8" \
 "w8_single:300:$W8 --set 29=0" \
 "w8_pairs2:300:$W8" \
 "w8_single2:300:$W8 --set 29=0" \
 "w10_pairs:300:$W10" \
 "w10_single:300:$W10 --set 29=0" \
 "w33_pairs:300:$W33" \
 "w33_single:300:$W33 --set 29=0"
grep -H median gpurun_out/w*.log
