#!/bin/bash
# Syndrome reconstruct (first use of an erasure pattern: no decode-pattern
# kernel) with the e x e mixing bit-sliced (mix=1, default) against the v_perm
# table mixing (mix=0), in one process per configuration.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
T="python -u tools/tune.py --op reconstruct --rounds 5 --nt-only --bitslice 1 --patterns 0 --recon-mix 1,0 --shapes 0:0"
P="python -u -m pytest -x -q --timeout 600 --timeout-method thread"
bash tools/gpu_session.sh \
 "pytest_recon:900:$P tests/test_gpu_parity.py -k 'reconstruct or bitslice or decode'" \
 "pytest_host:600:$P tests/test_gpu_host_paths.py" \
 "r16_e1:300:$T --field 16 --k 20 --p 8 --shard-mib 4 --stripes 256 --erase 0" \
 "r16_e2:300:$T --field 16 --k 20 --p 8 --shard-mib 4 --stripes 256 --erase 0,1" \
 "r16_e4:300:$T --field 16 --k 20 --p 8 --shard-mib 4 --stripes 256 --erase 0,1,2,3" \
 "r16_e8:300:$T --field 16 --k 20 --p 8 --shard-mib 4 --stripes 256 --erase 0,1,2,3,4,5,6,7" \
 "r8_e2:300:$T --k 10 --p 4 --stripes 128 --erase 0,1" \
 "r8_e4:300:$T --k 10 --p 4 --stripes 128 --erase 0,1,2,3" \
 "b16_e4:300:python -u tools/tune.py --op batch --rounds 5 --nt-only --bitslice 1 --shapes 0:0 --field 16 --k 20 --p 8 --shard-mib 4 --stripes 256 --erase 0,1,2,3"
