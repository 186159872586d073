#!/bin/bash
# Syndrome reconstruct, first use of an erasure pattern: the e x e mixing by
# Horner's rule (mix=2, default) against the round-2 doubling chains (mix=1)
# and the v_perm tables (mix=0), one process per configuration; then the
# per-stripe-pattern batch (device planner, default mixing).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
T="python -u tools/tune.py --op reconstruct --rounds 5 --nt-only --bitslice 1 --patterns 0 --recon-mix 2,1,0 --shapes 0:0"
B="python -u tools/tune.py --op batch --rounds 5 --nt-only --bitslice 1 --shapes 0:0"
P="python -u -m pytest -x -q --timeout 600 --timeout-method thread"
G16="--field 16 --k 20 --p 8 --shard-mib 4 --stripes 256"
bash tools/gpu_session.sh \
 "pytest_recon:900:$P tests/test_gpu_parity.py -k 'reconstruct or bitslice or decode or batch'" \
 "r16_e8:300:$T $G16 --erase 0,1,2,3,4,5,6,7" \
 "r16_e4:300:$T $G16 --erase 0,1,2,3" \
 "r16_e2:300:$T $G16 --erase 0,1" \
 "r16_e1:300:$T $G16 --erase 0" \
 "r16_p6:300:$T $G16 --erase 0,1,2,20,21,22" \
 "r8_e2:300:$T --k 10 --p 4 --stripes 128 --erase 0,1" \
 "r8_e4:300:$T --k 10 --p 4 --stripes 128 --erase 0,1,2,3" \
 "b16_e4:300:$B $G16 --erase 0,1,2,3" \
 "b16_e8:300:$B $G16 --erase 0,1,2,3,4,5,6,7" \
 "b8_e4:300:$B --k 10 --p 4 --stripes 128 --erase 0,1,2,3"
