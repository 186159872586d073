#!/bin/bash
# Round 5, session 22: the narrow modules' 1 / 2 KiB-shard kernels with 2 / 4
# inputs in flight per wave (RSE_OPT_SUB_DEPTH, rse_sub_ext.hpp) against 1:
# bytes against the oracle, then the reference bench's short 1 KiB launches.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}" || exit 1
export TMPDIR=/tmp
TU="python3 tools/tune.py --rounds 9 --nt-only --shapes 0:0"
E8="--k 8 --p 8 --shard-kib 1 --stripes 16384"
E4="--k 4 --p 4 --shard-kib 1 --stripes 32768"
R16="--op reconstruct --erase 0 --k 16 --p 16 --shard-kib 1 --stripes 8192"
bash tools/gpu_session.sh \
 "check:300:python3 tools/sub_depth_check.py 4 && python3 tools/sub_depth_check.py 2" \
 "e8:300:for i in 1 2; do $TU $E8 && $TU $E8 --set 50=2 && $TU $E8 --set 50=4 || exit 1; done" \
 "e4:300:for i in 1 2; do $TU $E4 && $TU $E4 --set 50=2 && $TU $E4 --set 50=4 || exit 1; done" \
 "r16:300:for i in 1 2; do $TU $R16 && $TU $R16 --set 50=2 && $TU $R16 --set 50=4 || exit 1; done"
