#!/bin/bash
# Round 5, session 13: half-chunk wide modules with 2 / 4 input pairs per
# scheduling region (RSE_OPT_WIDE_PIN_PAIRS, rse_wide_ext.hpp) against 1,
# alternating processes, for the 1 KiB reference-bench shapes.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}" || exit 1
export TMPDIR=/tmp
TU="python3 tools/tune.py --rounds 9 --nt-only --shapes 0:0"
W64="--k 64 --p 64 --shard-kib 1 --stripes 2048"
W32="--k 32 --p 32 --shard-kib 1 --stripes 4096"
W50="--k 50 --p 20 --shard-kib 1 --stripes 3744"
bash tools/gpu_session.sh \
 "pp64:300:for i in 1 2; do $TU $W64 && $TU $W64 --set 48=2 && $TU $W64 --set 48=4 || exit 1; done" \
 "pp32:300:for i in 1 2; do $TU $W32 && $TU $W32 --set 48=2 && $TU $W32 --set 48=4 || exit 1; done" \
 "pp50:300:for i in 1 2; do $TU $W50 && $TU $W50 --set 48=2 && $TU $W50 --set 48=4 || exit 1; done"
