#!/bin/bash
# Round 5, session 19: launch grid of the GF(2^16) 1000+24 chain's modules
# (2048 4 KiB chunks per launch at 128 stripes x 64 KiB): the fixed count (-1,
# the default for these shards) against 1 and 2 x the resident workgroups
# (RSE_OPT_WIDE_GRID), interleaved in one process.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}" || exit 1
export TMPDIR=/tmp
TU="python3 tools/tune.py --rounds 15 --nt-only --shapes 0:0"
G16="--field 16 --k 1000 --p 24 --shard-kib 64 --stripes 128"
bash tools/gpu_session.sh \
 "g16grid:400:$TU $G16 --ab 44=-1,1,2 && $TU $G16 --stripes 512 --ab 44=-1,1,2"
