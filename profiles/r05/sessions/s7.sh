#!/bin/bash
# Round 5, session 7 (library of 13121b4, kept in build-old/): inputs in flight per wave
# (RSE_OPT_WIDE_DEPTH 2, 3) for 64+64 / 32+32 x 1 KiB, and the GF(2^16) 1000+24
# chain at 3 outputs per wave (RSE_OPT_WIDE_SPLIT 4: 8 waves, 145-159 VGPRs)
# against 6 (4 waves, 231-242 VGPRs).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}" || exit 1
export TMPDIR=/tmp
TU="env RSE_LIB_PATH=reed-solomon-erasure_amd/build-old/librse_hip.so python3 tools/tune.py --rounds 9 --nt-only --shapes 0:0"
G16="--field 16 --k 1000 --p 24 --shard-kib 64 --stripes 128"
W64="--k 64 --p 64 --shard-kib 1 --stripes 2048"
W32="--k 32 --p 32 --shard-kib 1 --stripes 4096"
bash tools/gpu_session.sh \
 "d64:400:for i in 1 2; do $TU $W64 && $TU $W64 --set 26=2 && $TU $W64 --set 26=3 || exit 1; done" \
 "d32:400:for i in 1 2; do $TU $W32 && $TU $W32 --set 26=2 && $TU $W32 --set 26=3 || exit 1; done" \
 "g16s4:400:for i in 1 2; do $TU $G16 && $TU $G16 --set 18=4 || exit 1; done"
