#!/bin/bash
# Wide one-module kernels at 3 waves per SIMD: 4 outputs per wave (RSE_OPT_
# WIDE_SPLIT 4, no power-of-two rounding of W) fits 158 VGPRs with no spills
# (50+20: W = 5); 5 outputs per wave spills at 168.  One process per option
# set (modules are built with the options current at codec creation).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
W8="python3 -u tools/tune.py --rounds 5 --nt-only --shapes 0:0 --k 50 --p 20 --shard-mib 1 --stripes 128"
W16="python3 -u tools/tune.py --rounds 5 --nt-only --shapes 0:0 --field 16 --k 40 --p 12 --shard-mib 1 --stripes 128"
W100="python3 -u tools/tune.py --rounds 3 --nt-only --shapes 0:0 --field 16 --k 100 --p 30 --shard-mib 1 --stripes 32"
bash tools/gpu_session.sh \
 "w8_def:300:$W8" \
 "w8_s4:300:$W8 --set 18=4 --set 19=0 --set 20=3" \
 "w8_s4o2:300:$W8 --set 18=4 --set 19=0" \
 "w8_def2:300:$W8" \
 "w16_def:300:$W16" \
 "w16_s4:300:$W16 --set 18=4 --set 19=0 --set 20=3" \
 "w100_def:400:$W100" \
 "w100_s4:400:$W100 --set 18=4 --set 19=0 --set 20=3"
grep -H median gpurun_out/w*.log
