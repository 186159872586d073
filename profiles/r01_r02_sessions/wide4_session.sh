#!/bin/bash
# Wide codecs: waves per workgroup rounded to 2/4/8 (RSE_OPT_WIDE_BALANCE 19,
# default) against W = ceil(p / 8), and smaller shares per wave
# (RSE_OPT_WIDE_SPLIT 18).  One process per configuration (a codec's module is
# built once per process).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
P="python -u -m pytest -x -q --timeout 600 --timeout-method thread"
T="python -u tools/tune.py --rounds 5 --nt-only --shapes 0:0 --bitslice 1"
W8="--k 50 --p 20 --shard-mib 1 --stripes 64"
W16="--field 16 --k 40 --p 12 --shard-mib 1 --stripes 64"
W100="--field 16 --k 100 --p 30 --shard-mib 1 --stripes 32"
W10="--k 10 --p 16 --shard-mib 1 --stripes 256"
bash tools/gpu_session.sh \
 "pytest_wide:900:$P tests/test_gpu_parity.py -k wide" \
 "w8_bal:300:$T $W8" \
 "w8_unbal:300:$T $W8 --set 19=0" \
 "w8_s4:300:$T $W8 --set 18=4" \
 "w16_bal:300:$T $W16" \
 "w16_s4:300:$T $W16 --set 18=4" \
 "w16_s3:300:$T $W16 --set 18=3" \
 "w100_bal:400:$T $W100" \
 "w100_s5:400:$T $W100 --set 18=5" \
 "w10_bal:300:$T $W10" \
 "w10_s4:300:$T $W10 --set 18=4"
