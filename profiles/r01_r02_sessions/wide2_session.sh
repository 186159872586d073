#!/bin/bash
# Wide codecs (k > 32 or p > 8) on their bit-sliced block kernels
# (rse_jit.cpp kJitBlock / kJitBlockAcc) against the table kernels
# (--bitslice 0), same process; the block builds are waited for first.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
T="python -u tools/tune.py --rounds 3 --nt-only --shapes 0:0 --bitslice 0,1"
P="python -u -m pytest -x -v --timeout 300 --timeout-method thread"
case "$1" in
  a) bash tools/gpu_session.sh \
      "pytest_wide:500:$P tests/test_gpu_parity.py -k wide_codec" \
      "w8_10_16:200:$T --k 10 --p 16 --shard-mib 1 --stripes 256" \
      "w16_40_12:400:$T --field 16 --k 40 --p 12 --shard-mib 1 --stripes 64" ;;
  b) bash tools/gpu_session.sh \
      "w8_50_20:200:$T --k 50 --p 20 --shard-mib 1 --stripes 64" \
      "w16_100_30:300:$T --field 16 --k 100 --p 30 --shard-mib 1 --stripes 32" \
      "w16_200_56:600:$T --field 16 --k 200 --p 56 --shard-kib 256 --stripes 32" ;;
  c) R="python -u tools/tune.py --rounds 3 --nt-only --shapes 0:0 --op reconstruct --patterns 1 --bitslice 0,1"
     bash tools/gpu_session.sh \
      "r16_40_12:300:$R --field 16 --k 40 --p 12 --shard-mib 1 --stripes 64 --erase 0,1,2,3" \
      "r8_50_20:300:$R --k 50 --p 20 --shard-mib 1 --stripes 64 --erase 0,1,2,3,4,5,6,7,8,9" ;;
esac
