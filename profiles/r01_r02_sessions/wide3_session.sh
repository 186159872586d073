#!/bin/bash
# Wide codecs (k > 32 or p > 8) on their one-module kernels (rse_jit.cpp
# kJitWide: each wave of a workgroup codes <= 8 outputs over all k inputs of
# the same 4 KiB chunk) against the table kernels (--bitslice 0), same
# process; the builds are waited for first.  b: slicing shared through LDS
# (RSE_OPT_WIDE_LDS 1, default) against every wave slicing every input (0),
# separate processes (the module is built once per process).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
T="python -u tools/tune.py --rounds 3 --nt-only --shapes 0:0 --bitslice 0,1"
P="python -u -m pytest -x -v --timeout 600 --timeout-method thread"
case "$1" in
  a) bash tools/gpu_session.sh \
      "pytest_wide:900:$P tests/test_gpu_parity.py -k wide" \
      "w8_10_16:300:$T --k 10 --p 16 --shard-mib 1 --stripes 256" \
      "w16_40_12:400:$T --field 16 --k 40 --p 12 --shard-mib 1 --stripes 64" \
      "w8_50_20:400:$T --k 50 --p 20 --shard-mib 1 --stripes 64" ;;
  b) S="python -u tools/tune.py --rounds 5 --nt-only --shapes 0:0 --bitslice 1"
     bash tools/gpu_session.sh \
      "pytest_wide:900:$P tests/test_gpu_parity.py -k wide" \
      "lds1_8_10_16:300:$S --wide-lds 1 --k 10 --p 16 --shard-mib 1 --stripes 256" \
      "lds0_8_10_16:300:$S --wide-lds 0 --k 10 --p 16 --shard-mib 1 --stripes 256" \
      "lds1_16_40_12:400:$S --wide-lds 1 --field 16 --k 40 --p 12 --shard-mib 1 --stripes 64" \
      "lds0_16_40_12:400:$S --wide-lds 0 --field 16 --k 40 --p 12 --shard-mib 1 --stripes 64" \
      "lds1_8_50_20:400:$S --wide-lds 1 --k 50 --p 20 --shard-mib 1 --stripes 64" \
      "lds0_8_50_20:400:$S --wide-lds 0 --k 50 --p 20 --shard-mib 1 --stripes 64" \
      "lds1_16_100_30:600:$S --wide-lds 1 --field 16 --k 100 --p 30 --shard-mib 1 --stripes 32" ;;
esac
