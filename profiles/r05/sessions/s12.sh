#!/bin/bash
# Round 5, session 12: RSE_OPT_WIDE_SPLIT auto (4 outputs per wave for GF(2^8)
# codecs past 48 parity rows: 64+64 in 16 waves) against 8, with the default
# launch grid (resident workgroups for 1 KiB k x p >= 1000 codecs); the wide
# parity tests; a kernel trace of one-stripe verify calls (tools/verify_probe.py).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}" || exit 1
export TMPDIR=/tmp
PY="python -u -m pytest -x -v --timeout 300 --timeout-method thread"
TU="python3 tools/tune.py --rounds 9 --nt-only --shapes 0:0"
W64="--k 64 --p 64 --shard-kib 1 --stripes 2048"
bash tools/gpu_session.sh \
 "tests:600:$PY tests/test_gpu_parity.py -k 'wide or sub_chunk'" \
 "s64:300:for i in 1 2; do $TU $W64 && $TU $W64 --set 18=8 || exit 1; done" \
 "vp:200:timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/vp -o t -- python3 tools/verify_probe.py"
