#!/bin/bash
# Round 6, session 14: which kernels the batch reconstruct runs under
# RSE_OPT_RECON_W4_PAIRS 0 / 2 (kernel trace), and their durations.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}" || exit 1
export TMPDIR=/tmp
B="python3 -u tools/tune.py --op batch --batch-parity --field 16 --k 20 --p 8 --shard-kib 4 --stripes 65536 --erase 0,1,2,3 --nt-only --shapes 0:0 --rounds 3"
bash tools/gpu_session.sh \
 "tr0:200:rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/b4k_w4p/t0 -o t -- $B --set 54=0" \
 "tr2:200:rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/b4k_w4p/t2 -o t -- $B --set 54=2"
