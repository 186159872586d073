#!/bin/bash
# Round 5, session 14: what the batch's largest need costs.  reconstruct_batch
# of GF(2^16) 20+8 x 4 KiB x 65536 with parity rebuilt (tools/tune.py
# --batch-parity), every stripe the same pattern: 3 data + parity 0 lost (sigma
# rows 0-3: the 4-row kernels) against 3 data + parity 5-7 (8 rows), three
# rotations of each pattern (--batch-cycle 3: no shared-pattern kernel), and the
# random-pattern batch as the bench runs it.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}" || exit 1
export TMPDIR=/tmp
TB="python3 tools/tune.py --op batch --batch-parity --field 16 --k 20 --p 8 --shard-kib 4 --stripes 65536 --rounds 9 --nt-only --shapes 0:0"
bash tools/gpu_session.sh \
 "b4:400:for i in 1 2; do $TB --erase 0,1,2,20 --batch-cycle 3 && $TB --erase 0,1,2,25 --batch-cycle 3 && $TB --erase 0,1,2,3 || exit 1; done"
