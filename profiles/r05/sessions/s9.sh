#!/bin/bash
# Round 5, session 9: the whole GPU suite (as the driver runs it), smoke and
# the bench at HEAD (wide launches sized to the device's resident workgroups
# for 1 / 2 KiB shards of k x p >= 1000 codecs; GF(2^16) 1000+24 on the chain).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}" || exit 1
export TMPDIR=/tmp
bash tools/gpu_session.sh \
 "gpu:900:python -u -m pytest tests/ -x -q -m gpu --timeout 300 --timeout-method thread" \
 "smoke:120:python3 -c 'import __graft_entry__ as g; g.smoke()'" \
 "bench:600:python3 -u bench.py --full-out gpurun_out/bench_full_n1.json"
