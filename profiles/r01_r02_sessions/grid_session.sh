#!/bin/bash
# Workgroup-count sweep: does a grid that is a whole number of co-resident
# rounds (occupancy x 256 CUs) beat the fixed defaults?
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
R="python -u tools/tune.py --op reconstruct --rounds 3 --nt-only --bitslice 1 --patterns 1 --k 10 --p 4 --erase 0,1"
bash tools/gpu_session.sh \
 "enc:300:python -u tools/tune.py --k 10 --p 4 --stripes 448 --rounds 3 --nt-only --shapes 768:1,1536:1,2304:1,3072:1,3840:1,4096:1,4608:1,6144:1,8192:1" \
 "rec64:300:$R --stripes 64 --shapes 1024:1,1280:1,2048:1,2560:1,3840:1,4096:1,5120:1,6400:1" \
 "rec448:300:$R --stripes 448 --shapes 1024:1,1280:1,2048:1,2560:1,3840:1,4096:1,5120:1,6400:1"
