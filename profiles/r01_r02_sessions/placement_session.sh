#!/bin/bash
# 10+2 x 1 MiB (benches/bandwidth.rs's config) as the process's first device
# allocation vs after a 112 GiB one (the bench's order): throughput, kernel
# trace, and address-translation counters of the kernel in both placements.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
T="python3 tools/tune.py --field 8 --k 10 --p 2 --shard-mib 1 --stripes 2048 --rounds 2 --shapes 0:0 --nt-only"
C="TCP_UTCL1_TRANSLATION_MISS TCP_UTCL1_TRANSLATION_HIT TCP_UTCL1_STALL_MULTI_MISS TCP_UTCL1_STALL_UTCL2_REQ_OUT_OF_CREDITS"
C2="TCP_UTCL1_REQUEST TCP_UTCL1_THRASHING_STALL TCP_UTCL1_SERIALIZATION_STALL GRBM_UTCL2_BUSY GRBM_GUI_ACTIVE"
bash tools/gpu_session.sh \
 "nohog:150:$T" "hog:200:$T --hog-gib 112" \
 "tlb_nohog:150:timeout -s KILL 140 rocprofv3 --pmc $C --kernel-include-regex bitslice_kernel --output-format csv -d gpurun_out/tlb_nohog -o p -- $T" \
 "tlb_hog:200:timeout -s KILL 190 rocprofv3 --pmc $C --kernel-include-regex bitslice_kernel --output-format csv -d gpurun_out/tlb_hog -o p -- $T --hog-gib 112" \
 "tlb2_nohog:150:timeout -s KILL 140 rocprofv3 --pmc $C2 --kernel-include-regex bitslice_kernel --output-format csv -d gpurun_out/tlb2_nohog -o p -- $T" \
 "tlb2_hog:200:timeout -s KILL 190 rocprofv3 --pmc $C2 --kernel-include-regex bitslice_kernel --output-format csv -d gpurun_out/tlb2_hog -o p -- $T --hog-gib 112"
