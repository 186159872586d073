#!/bin/bash
# Average shader clock per kernel: GRBM_GUI_ACTIVE (GPU-busy cycles) over the
# dispatch's own Start/End timestamps (tools/clock_summary.py), one rocprofv3
# --pmc pass per workload: the headline encode, GF(2^16) 20+8 encode and
# 8-erasure reconstruct, the wide 50+20 / GF(2^16) 40+12 encodes; then
# UTCL1 translation counters of 10+2 x 1 MiB as the process's first
# allocation and after a 112 GiB one (the placement spread).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out/clock
T="python3 tools/tune.py --rounds 2 --nt-only --shapes 0:0"
run() {  # name command...
  local name=$1; shift
  timeout -s KILL 150 rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT --output-format csv \
    -d gpurun_out/clock/$name -o p -- "$@" > gpurun_out/clock/$name.log 2>&1 || return $?
}
tlb() {  # name command...: translation misses of the 10+2 placement cases
  local name=$1; shift
  timeout -s KILL 150 rocprofv3 --pmc TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum \
    TCP_UTCL1_REQUEST_sum GRBM_GUI_ACTIVE --output-format csv \
    -d gpurun_out/clock/$name -o p -- "$@" > gpurun_out/clock/$name.log 2>&1 || return $?
}
run enc8_10_4 $T --k 10 --p 4 --shard-mib 16 --stripes 64 &&
run enc16_20_8 $T --field 16 --k 20 --p 8 --shard-mib 4 --stripes 128 &&
run rec16_e8 $T --field 16 --k 20 --p 8 --shard-mib 4 --stripes 128 --op reconstruct --erase 0,1,2,3,4,5,6,7 --patterns 0 --recon-mix 3 &&
run rec16_e8_onewave $T --field 16 --k 20 --p 8 --shard-mib 4 --stripes 128 --op reconstruct --erase 0,1,2,3,4,5,6,7 --patterns 0 --recon-mix 3 --set 28=0 &&
run rec16_e4 $T --field 16 --k 20 --p 8 --shard-mib 4 --stripes 128 --op reconstruct --erase 0,1,2,3 --patterns 0 --recon-mix 3 &&
run wide8_50_20 $T --k 50 --p 20 --shard-mib 1 --stripes 128 &&
run wide16_40_12 $T --field 16 --k 40 --p 12 --shard-mib 1 --stripes 128 &&
tlb tlb_10_2_first $T --k 10 --p 2 --shard-mib 1 --stripes 2048 &&
tlb tlb_10_2_hog $T --k 10 --p 2 --shard-mib 1 --stripes 2048 --hog-gib 112 &&
python3 tools/clock_summary.py gpurun_out/clock > gpurun_out/clock/summary.txt
cat gpurun_out/clock/summary.txt
