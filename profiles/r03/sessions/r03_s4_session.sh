#!/bin/bash
# GPU suite and bench at HEAD; then the 10+2 placement with L2-TLB and DRAM
# credit counters (first allocation vs after 16 GiB).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
bash tools/gpu_session.sh \
 "pytest:900:python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread" \
 "bench:600:python3 -u bench.py" || exit $?
T="python3 tools/tune.py --rounds 2 --nt-only --shapes 0:0 --k 10 --p 2 --shard-mib 1 --stripes 2048"
C="GRBM_UTCL2_BUSY GRBM_GUI_ACTIVE TCC_EA0_RDREQ_DRAM_CREDIT_STALL_sum TCC_EA0_WRREQ_DRAM_CREDIT_STALL_sum"
mkdir -p gpurun_out/place
for h in 0 16; do
  timeout -s KILL 150 rocprofv3 --pmc $C --output-format csv -d gpurun_out/place/hog$h -o p -- $T --hog-gib $h \
    > gpurun_out/place/hog$h.log 2>&1 || exit $?
done
python3 tools/clock_summary.py gpurun_out/place > gpurun_out/place/summary.txt
cat gpurun_out/place/summary.txt
