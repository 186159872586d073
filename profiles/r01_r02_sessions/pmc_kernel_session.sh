#!/bin/bash
# SQ counters of one kernel, three passes (rocprofv3 takes at most 8 SQ
# counters per pass): tools/pmc_kernel_session.sh NAME REGEX COMMAND...
# Output: gpurun_out/pmc_NAME/pass{1,2,3}, summarised by tools/pmc_summary.py.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
name=$1; regex=$2; shift 2
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_WAVES"
P2="SQ_WAVE_CYCLES SQ_INSTS_SALU SQ_INSTS_BRANCH SQ_INSTS_SMEM SQ_INST_CYCLES_SALU SQ_ACTIVE_INST_SCA SQ_IFETCH SQ_WAVES"
P3="SQ_WAVE_CYCLES SQ_ACTIVE_INST_VMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_MISC SQ_INSTS_LDS SQ_WAVES"
i=0
for C in "$P1" "$P2" "$P3"; do
  i=$((i + 1))
  timeout -s KILL 150 rocprofv3 --pmc $C --kernel-include-regex "$regex" --output-format csv \
    -d gpurun_out/pmc_$name/pass$i -o p -- "$@" > gpurun_out/pmc_${name}_pass$i.log 2>&1 || exit $?
done
python3 tools/pmc_summary.py gpurun_out/pmc_$name "$regex" > gpurun_out/pmc_${name}_summary.json
cat gpurun_out/pmc_${name}_summary.json
