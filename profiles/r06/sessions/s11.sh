#!/bin/bash
# Round 6, session 11: FFT tests (GF(2^16) subfield codecs added); the batch
# reconstruct (GF(2^16) 20+8 x 4 KiB x 65536 stripes, 4 random shards lost
# per stripe, lost parity rebuilt too): timing, kernel trace and PMC passes.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}" || exit 1
export TMPDIR=/tmp
T="python -u -m pytest -x -q -m gpu --timeout 120 --timeout-method thread"
B="python3 -u tools/tune.py --op batch --batch-parity --field 16 --k 20 --p 8 --shard-kib 4 --stripes 65536 --erase 0,1,2,3 --nt-only --shapes 0:0"
SQ=SQ_INSTS_VALU,SQ_WAVES,SQ_WAVE_CYCLES,SQ_BUSY_CYCLES,SQ_WAIT_ANY,SQ_ACTIVE_INST_VALU,SQ_WAIT_INST_ANY,SQ_ACTIVE_INST_ANY
LDS=SQ_INSTS_LDS,SQ_LDS_BANK_CONFLICT,SQ_WAIT_INST_LDS,SQ_INSTS_SALU,SQ_INSTS_VMEM_RD,SQ_INSTS_VMEM_WR,SQ_INSTS_BRANCH,GRBM_GUI_ACTIVE
steps=("fft_tests:300:$T tests/test_gpu_fft.py" "batch_time:200:$B --rounds 5"
       "batch_trace:200:rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/b4k/trace -o t -- $B --rounds 2")
for pass in FETCH_SIZE WRITE_SIZE $SQ $LDS; do
  tag=$(echo $pass | cut -c1-12)
  steps+=("b4k_$tag:120:rocprofv3 --pmc $pass --kernel-trace --output-format csv -d gpurun_out/b4k/$tag -o p -- $B --rounds 1")
done
bash tools/gpu_session.sh "${steps[@]}"
