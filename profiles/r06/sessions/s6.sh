#!/bin/bash
# Round 6, session 6: FFT kernels with the one-direction labels; PMC passes of
# GF(2^8) 64+64 x 1 KiB encode on the FFT kernel (RSE_OPT_FFT 1) and on the
# wide module it replaced (0): HBM traffic (FETCH_SIZE x 2, WRITE_SIZE), SQ
# instruction / wait counters, LDS.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}" || exit 1
export TMPDIR=/tmp
T="python -u -m pytest -x -q -m gpu --timeout 120 --timeout-method thread"
TUNE="python3 -u tools/tune.py --k 64 --p 64 --shard-kib 1 --stripes 4096 --nt-only --shapes 0:0 --rounds 1"
SQ=SQ_INSTS_VALU,SQ_WAVES,SQ_WAVE_CYCLES,SQ_BUSY_CYCLES,SQ_WAIT_ANY,SQ_ACTIVE_INST_VALU,SQ_WAIT_INST_ANY,SQ_ACTIVE_INST_ANY
LDS=SQ_INSTS_LDS,SQ_LDS_BANK_CONFLICT,SQ_WAIT_INST_LDS,SQ_INSTS_SALU,SQ_INSTS_VMEM_RD,SQ_INSTS_VMEM_WR,GRBM_GUI_ACTIVE
steps=("fft_tests:300:$T tests/test_gpu_fft.py")
# same-process A/B, FFT kernel (51=1) against the wide modules (51=0)
for kp in 16:8192 32:4096 64:2048; do
  k=${kp%:*}; n=${kp#*:}
  steps+=("ab$k:180:python3 -u tools/tune.py --k $k --p $k --shard-kib 1 --stripes $n --nt-only --shapes 0:0 --rounds 7 --ab 51=0,1")
done
for f in 1 0; do
  steps+=("time$f:120:$TUNE --set 51=$f")
  for pass in FETCH_SIZE WRITE_SIZE $SQ $LDS; do
    tag=$(echo $pass | cut -c1-12)
    steps+=("pmc${f}_$tag:90:rocprofv3 --pmc $pass --kernel-trace --output-format csv -d gpurun_out/pmc64_$f/$tag -o p -- $TUNE --set 51=$f")
  done
done
bash tools/gpu_session.sh "${steps[@]}"
