#!/bin/bash
# Round 4, session 2: the new bench legs and pair variants on the GPU; the
# 8-erasure GF(2^16) reconstruct split by phase (RSE_OPT_RECON_PAIRS 4 / 5
# skip the Horner steps / data networks) and the compact mixing (6); wide
# codecs' occupancy (SQ + GRBM pass beside a kernel trace of the same
# command) and grid; reconstruct_batch of 4 KiB shards with the new planner;
# the reference's bench matrix.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
export RSE_JIT_CACHE_DIR=$PWD/jitcache
T16="python3 -u tools/tune.py --nt-only --field 16 --k 20 --p 8 --shapes 0:0"
W50="python3 -u tools/tune.py --nt-only --field 8 --k 50 --p 20 --shard-mib 1 --stripes 128"
W40="python3 -u tools/tune.py --nt-only --field 16 --k 40 --p 12 --shard-mib 1 --stripes 128"
bash tools/gpu_session.sh \
 "tests:400:python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_bench_checks.py tests/test_gpu_parity.py -m gpu -k 'bench or wave_pairs'" \
 "r8ab:300:$T16 --rounds 3 --shard-mib 4 --stripes 128 --op reconstruct --patterns 0 --erase 0,1,2,3,4,5,6,7 --recon-mix 3 --ab 28=1,4,5,6" \
 "w50:300:$W50 --rounds 3 --shapes 2048:0,4096:0,8192:0,16384:0" \
 "w40:300:$W40 --rounds 3 --shapes 2048:0,4096:0,8192:0,16384:0" \
 "w50_trace:200:rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/w50_trace -o t -- $W50 --rounds 1 --shapes 0:0" \
 "w50_pmc:200:timeout -s KILL 150 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAVES SQ_INSTS_VALU SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_WAIT_ANY GRBM_GUI_ACTIVE GRBM_COUNT --kernel-include-regex rse_jit_wide --output-format csv -d gpurun_out/w50_pmc -o p -- $W50 --rounds 1 --shapes 0:0" \
 "w40_trace:200:rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/w40_trace -o t -- $W40 --rounds 1 --shapes 0:0" \
 "w40_pmc:200:timeout -s KILL 150 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAVES SQ_INSTS_VALU SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_WAIT_ANY GRBM_GUI_ACTIVE GRBM_COUNT --kernel-include-regex rse_jit_wide --output-format csv -d gpurun_out/w40_pmc -o p -- $W40 --rounds 1 --shapes 0:0" \
 "b4k_e4:300:$T16 --rounds 3 --shard-kib 4 --stripes 65536 --op batch --erase 0,1,2,3" \
 "b4k_e8:300:$T16 --rounds 3 --shard-kib 4 --stripes 65536 --op batch --erase 0,1,2,3,4,5,6,7" \
 "b4k_trace:200:rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/b4k_trace -o t -- python3 tools/tune.py --rounds 2 --nt-only --shapes 0:0 --field 16 --k 20 --p 8 --shard-kib 4 --stripes 65536 --op batch --erase 0,1,2,3" \
 "matrix:300:python3 -u -c 'import json, torch, bench; print(json.dumps(bench.reference_bench_matrix(torch.cuda.current_stream())))'"
