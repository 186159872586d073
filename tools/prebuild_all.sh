#!/bin/bash
# Prebuilds, on the host CPU, every run-time specialised module bench.py loads
# (its wide codecs, the reference bench matrix's codecs and decode patterns,
# the GF(2^16) cached-pattern leg) into the tree's jitcache/, so a GPU run
# loads them in milliseconds.  Rerun after any change to the JIT sources
# (rse_bitslice_core.hpp and the headers rse_jit.cpp embeds): the cache key
# hashes the whole source, so stale entries are simply never hit.
cd "$(dirname "$0")/.." || exit 1
export RSE_JIT_CACHE_DIR=$PWD/jitcache
mkdir -p jitcache
pat=()
seq_csv() { python3 -c "print(','.join(str(i) for i in range($1)))"; }
# benches/bandwidth.rs:88-190 shapes (bench.py REF_BENCH_SHAPES): erase shard 0,
# and data shards 0..p-1
# (16+16, 32+32, 64+64 rebuild all data from the parity on the additive-FFT
# kernels, rse_fft.hip: no pattern module)
for kp in 4:4 8:8 16:16 32:32 64:64 5:2 10:4 50:20; do
  k=${kp%:*}; p=${kp#*:}
  pat+=(--pattern "8:$k:$p:1024:0")
  case $k in 16|32|64) ;; *) pat+=(--pattern "8:$k:$p:1024:$(seq_csv "$p")") ;; esac
done
pat+=(--pattern "8:4:4:2048:0" --pattern "8:4:4:2048:0,1,2,3")
pat+=(--pattern "16:20:8:4194304:0,1,2,3")  # other_configs gf16_20_8 cached pattern
# tests/test_gpu_parity.py test_wide_full_chunks_option: one codec on full
# (4 KiB) chunks, RSE_OPT_WIDE_HALF 0, in a process of its own
python3 tools/prebuild_jit.py --set 38=0 --codec 8:34:10 || exit 1
# 16+16 .. 64+64's wide modules (RSE_OPT_FFT 0: tests/test_gpu_parity.py
# test_wide_codec_kernels, test_sub_chunk_shards; the default is the FFT kernels)
python3 tools/prebuild_jit.py --set 51=0 --codec 8:16:16 --codec 8:32:32 --codec 8:64:64 || exit 1
# tests/test_gpu_parity.py test_wide_output_groups: past 64 outputs, groups
# of <= 64 (one module each; 40+70 with 16-input blocks: chains of three)
python3 tools/prebuild_jit.py --set 46=16 --codec 8:40:70 || exit 1
# test_wide_sixteen_waves: 4 outputs per wave (a 16-wave module)
python3 tools/prebuild_jit.py --set 18=4 --codec 8:60:60 || exit 1
exec python3 tools/prebuild_jit.py --codec 8:35:10 --codec 8:20:70 --codec 8:128:128 --codec 8:4:66 \
  --codec 8:50:20 --codec 16:40:12 --codec 16:100:30 \
  --codec 8:4:4 --codec 8:8:8 --codec 8:16:16 --codec 8:32:32 --codec 8:64:64 --codec 8:5:2 \
  --codec 8:12:4 --codec 16:6:3 --codec 8:6:3 --codec 8:32:8 --codec 8:17:5 --codec 16:1000:24 \
  "${pat[@]}"
