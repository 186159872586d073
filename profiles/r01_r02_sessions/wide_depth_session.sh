#!/bin/bash
# Wide codecs: inputs in flight per wave (RSE_OPT_WIDE_DEPTH 1..4), one process
# per depth and codec, modules prebuilt on the host (tools/prebuild_jit.py).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export RSE_JIT_CACHE_DIR="$PWD/jitcache"
steps=()
for c in "8 50 20 1024" "16 40 12 1024" "16 100 30 1024" "8 10 16 1024"; do
  set -- $c
  for d in 1 2 3 4; do
    steps+=("wide_${1}_${2}_${3}_d$d:120:python3 tools/tune.py --field $1 --k $2 --p $3 --shard-kib $4 --stripes 128 --rounds 3 --shapes 0:0 --nt-only --set 26=$d")
  done
done
bash tools/gpu_session.sh "${steps[@]}"
