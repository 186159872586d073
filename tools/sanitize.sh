#!/bin/bash
# Host-side sanitizer runs of the library, in the build container
# (no GPU): the C++ host codec (validation, planning, LRU), the run-time
# specialisation (registry, build threads, rse_jitc helper processes, disk
# cache) and the C ABI.  Device code is never instrumented: every -fsanitize=
# sits behind -Xarch_host.
#  1. ASan + UBSan build; the CPU test files that exercise the library
#     (test_capi.py: exports, matrices, every validation error, JIT builds,
#     the disk cache, exit with builds in flight) run against it.
#  2. TSan build; tools/jit_stress.cpp hammers it from 8 threads.
set -o pipefail
cd "$(dirname "$0")/.." || exit 1
PKG=reed-solomon-erasure_amd
ROOT=$(pwd)
RT=$(/opt/rocm/bin/hipcc -print-file-name=libclang_rt.asan-x86_64.so)
A=$ROOT/$PKG/build-asan
T=$ROOT/$PKG/build-tsan
echo "== ASan+UBSan build"
make -s -C $PKG -j8 OBJ=$A OUT=$A/librse_hip.so JITC=$A/rse_jitc \
  SAN="-Xarch_host -fsanitize=address -Xarch_host -fsanitize=undefined -Xarch_host -fno-sanitize-recover=undefined -Xarch_host -fno-omit-frame-pointer" || exit 1
echo "== CPU tests against the ASan+UBSan library"
ASAN_OPTIONS=detect_leaks=0:verify_asan_link_order=0:abort_on_error=1 \
UBSAN_OPTIONS=print_stacktrace=1:halt_on_error=1 \
LD_PRELOAD=$RT RSE_LIB_PATH=$A/librse_hip.so \
  python -m pytest tests/test_capi.py -q -p no:cacheprovider || exit 1
echo "== TSan build"
make -s -C $PKG -j8 OBJ=$T OUT=$T/librse_hip.so JITC=$T/rse_jitc \
  SAN="-Xarch_host -fsanitize=thread -Xarch_host -fno-omit-frame-pointer" || exit 1
/opt/rocm/bin/hipcc -O1 -g -Xarch_host -fsanitize=thread -o $T/jit_stress tools/jit_stress.cpp \
  -L$T -lrse_hip -Wl,-rpath,$T || exit 1
echo "== jit_stress under TSan"
RSE_JIT_CACHE_DIR=$(mktemp -d) TSAN_OPTIONS=halt_on_error=1:second_deadlock_stack=1 $T/jit_stress
