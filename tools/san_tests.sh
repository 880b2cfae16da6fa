#!/bin/bash
# Sanitized CPU run (CPU only, never on the GPU box): the library's host code
# (scene compile, SBVH / 4-wide builders, .xmsh reader and writer, the C ABI's
# host side) and the oracle built with AddressSanitizer + UndefinedBehavior-
# Sanitizer (make SAN=1), then the CPU test suite against those builds with the
# clang runtime preloaded.  The reference keeps its bounds checks on
# (Defines.h:65-75, Base/Buffer_device.h:17); this is the build's equivalent.
set -eo pipefail
cd "$(dirname "$0")/.."
make -s -C cudatracerlib_amd SAN=1 -j"${JOBS:-8}"
make -s -C oracle SAN=1
RT=$(/opt/rocm/lib/llvm/bin/clang++ -print-file-name=libclang_rt.asan-x86_64.so)
# python and numpy allocate outside the sanitizer's view: no leak report at exit
export ASAN_OPTIONS=detect_leaks=0:abort_on_error=1:halt_on_error=1
export UBSAN_OPTIONS=print_stacktrace=1:halt_on_error=1
export CTL_LIB=$PWD/cudatracerlib_amd/_san/lib/libctl_trace.so
export ORACLE_LIB=$PWD/oracle/_san/liboracle.so
LD_PRELOAD="$RT${LD_PRELOAD:+ $LD_PRELOAD}" python -m pytest tests -x -q -m "not gpu" -p no:cacheprovider "$@"
