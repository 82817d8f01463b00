#!/bin/bash
# Host-side sanitizer run: the C oracle and the CPU
# build of the device rules engine (tests/hostcheck, narde_rules.h) compiled
# with AddressSanitizer + UndefinedBehaviorSanitizer (clang, host code only),
# then the CPU tests that drive them (golden vectors, random run-heavy
# positions, self-play against the oracle, FULL4).  GPU code is never
# sanitized (not available on the pool).  Usage: bash tools/sanitize.sh
set -euo pipefail
cd "$(dirname "$0")/.."
CLANG=/opt/rocm/lib/llvm/bin/clang
HIPCC=/opt/rocm/bin/hipcc
RT=$(ls /opt/rocm/lib/llvm/lib/clang/*/lib/linux/libclang_rt.asan-x86_64.so | head -1)
OUT=build/sanitize
mkdir -p "$OUT"
SAN="-fsanitize=address,undefined -fno-sanitize-recover=undefined -fno-omit-frame-pointer -g -O1"
$CLANG $SAN -std=c99 -fPIC -shared -o "$OUT/libnarde_oracle_san.so" oracle/narde_oracle.c
$HIPCC -std=c++17 -fPIC -shared -x c++ -D__HIP_PLATFORM_AMD__ -I/opt/rocm/include \
  -Xarch_host -fsanitize=address,undefined -Xarch_host -fno-sanitize-recover=undefined \
  -fno-gpu-sanitize -fno-omit-frame-pointer -g -O1 -o "$OUT/libhostcheck_san.so" tests/hostcheck/hostcheck.cpp
export NARDE_ORACLE_LIB=$PWD/$OUT/libnarde_oracle_san.so
export NARDE_HOSTCHECK_LIB=$PWD/$OUT/libhostcheck_san.so
export ASAN_OPTIONS=detect_leaks=0:abort_on_error=1
export UBSAN_OPTIONS=print_stacktrace=1:halt_on_error=1
LD_PRELOAD=$RT "${PYTHON:-python}" -m pytest -q -p no:cacheprovider tests/test_oracle_golden.py tests/test_full4_cpu.py "$@"
