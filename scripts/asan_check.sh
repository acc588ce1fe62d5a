#!/bin/bash
# Host AddressSanitizer + UndefinedBehaviorSanitizer run of the CPU test
# suite's native code: the library's host side (packer K0, synthetic generator, runtime
# host paths with device = -1, scalar decision math), the C oracle (incl. the OpenMP
# B-opt pass) and the C harness of the cgo shim's call sequence.  CPU only: GPU
# sanitizers are not available on the GPU pool.
set -euo pipefail
cd "$(dirname "$0")/.."
make -s -C escalator_amd/csrc            # the device-code object the ASan build links
make -s -C escalator_amd/csrc asan
make -s -C oracle asan
rm -f build/asan/esc_harness
make -s -C go/escalatorhip/harness OUT=../../../build/asan/esc_harness CC=/opt/rocm/llvm/bin/clang \
    CFLAGS="-O1 -g -std=c11 -Wall -fsanitize=address -fsanitize=undefined -fno-sanitize-recover=undefined -shared-libasan" \
    LIBDIR=../../../build/asan RPATH=$PWD/build/asan >/dev/null
RT=$(/opt/rocm/llvm/bin/clang -print-file-name=libclang_rt.asan-x86_64.so)
[ -f "$RT" ] || RT=/opt/rocm/llvm/lib/clang/22/lib/linux/libclang_rt.asan-x86_64.so
export LD_PRELOAD="$RT"
export ASAN_OPTIONS=detect_leaks=0:abort_on_error=1:halt_on_error=1:detect_odr_violation=0
export UBSAN_OPTIONS=print_stacktrace=1:halt_on_error=1
export ESC_LIB_PATH=$PWD/build/asan/libescalator_hip.so
export ESC_ORACLE_LIB=$PWD/build/asan/liboracle.so
export ESC_HARNESS=$PWD/build/asan/esc_harness
export ESC_NO_TORCH_PRELOAD=1
python -m pytest -q -p no:cacheprovider -m "not gpu" \
    tests/test_abi.py tests/test_pack_parity.py tests/test_oracle_fixtures.py tests/test_oracle_par.py \
    tests/test_harness.py "$@"
echo "asan/ubsan: clean"
