#!/bin/bash
# Host-code sanitizer run: rebuild the C++ runtime (bindings, RCCL comm,
# fusion engine, PS service, loader) and the ImageNet reader with AddressSanitizer + UBSan
# into build_san/ (the in-tree modules are untouched; device code is compiled as usual), then
# run the CPU tests that drive that host code -- native PS over shared memory incl. worker
# failure, the fusion engine over gloo, the mmap loader, TFRecord/JPEG decoding -- with the
# sanitizer runtime preloaded into Python.  CPU only; never on the GPU pool.
#
#   bash scripts/sanitize_host.sh [pytest -k expression]
set -euo pipefail
cd "$(dirname "$0")/.."
OUT=${PDDL_SAN_DIR:-build_san}
mkdir -p "$OUT"
PDDL_SANITIZE=1 PDDL_BUILD_TEMP=/tmp/pddl_build_san python setup.py build_ext --build-lib "$OUT" \
    --build-temp /tmp/pddl_build_san > "$OUT/build.log" 2>&1 || { tail -30 "$OUT/build.log"; exit 1; }
rm -rf build
ASAN_LIB=$(gcc -print-file-name=libasan.so)
UBSAN_LIB=$(gcc -print-file-name=libubsan.so)
export PDDL_NATIVE_DIR="$PWD/$OUT"
# leaks: CPython and libtorch keep interned / cached allocations alive at exit by design
export ASAN_OPTIONS=detect_leaks=0:halt_on_error=1:abort_on_error=0:protect_shadow_gap=0:verify_asan_link_order=0
export UBSAN_OPTIONS=print_stacktrace=1:halt_on_error=1
K=${1:-"native or records or tfrecord or folder or horovod"}
LD_PRELOAD="$ASAN_LIB $UBSAN_LIB" python -m pytest -x -q -m "not gpu" -p no:cacheprovider \
    tests/test_ps_checkpoint_cli.py tests/test_imagenet_io.py tests/test_launch_data_callbacks.py \
    tests/test_strategies_cpu.py -k "$K" 2>&1 | tee "$OUT/sanitize.log"
