#!/bin/bash
# Host-code sanitizer runs.  CPU only; never on the GPU pool.
#
#  1. UBSan inside Python: rebuild the C++ runtime (bindings, RCCL comm, fusion engine, PS
#     service, loader) and the ImageNet reader with -fsanitize=undefined into build_san/ (the
#     in-tree modules are untouched; device code is compiled as usual) and run the CPU tests
#     that drive that host code -- native PS over shared memory incl. worker failure, the
#     fusion engine over gloo, the mmap loader, TFRecord / JPEG decoding -- with the UBSan
#     runtime preloaded (AddressSanitizer cannot share a process with libtorch's memory map on
#     this kernel: "shadow memory range interleaves with an existing mapping").
#  2. ASan + UBSan natively: csrc/tests/io_core_test.cpp drives the torch-free reader core
#     (CRC32C, tf.Example parser, libjpeg decode + crop/pad, thread pool) including truncated
#     and corrupted inputs.
#  3. ThreadSanitizer natively: the same driver, whose pool section runs concurrent callers
#     that hand plain (non-atomic) buffers from the decode workers back to the caller.
#  4. ThreadSanitizer + ASan/UBSan natively over the concurrent runtime cores (a libtorch
#     Python process cannot run under TSan here): csrc/tests/fusion_core_test.cpp drives the
#     fusion engine's worker / watchdog / caller threads (runtime/fusion_core.h) with a fake
#     network completing collectives at random delays and a hung collective for the stall
#     inspector; csrc/tests/ps_protocol_test.cpp runs the PS service loop against 4 worker
#     threads over one control segment (runtime/ps_protocol.h), whose plain mailbox / receive
#     buffer traffic is ordered only by the protocol's release / acquire sequence numbers;
#     csrc/tests/launch_pool_test.cpp runs the graph group-launch pool (runtime/launch_pool.h).
#     TSan uses ROCm's clang runtime: GCC 11's libtsan does not intercept
#     pthread_cond_clockwait (std::condition_variable::wait_for) and reports a false "double lock".
#
#   bash scripts/sanitize_host.sh [pytest -k expression]
set -euo pipefail
cd "$(dirname "$0")/.."
OUT=${PDDL_SAN_DIR:-build_san}
mkdir -p "$OUT"
echo "== ASan+UBSan: io core"
# (libjpeg through a private rpath dir: /opt/conda/lib also holds an older libstdc++)
mkdir -p "$OUT/lib" && ln -sf /opt/conda/lib/libjpeg.so.9 "$OUT/lib/libjpeg.so.9"
g++ -std=c++17 -O1 -g -fsanitize=address,undefined -fno-omit-frame-pointer -I csrc -I /opt/conda/include \
    csrc/tests/io_core_test.cpp "$OUT/lib/libjpeg.so.9" -Wl,-rpath,"$PWD/$OUT/lib" -lpthread -o "$OUT/io_core_test"
ASAN_OPTIONS=detect_leaks=1:halt_on_error=1 UBSAN_OPTIONS=print_stacktrace=1:halt_on_error=1 "$OUT/io_core_test"
echo "== TSan: io core"
g++ -std=c++17 -O1 -g -fsanitize=thread -I csrc -I /opt/conda/include \
    csrc/tests/io_core_test.cpp "$OUT/lib/libjpeg.so.9" -Wl,-rpath,"$PWD/$OUT/lib" -lpthread -o "$OUT/io_core_tsan"
TSAN_OPTIONS=halt_on_error=1 "$OUT/io_core_tsan"
CLANG=${CLANG:-/opt/rocm/llvm/bin/clang++}
for t in fusion_core comm_watch ps_protocol launch_pool; do
  echo "== TSan: $t"
  "$CLANG" -std=c++17 -O1 -g -fsanitize=thread -I csrc "csrc/tests/${t}_test.cpp" -lpthread -o "$OUT/${t}_tsan"
  TSAN_OPTIONS=halt_on_error=1 "$OUT/${t}_tsan"
  echo "== ASan+UBSan: $t"
  g++ -std=c++17 -O1 -g -fsanitize=address,undefined -fno-omit-frame-pointer -I csrc "csrc/tests/${t}_test.cpp" \
      -lpthread -o "$OUT/${t}_asan"
  ASAN_OPTIONS=detect_leaks=1:halt_on_error=1 UBSAN_OPTIONS=print_stacktrace=1:halt_on_error=1 "$OUT/${t}_asan"
done
echo "== UBSan: runtime + reader under the CPU tests"
PDDL_SANITIZE=1 PDDL_BUILD_TEMP=/tmp/pddl_build_san python setup.py build_ext --build-lib "$OUT" \
    --build-temp /tmp/pddl_build_san > "$OUT/build.log" 2>&1 || { tail -30 "$OUT/build.log"; exit 1; }
rm -rf build
export PDDL_NATIVE_DIR="$PWD/$OUT"
export UBSAN_OPTIONS=print_stacktrace=1:halt_on_error=1
K=${1:-"native or records or tfrecord or folder or horovod"}
# (appends to any preload already in the environment instead of replacing it)
LD_PRELOAD="$(gcc -print-file-name=libubsan.so)${LD_PRELOAD:+ $LD_PRELOAD}" python -m pytest -x -q -m "not gpu" \
    -p no:cacheprovider tests/test_ps_checkpoint_cli.py tests/test_imagenet_io.py \
    tests/test_launch_data_callbacks.py tests/test_strategies_cpu.py -k "$K" 2>&1 | tee "$OUT/sanitize.log"
