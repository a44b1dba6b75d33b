#!/bin/bash
# Host-side AddressSanitizer + UBSan run of the CPU test suite against libzarrhip_asan.so:
# the planner, metadata validation, host CRC, blosc decompression (untrusted frames), the
# C-ABI entry points that need no GPU, and the JNI shim's bookkeeping under the fake JVM.  usage: zarr-java_amd/tools/run_host_asan.sh
set -eu
R=$(cd "$(dirname "$0")/../.." && pwd)
make -C "$R/zarr-java_amd" asan
# the JNI shim under the fake JVM (tests/jni), built with the same sanitizers against it
make -C "$R/tests/jni" asan
# the sanitizer builds are local artefacts: never shipped to the GPU box with the tree
trap 'rm -f "$R/zarr-java_amd/zarrhip/libzarrhip_asan.so" "$R/tests/jni/_build/libzh_jni_test_asan.so"' EXIT
RT=$(ls /opt/rocm/lib/llvm/lib/clang/*/lib/linux/libclang_rt.asan-x86_64.so | head -1)
cd "$R"
ZH_LIB_PATH="$R/zarr-java_amd/zarrhip/libzarrhip_asan.so" LD_PRELOAD="$RT" \
  ZH_JNI_TEST_LIB="$R/tests/jni/_build/libzh_jni_test_asan.so" \
  ASAN_OPTIONS=detect_leaks=0:abort_on_error=1 UBSAN_OPTIONS=print_stacktrace=1 \
  python3 -m pytest tests -q -m "not gpu" -p no:cacheprovider "$@"
