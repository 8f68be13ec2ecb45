#!/bin/bash
# Host-side ASan/LSan build of the C ABI (ec_capi.cpp sanitized; the kernel
# objects linked as built) and a run of tests/cpp/asan_capi.c on the CPU.
# Usage: asan_host.sh OUTDIR   (needs hdfs-native_amd/build/*.o: run make first)
set -eo pipefail
out=${1:-/tmp/hec_asan}
root=$(cd "$(dirname "$0")/.." && pwd)
mkdir -p "$out"
HIPCC=/opt/rocm/bin/hipcc
CLANG=/opt/rocm/lib/llvm/bin/clang
$HIPCC -O1 -g -std=c++17 -fPIC --offload-arch=gfx950 -Xarch_host -fsanitize=address \
    -Xarch_host -fno-omit-frame-pointer -x hip -c "$root/hdfs-native_amd/csrc/ec_capi.cpp" -o "$out/capi_asan.o"
# the host small-row routine (AVX-512BW+GFNI / AVX2 / scalar) sanitized too,
# with clang: its ASan instruments AVX-512 masked loads lane by lane (GCC 11's
# does not, and faults on the masked tail)
/opt/rocm/lib/llvm/bin/clang++ -O1 -g -std=c++17 -fPIC -fsanitize=address -fno-omit-frame-pointer \
    -c "$root/hdfs-native_amd/csrc/host_gf.cpp" -o "$out/host_gf_asan.o"
$HIPCC -shared -fPIC --offload-arch=gfx950 -fno-gpu-sanitize -fsanitize=address -o "$out/libhec_asan.so" "$out/capi_asan.o" \
    "$out/host_gf_asan.o" "$root/hdfs-native_amd/build/ec_kernels.o" "$root/hdfs-native_amd/build/ec_fused.o" \
    "$root/hdfs-native_amd/build/checksum.o" "$root/hdfs-native_amd/build/tuning.o"
$CLANG -g -fsanitize=address -I"$root/include" "$root/tests/cpp/asan_capi.c" -o "$out/asan_capi" \
    -L"$out" -lhec_asan -Wl,-rpath,"$out" -Wl,-rpath,/opt/rocm/lib
ASAN_OPTIONS=detect_leaks=1 "$out/asan_capi"
