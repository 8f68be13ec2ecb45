// probe_shift64.hip -- measurement tool (not shipped): issue rate of
// v_lshrrev_b64 against v_lshrrev_b32 on gfx950, to price 64-bit shifts for
// the bit-sliced transposes (bitslice.hpp: one 64-bit shift could serve two
// delta swaps, the bits it carries across the dword boundary are masked out).
// Each lane runs independent chains (8 registers, 8 shifts per step); the
// kernel time per instruction gives the rate.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 scripts/probe_shift64.hip -o scripts/probe_shift64
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                                      \
    do {                                                                                           \
        hipError_t e_ = (x);                                                                       \
        if (e_ != hipSuccess) {                                                                    \
            std::fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
            std::exit(1);                                                                          \
        }                                                                                          \
    } while (0)

constexpr int kIters = 4096;

__global__ __launch_bounds__(256) void shifts32(uint32_t* out, uint32_t seed) {
    uint32_t r[16];
#pragma unroll
    for (int i = 0; i < 16; i++) r[i] = seed + threadIdx.x * 16 + i;
    for (int it = 0; it < kIters; it++) {
#pragma unroll
        for (int i = 0; i < 16; i++) asm volatile("v_lshrrev_b32 %0, 3, %0" : "+v"(r[i]));
    }
    uint32_t a = 0;
#pragma unroll
    for (int i = 0; i < 16; i++) a ^= r[i];
    out[blockIdx.x * 256 + threadIdx.x] = a;
}

__global__ __launch_bounds__(256) void shifts64(uint32_t* out, uint32_t seed) {
    uint64_t r[8];
#pragma unroll
    for (int i = 0; i < 8; i++) r[i] = (uint64_t(seed + threadIdx.x) << 32) | uint32_t(seed * 3 + i);
    for (int it = 0; it < kIters; it++) {
#pragma unroll
        for (int i = 0; i < 8; i++) asm volatile("v_lshrrev_b64 %0, 3, %0" : "+v"(r[i]));
    }
    uint64_t a = 0;
#pragma unroll
    for (int i = 0; i < 8; i++) a ^= r[i];
    out[blockIdx.x * 256 + threadIdx.x] = uint32_t(a ^ (a >> 32));
}

// v_bitop3 (the transposes' other op), for scale
__global__ __launch_bounds__(256) void bitop3s(uint32_t* out, uint32_t seed) {
    uint32_t r[16];
#pragma unroll
    for (int i = 0; i < 16; i++) r[i] = seed + threadIdx.x * 16 + i;
    const uint32_t m = seed | 0x0F0F0F0Fu;
    for (int it = 0; it < kIters; it++) {
#pragma unroll
        for (int i = 0; i < 16; i++) r[i] = __builtin_amdgcn_bitop3_b32(m, r[(i + 1) & 15], r[i], 0xCA);
    }
    uint32_t a = 0;
#pragma unroll
    for (int i = 0; i < 16; i++) a ^= r[i];
    out[blockIdx.x * 256 + threadIdx.x] = a;
}

template <typename F>
float time_it(F launch) {
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    launch();
    CK(hipDeviceSynchronize());
    float best = 1e30f;
    for (int rep = 0; rep < 5; rep++) {
        CK(hipEventRecord(a));
        launch();
        CK(hipEventRecord(b));
        CK(hipEventSynchronize(b));
        float t;
        CK(hipEventElapsedTime(&t, a, b));
        if (t < best) best = t;
    }
    return best;
}

int main() {
    hipDeviceProp_t p;
    CK(hipGetDeviceProperties(&p, 0));
    const int blocks = p.multiProcessorCount * 8;  // 8 waves per SIMD pair... 2 blocks x 4 waves per SIMD set
    uint32_t* out;
    CK(hipMalloc(&out, size_t(blocks) * 256 * 4));
    const double waves = blocks * 4.0;
    const float t32 = time_it([&] { shifts32<<<blocks, 256>>>(out, 7); });
    const float t64 = time_it([&] { shifts64<<<blocks, 256>>>(out, 7); });
    const float tb3 = time_it([&] { bitop3s<<<blocks, 256>>>(out, 7); });
    const double n = waves * kIters;  // per-lane-group instruction counts below are per wave
    std::printf("v_lshrrev_b32: %.3f ms for %.3g wave-instr (16 per step): %.3f ns per wave-instr chip-wide\n", t32,
                n * 16, t32 * 1e6 / (n * 16));
    std::printf("v_lshrrev_b64: %.3f ms for %.3g wave-instr (8 per step):  %.3f ns per wave-instr chip-wide\n", t64,
                n * 8, t64 * 1e6 / (n * 8));
    std::printf("v_bitop3_b32:  %.3f ms for %.3g wave-instr (16 per step): %.3f ns per wave-instr chip-wide\n", tb3,
                n * 16, tb3 * 1e6 / (n * 16));
    std::printf("b64 / b32 cost per instruction: %.2f (1 = full rate)\n", (t64 / 8) / (t32 / 16));
    CK(hipFree(out));
    return 0;
}
