// probe_pattern.hip -- measurement tool (not shipped): which streaming
// pattern gets closest to HBM peak on MI355X for read/write mixes.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 scripts/probe_pattern.hip -o scripts/probe_pattern
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                                           \
    do {                                                                                                \
        hipError_t e = (x);                                                                             \
        if (e != hipSuccess) {                                                                          \
            std::fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e));       \
            std::exit(1);                                                                               \
        }                                                                                               \
    } while (0)

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

template <bool NT>
__device__ __forceinline__ u32x4 ld(const u32x4* p) {
    if constexpr (NT) return __builtin_nontemporal_load(p);
    else return *p;
}
template <bool NT>
__device__ __forceinline__ void st(u32x4* p, u32x4 v) {
    if constexpr (NT) __builtin_nontemporal_store(v, p);
    else *p = v;
}

// grid-stride copy, U 16-B chunks per lane per iteration (contiguous per wave)
template <int U, bool NTL, bool NTS>
__global__ __launch_bounds__(256) void copy_k(const u32x4* __restrict__ in, u32x4* __restrict__ out, size_t n) {
    const size_t step = size_t(gridDim.x) * 256 * U;
    for (size_t base = size_t(blockIdx.x) * 256 * U; base < n; base += step) {
        u32x4 v[U];
#pragma unroll
        for (int u = 0; u < U; u++) {
            size_t i = base + u * 256 + threadIdx.x;
            if (i < n) v[u] = ld<NTL>(in + i);
        }
#pragma unroll
        for (int u = 0; u < U; u++) {
            size_t i = base + u * 256 + threadIdx.x;
            if (i < n) st<NTS>(out + i, v[u]);
        }
    }
}

// copy with BS threads per block
template <int U, bool NTL, bool NTS, int BS>
__global__ __launch_bounds__(BS) void copyb_k(const u32x4* __restrict__ in, u32x4* __restrict__ out, size_t n) {
    const size_t step = size_t(gridDim.x) * BS * U;
    for (size_t base = size_t(blockIdx.x) * BS * U; base < n; base += step) {
        u32x4 v[U];
#pragma unroll
        for (int u = 0; u < U; u++) {
            size_t i = base + u * BS + threadIdx.x;
            if (i < n) v[u] = ld<NTL>(in + i);
        }
#pragma unroll
        for (int u = 0; u < U; u++) {
            size_t i = base + u * BS + threadIdx.x;
            if (i < n) st<NTS>(out + i, v[u]);
        }
    }
}

// copy where each block owns one contiguous range (no grid stride)
template <int U, bool NTL, bool NTS>
__global__ __launch_bounds__(256) void copyr_k(const u32x4* __restrict__ in, u32x4* __restrict__ out, size_t n) {
    const size_t per = (n + gridDim.x - 1) / gridDim.x;
    const size_t b0 = blockIdx.x * per, b1 = min(n, b0 + per);
    for (size_t base = b0; base < b1; base += 256 * U) {
        u32x4 v[U];
#pragma unroll
        for (int u = 0; u < U; u++) {
            size_t i = base + u * 256 + threadIdx.x;
            if (i < b1) v[u] = ld<NTL>(in + i);
        }
#pragma unroll
        for (int u = 0; u < U; u++) {
            size_t i = base + u * 256 + threadIdx.x;
            if (i < b1) st<NTS>(out + i, v[u]);
        }
    }
}

template <int U, bool NTL>
__global__ __launch_bounds__(256) void read_k(const u32x4* __restrict__ in, u32x4* __restrict__ out, size_t n) {
    const size_t step = size_t(gridDim.x) * 256 * U;
    u32x4 acc = {0, 0, 0, 0};
    for (size_t base = size_t(blockIdx.x) * 256 * U; base < n; base += step) {
#pragma unroll
        for (int u = 0; u < U; u++) {
            size_t i = base + u * 256 + threadIdx.x;
            if (i < n) acc ^= ld<NTL>(in + i);
        }
    }
    if (acc.x == 0x12345678u) out[threadIdx.x] = acc;
}

template <int U, bool NTS>
__global__ __launch_bounds__(256) void write_k(u32x4* __restrict__ out, size_t n) {
    const size_t step = size_t(gridDim.x) * 256 * U;
    for (size_t base = size_t(blockIdx.x) * 256 * U; base < n; base += step) {
#pragma unroll
        for (int u = 0; u < U; u++) {
            size_t i = base + u * 256 + threadIdx.x;
            if (i < n) st<NTS>(out + i, u32x4{uint32_t(i), 1, 2, 3});
        }
    }
}

// 6-read/3-write stripe pattern; tile = 256*U chunks of one stripe; ORDER 0 =
// grid-stride over tiles, 1 = contiguous tile range per block.
template <int U, bool NTL, bool NTS, int ORDER>
__global__ __launch_bounds__(256) void ec_k(const uint8_t* __restrict__ in, uint8_t* __restrict__ out,
                                            uint32_t chunks, uint32_t tps, uint32_t total, size_t cell) {
    constexpr int K = 6, R = 3;
    uint32_t t0, t1, ts;
    if (ORDER == 0) {
        t0 = blockIdx.x; t1 = total; ts = gridDim.x;
    } else {
        uint32_t per = (total + gridDim.x - 1) / gridDim.x;
        t0 = blockIdx.x * per; t1 = min(total, t0 + per); ts = 1;
    }
    for (uint32_t tile = t0; tile < t1; tile += ts) {
        uint32_t stripe = tile / tps, tcol = tile - stripe * tps;
        u32x4 x[U][K];
#pragma unroll
        for (int u = 0; u < U; u++) {
            uint32_t col = tcol * 256 * U + u * 256 + threadIdx.x;
            const uint8_t* b = in + size_t(stripe) * K * cell + size_t(col) * 16;
#pragma unroll
            for (int i = 0; i < K; i++) x[u][i] = ld<NTL>((const u32x4*)(b + i * cell));
        }
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int u = 0; u < U; u++) {
            uint32_t col = tcol * 256 * U + u * 256 + threadIdx.x;
            uint8_t* ob = out + size_t(stripe) * R * cell + size_t(col) * 16;
#pragma unroll
            for (int j = 0; j < R; j++) {
                u32x4 a = x[u][j] ^ x[u][j + 3];
                a ^= x[u][(j + 1) % 6] + u32x4{1u, 0, 0, 0};
                st<NTS>((u32x4*)(ob + j * cell), a);
            }
        }
    }
}

template <typename F>
float time_ms(F&& f, hipStream_t s) {
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    f();
    f();
    std::vector<float> v;
    for (int r = 0; r < 8; r++) {
        CK(hipEventRecord(a, s));
        f();
        CK(hipEventRecord(b, s));
        CK(hipEventSynchronize(b));
        float ms;
        CK(hipEventElapsedTime(&ms, a, b));
        v.push_back(ms);
    }
    std::sort(v.begin(), v.end());
    return v[v.size() / 2];
}

int main() {
    const size_t cell = 1 << 20, S = 1024;
    const size_t bytes = S * 6 * cell;  // 6 GiB
    uint8_t *din, *dout;
    CK(hipMalloc(&din, bytes));
    CK(hipMalloc(&dout, bytes));
    CK(hipMemset(din, 0x5a, bytes));
    hipStream_t s;
    CK(hipStreamCreate(&s));
    const size_t n = bytes / 16;
    const size_t n_copy = S * 9 * cell / 2 / 16;  // 4.5 GiB each way

    const uint32_t chunks = cell / 16;
#define EC(U, NL, NS, O)                                                                                       \
    for (int g : {256}) {                                                                                      \
        uint32_t tps = chunks / (256 * U), total = tps * S;                                                    \
        float ms = time_ms([&] { ec_k<U, NL, NS, O><<<g, 256, 0, s>>>(din, dout, chunks, tps, total, cell); }, s); \
        std::printf("ec63 U=%d ntl=%d nts=%d order=%d grid=%d: %.1f GB/s\n", U, NL, NS, O, g,                 \
                    9.0 * cell * S / ms / 1e6);                                                                \
    }
    EC(4, 1, 1, 0) EC(4, 1, 0, 0) EC(4, 0, 1, 0) EC(4, 0, 0, 0) EC(4, 1, 1, 0) EC(4, 1, 0, 0)
    EC(2, 1, 1, 0) EC(2, 1, 0, 0)
    return 0;
}
