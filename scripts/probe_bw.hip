// probe_bw.hip -- measurement tool (not shipped): HBM ceilings for the EC
// access pattern vs the engine's kernel and its tuning variants.
//   build: hipcc --offload-arch=gfx950 -O3 -std=c++17 scripts/probe_bw.hip \
//            -Ihdfs-native_amd/csrc -Lhdfs-native_amd/lib -lhdfs_ec_amd \
//            -Wl,-rpath,'$ORIGIN/../hdfs-native_amd/lib' -o scripts/probe_bw
// Output: one line per variant, GB/s of algorithmic bytes (read + write).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "../include/hdfs_ec_amd.h"

#define CK(x)                                                                              \
    do {                                                                                   \
        hipError_t e = (x);                                                                \
        if (e != hipSuccess) {                                                             \
            std::fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e)); \
            std::exit(1);                                                                  \
        }                                                                                  \
    } while (0)

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

__global__ void copy_kernel(const u32x4* __restrict__ in, u32x4* __restrict__ out, size_t n) {
    for (size_t i = blockIdx.x * size_t(blockDim.x) + threadIdx.x; i < n; i += size_t(gridDim.x) * blockDim.x)
        out[i] = in[i];
}

__global__ void fill_kernel(u32x4* p, size_t n, uint32_t seed) {
    for (size_t i = blockIdx.x * size_t(blockDim.x) + threadIdx.x; i < n; i += size_t(gridDim.x) * blockDim.x) {
        uint32_t x = uint32_t(i) * 2654435761u ^ seed;
        p[i] = u32x4{x, x * 3u + 1u, x ^ 0x5bd1e995u, x * 7u};
    }
}

// Same stripe walk as the engine, XOR only (no GF multiply): the memory
// ceiling of "K read streams + R write streams" at this tiling.
template <int K, int R>
__global__ __launch_bounds__(256) void xor_kernel(const uint8_t* __restrict__ in, uint8_t* __restrict__ out,
                                                  uint32_t chunks, uint32_t tps, uint32_t total, size_t cell) {
    for (uint32_t tile = blockIdx.x; tile < total; tile += gridDim.x) {
        uint32_t stripe = tile / tps, tcol = tile - stripe * tps;
        uint32_t col = tcol * 256 + threadIdx.x;
        if (col >= chunks) continue;
        const uint8_t* base = in + size_t(stripe) * K * cell + size_t(col) * 16;
        u32x4 x[K];
#pragma unroll
        for (int i = 0; i < K; i++) x[i] = *(const u32x4*)(base + i * cell);
        __builtin_amdgcn_sched_barrier(0);
        uint8_t* ob = out + size_t(stripe) * R * cell + size_t(col) * 16;
#pragma unroll
        for (int j = 0; j < R; j++) {
            u32x4 a = x[j];
#pragma unroll
            for (int i = 0; i < K; i++)
                if (i != j) a ^= x[i] + u32x4{uint32_t(j), 0, 0, 0};
            *(u32x4*)(ob + j * cell) = a;
        }
    }
}

template <typename F>
float time_ms(F&& f, int reps, hipStream_t s) {
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    f();
    f();
    std::vector<float> v;
    for (int r = 0; r < reps; r++) {
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

int main(int argc, char** argv) {
    const int K = argc > 3 ? std::atoi(argv[3]) : 6, R = argc > 4 ? std::atoi(argv[4]) : 3;
    const size_t cell = argc > 1 ? std::strtoull(argv[1], nullptr, 0) : (1u << 20);
    const size_t S = argc > 2 ? std::strtoull(argv[2], nullptr, 0) : 1024;
    const size_t pad = argc > 5 ? std::strtoull(argv[5], nullptr, 0) : 0;
    const size_t pitch = cell + pad;  // bytes between consecutive shards of a stripe
    const int reps = 10;
    uint8_t *din, *dout;
    CK(hipMalloc(&din, S * K * pitch));
    CK(hipMalloc(&dout, S * (K > R ? K : R) * pitch));
    hipStream_t s;
    CK(hipStreamCreate(&s));
    fill_kernel<<<4096, 256, 0, s>>>((u32x4*)din, S * K * pitch / 16, 1);
    CK(hipStreamSynchronize(s));
    const double algo = double((K + R) * cell * S);

    // plain copy with the same total bytes moved: read 4.5 cells + write 4.5 cells per stripe
    if (K == 6 && R == 3 && pad == 0 && argc <= 6) {
        size_t n = S * (K + R) * cell / 2 / 16;
        for (int grid : {1024, 2048, 4096, 8192}) {
            float ms = time_ms([&] { copy_kernel<<<grid, 256, 0, s>>>((const u32x4*)din, (u32x4*)dout, n); }, reps, s);
            std::printf("copy grid=%d: %.1f GB/s\n", grid, 2.0 * n * 16 / (ms * 1e-3) / 1e9);
        }
    }
    if (K == 6 && R == 3 && pad == 0 && argc <= 6) {
        uint32_t chunks = uint32_t(cell / 16), tps = (chunks + 255) / 256, total = uint32_t(tps * S);
        for (int bpc : {2, 4, 8}) {
            int grid = 256 * bpc;
            float ms = time_ms(
                [&] { xor_kernel<6, 3><<<grid, 256, 0, s>>>(din, dout, chunks, tps, total, cell); }, reps, s);
            std::printf("xor%d%d bpc=%d: %.1f GB/s\n", K, R, bpc, algo / (ms * 1e-3) / 1e9);
        }
    }
    hec_coder_t* c;
    if (hec_coder_create(K, R, 0, &c) != HEC_OK) {
        std::printf("coder: %s\n", hec_last_error());
        return 1;
    }
    const uint8_t* dp[32];
    size_t ds[32];
    uint8_t* pp[16];
    size_t ps[16];
    for (int i = 0; i < K; i++) {
        dp[i] = din + i * pitch;
        ds[i] = K * pitch;
    }
    for (int j = 0; j < R; j++) {
        pp[j] = dout + j * pitch;
        ps[j] = R * pitch;
    }
    const bool quick = pad != 0 || (argc > 6);
    struct V { int u, bs, bpc, pipe, map, grid, group; };
    const V vs[] = {{0, 0, 0, 0, 0, 0, 1}, {0, 0, 0, 0, 0, 0, 1}, {0, 0, 0, 0, 0, 0, 2}, {0, 0, 0, 0, 0, 0, 4},
                    {0, 0, 0, 0, 0, 0, 8}, {0, 0, 0, 0, 0, 0, 16}, {0, 0, 0, 0, 0, 0, 32}, {0, 0, 0, 0, 0, 0, 64},
                    {0, 0, 0, 0, 0, 0, 256}, {0, 0, 0, 0, 0, 0, 1024}, {0, 0, 0, 2, 0, 0, 1}, {0, 0, 0, 2, 0, 0, 16},
                    {0, 0, 0, 2, 0, 0, 64}, {0, 0, 0, 0, 0, 0, 1}};
    for (const V& v : vs) {
        hec_tune_set(8, v.group);
        hec_tune_set(1, v.u);
        hec_tune_set(4, v.bs);
        hec_tune_set(3, v.bpc);
        hec_tune_set(5, v.pipe);
        hec_tune_set(6, v.map);
        hec_tune_set(7, v.grid);
        float ms = time_ms([&] { hec_encode_device(c, dp, ds, pp, ps, cell, S, s); }, reps, s);
        std::printf("engine pipe=%d group=%d u=%d bs=%d bpc=%d: %.1f GB/s (%.3f ms)\n", v.pipe, v.group, v.u,
                    v.bs, v.bpc,
                    algo / (ms * 1e-3) / 1e9, ms);
    }
    hec_coder_destroy(c);
    return 0;
}
