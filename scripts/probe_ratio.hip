// probe_ratio.hip -- measurement tool (not shipped): the HBM rate of the
// engine's streaming skeleton with the GF math taken out, per read:write mix.
// Same layout and schedule as gf_matmul_v16 (ec_kernels.hip): stripes of k
// input cells and m output cells ([stripe][k][cell] / [stripe][m][cell]),
// 16 B per lane per shard, U = 4 chunks per lane, 256-thread blocks, one
// block per CU, 4-stripe column-interleaved tile order, non-temporal loads
// and stores, stores drained before the next tile's loads.  The "math" is
// out_j = XOR_i in_i (K - 1 XORs per dword, shared by the outputs), so the
// rate is the layout's ceiling for that (k, m) on this box.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 scripts/probe_ratio.hip -o scripts/probe_ratio
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <string>
#include <vector>

#define CK(x)                                                                                      \
    do {                                                                                           \
        hipError_t e_ = (x);                                                                       \
        if (e_ != hipSuccess) {                                                                    \
            std::fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
            std::exit(1);                                                                          \
        }                                                                                          \
    } while (0)

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

// e of a stripe in the mixed mode: 1 + (hash % R), as a per-stripe random
// erasure count of 1..R (stores of rows past e skipped, as gf_decode_mixed)
__host__ __device__ inline uint32_t stripe_e(uint32_t s, int R) {
    uint32_t h = s * 0x9E3779B1u;
    h ^= h >> 15;
    h *= 0x85EBCA77u;
    h ^= h >> 13;
    return 1u + h % uint32_t(R);
}

template <int K, int R, int U, int BS, bool MIXED = false>
__global__ __launch_bounds__(BS) void skel(const uint8_t* __restrict__ in, uint8_t* __restrict__ out, uint32_t chunks,
                                           uint32_t tps, uint32_t total, uint32_t group) {
    constexpr uint32_t TILE = BS * U;
    const uint64_t cell = uint64_t(chunks) * 16;
    for (uint32_t tile = blockIdx.x; tile < total; tile += gridDim.x) {
        const uint32_t per = group * tps, g = tile / per, r = tile - g * per;
        const uint32_t tcol = r / group, stripe = g * group + (r - tcol * group);
        const uint8_t* ib = in + uint64_t(stripe) * K * cell;
        uint8_t* ob = out + uint64_t(stripe) * R * cell;
        const int e = MIXED ? int(__builtin_amdgcn_readfirstlane(int(stripe_e(stripe, R)))) : R;
        u32x4 x[U][K];
#pragma unroll
        for (int u = 0; u < U; u++)
#pragma unroll
            for (int i = 0; i < K; i++)
                x[u][i] = __builtin_nontemporal_load(
                    reinterpret_cast<const u32x4*>(ib + i * cell + uint64_t(tcol * TILE + u * BS + threadIdx.x) * 16));
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int u = 0; u < U; u++) {
            u32x4 acc = x[u][0];
#pragma unroll
            for (int i = 1; i < K; i++) acc ^= x[u][i];
#pragma unroll
            for (int j = 0; j < R; j++) {
                if (MIXED && j >= e) break;
                __builtin_nontemporal_store(acc + u32x4{uint32_t(j), 0, 0, 0}, reinterpret_cast<u32x4*>(
                                                ob + j * cell + uint64_t(tcol * TILE + u * BS + threadIdx.x) * 16));
            }
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
}

static bool g_contig = false;  // PROBE_CONTIG=1: physically contiguous allocations

template <int K, int R, bool MIXED = false>
void run(int cus, size_t cell, uint32_t stripes) {
    constexpr int U = 4, BS = 256;
    const uint32_t chunks = uint32_t(cell / 16), tps = chunks / (BS * U), total = tps * stripes;
    uint8_t *in, *out;
    const unsigned fl = g_contig ? hipDeviceMallocContiguous : hipDeviceMallocDefault;
    CK(hipExtMallocWithFlags(reinterpret_cast<void**>(&in), size_t(stripes) * K * cell, fl));
    CK(hipExtMallocWithFlags(reinterpret_cast<void**>(&out), size_t(stripes) * R * cell, fl));
    CK(hipMemset(in, 1, size_t(stripes) * K * cell));
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    for (int w = 0; w < 20; w++) skel<K, R, U, BS, MIXED><<<cus, BS>>>(in, out, chunks, tps, total, 4);
    CK(hipDeviceSynchronize());
    std::vector<float> ms;
    for (int rep = 0; rep < 3; rep++) {
        CK(hipEventRecord(a));
        for (int it = 0; it < 20; it++) skel<K, R, U, BS, MIXED><<<cus, BS>>>(in, out, chunks, tps, total, 4);
        CK(hipEventRecord(b));
        CK(hipEventSynchronize(b));
        float t;
        CK(hipEventElapsedTime(&t, a, b));
        ms.push_back(t / 20);
    }
    const float best = *std::min_element(ms.begin(), ms.end());
    double shards = 0;
    for (uint32_t s = 0; s < stripes; s++) shards += K + (MIXED ? stripe_e(s, R) : R);
    const double bytes = shards * cell;
    std::printf("skeleton RS(%d,%d)%s %zu KiB x %u: %.4f ms/launch (best of 3 x 20) %.1f GB/s = %.3f of 8 TB/s"
                " (mean writes %.2f)\n",
                K, R, MIXED ? " mixed e" : "", cell >> 10, stripes, best, bytes / best / 1e6, bytes / best / 1e6 / 8000.0,
                shards / stripes - K);
    CK(hipFree(in));
    CK(hipFree(out));
}

int main() {
    hipDeviceProp_t p;
    CK(hipGetDeviceProperties(&p, 0));
    const int cus = p.multiProcessorCount;
    const char* mode = std::getenv("PROBE_MODE");
    g_contig = std::getenv("PROBE_CONTIG") && std::atoi(std::getenv("PROBE_CONTIG")) == 1;
    if (mode && std::string(mode) == "mixed") {
        // per-stripe erasure counts 1..R against the fixed mixes of the same mean
        for (int rep = 0; rep < 2; rep++) {
            run<10, 4, true>(cus, 1 << 20, 256);
            run<10, 2>(cus, 1 << 20, 256);
            run<10, 3>(cus, 1 << 20, 256);
            run<6, 3, true>(cus, 1 << 20, 1024);
            run<6, 2>(cus, 1 << 20, 1024);
            run<3, 2, true>(cus, 1 << 20, 1024);
        }
        return 0;
    }
    if (mode && std::string(mode) == "footprint") {
        // RS(10,4) at growing stripe counts (footprint 3.5 .. 28 GiB), warmed up first
        run<10, 4>(cus, 1 << 20, 256);
        for (uint32_t s : {256u, 512u, 1024u, 2048u, 256u}) run<10, 4>(cus, 1 << 20, s);
        return 0;
    }
    run<1, 1>(cus, 1 << 20, 4096);
    run<3, 2>(cus, 1 << 20, 1024);
    run<6, 3>(cus, 1 << 20, 1024);
    run<10, 4>(cus, 1 << 20, 256);
    run<10, 4>(cus, 1 << 20, 1024);
    run<3, 2>(cus, 1 << 20, 1024);
    run<6, 3>(cus, 1 << 20, 1024);
    // the read:write mixes of the mixed-pattern decodes (1..m data shards lost
    // per stripe: e averages 2.43 at k = 10 and 2.0 at k = 6)
    run<10, 2>(cus, 1 << 20, 256);
    run<10, 3>(cus, 1 << 20, 256);
    run<6, 2>(cus, 1 << 20, 1024);
    return 0;
}
