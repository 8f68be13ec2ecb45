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
            if constexpr (R == 0) {  // read-only mix: a store that never happens keeps the loads
                if (acc[0] == 0xDEADBEEFu && acc[1] == 0x01234567u) *reinterpret_cast<u32x4*>(out) = acc;
            }
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

// write-only: the same tiles and order, R output cells per stripe, no loads
template <int R, int U, int BS, bool NT = true, bool DRAIN = true>
__global__ __launch_bounds__(BS) void skelw(uint8_t* __restrict__ out, uint32_t chunks, uint32_t tps, uint32_t total,
                                            uint32_t group) {
    constexpr uint32_t TILE = BS * U;
    const uint64_t cell = uint64_t(chunks) * 16;
    for (uint32_t tile = blockIdx.x; tile < total; tile += gridDim.x) {
        const uint32_t per = group * tps, g = tile / per, r = tile - g * per;
        const uint32_t tcol = r / group, stripe = g * group + (r - tcol * group);
        uint8_t* ob = out + uint64_t(stripe) * R * cell;
#pragma unroll
        for (int u = 0; u < U; u++)
#pragma unroll
            for (int j = 0; j < R; j++) {
                u32x4* dst = reinterpret_cast<u32x4*>(ob + j * cell + uint64_t(tcol * TILE + u * BS + threadIdx.x) * 16);
                const u32x4 v{tile, uint32_t(j), uint32_t(u), threadIdx.x};
                if constexpr (NT)
                    __builtin_nontemporal_store(v, dst);
                else
                    *dst = v;
            }
        if constexpr (DRAIN) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
}

template <int R, int U = 4, int BS = 256, bool NT = true, bool DRAIN = true>
void run_w(int cus, size_t cell, uint32_t stripes, int bpc = 1) {
    const uint32_t chunks = uint32_t(cell / 16), tps = chunks / (BS * U), total = tps * stripes;
    uint8_t* out;
    CK(hipMalloc(&out, size_t(stripes) * R * cell));
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    for (int w = 0; w < 20; w++) skelw<R, U, BS, NT, DRAIN><<<cus * bpc, BS>>>(out, chunks, tps, total, 4);
    CK(hipDeviceSynchronize());
    float best = 1e30f;
    for (int rep = 0; rep < 3; rep++) {
        CK(hipEventRecord(a));
        for (int it = 0; it < 20; it++) skelw<R, U, BS, NT, DRAIN><<<cus * bpc, BS>>>(out, chunks, tps, total, 4);
        CK(hipEventRecord(b));
        CK(hipEventSynchronize(b));
        float t;
        CK(hipEventElapsedTime(&t, a, b));
        best = std::min(best, t / 20);
    }
    const double bytes = double(R) * cell * stripes;
    std::printf("skeleton write-only %d cells %zu KiB x %u (U %d, %d threads, %d per CU, %s, %s): %.4f ms/launch "
                "(best of 3 x 20) %.1f GB/s = %.3f of 8 TB/s\n",
                R, cell >> 10, stripes, U, BS, bpc, NT ? "nt" : "default policy", DRAIN ? "drained" : "no drain", best,
                bytes / best / 1e6, bytes / best / 1e6 / 8000.0);
    CK(hipFree(out));
}

// Phase-aligned variant: the chip's 100 MHz real-time clock (s_memrealtime,
// common to every CU) splits time into periods of P ticks; loads are issued
// only in [0, pr) of a period (gate & 1) and stores only in [pr, P) (gate &
// 2), so the CUs' reads and writes reach DRAM in chip-wide phases instead of
// interleaved.  Each wait is bounded.
__device__ __forceinline__ void wait_window(uint32_t P, uint32_t lo, uint32_t hi) {
    for (int n = 0; n < 200000; n++) {
        const uint32_t t = uint32_t(__builtin_amdgcn_s_memrealtime() % P);
        if (t >= lo && t < hi) return;
        __builtin_amdgcn_s_sleep(1);
    }
}

template <int K, int R, int U, int BS>
__global__ __launch_bounds__(BS) void skelp(const uint8_t* __restrict__ in, uint8_t* __restrict__ out, uint32_t chunks,
                                            uint32_t tps, uint32_t total, uint32_t group, uint32_t P, uint32_t pr,
                                            uint32_t gate) {
    constexpr uint32_t TILE = BS * U;
    const uint64_t cell = uint64_t(chunks) * 16;
    for (uint32_t tile = blockIdx.x; tile < total; tile += gridDim.x) {
        const uint32_t per = group * tps, g = tile / per, r = tile - g * per;
        const uint32_t tcol = r / group, stripe = g * group + (r - tcol * group);
        const uint8_t* ib = in + uint64_t(stripe) * K * cell;
        uint8_t* ob = out + uint64_t(stripe) * R * cell;
        if (gate & 1) wait_window(P, 0, pr);
        u32x4 x[U][K];
#pragma unroll
        for (int u = 0; u < U; u++)
#pragma unroll
            for (int i = 0; i < K; i++)
                x[u][i] = __builtin_nontemporal_load(
                    reinterpret_cast<const u32x4*>(ib + i * cell + uint64_t(tcol * TILE + u * BS + threadIdx.x) * 16));
        __builtin_amdgcn_sched_barrier(0);
        u32x4 acc[U];
#pragma unroll
        for (int u = 0; u < U; u++) {
            acc[u] = x[u][0];
#pragma unroll
            for (int i = 1; i < K; i++) acc[u] ^= x[u][i];
        }
        __builtin_amdgcn_sched_barrier(0);
        if (gate & 2) wait_window(P, pr, P);
#pragma unroll
        for (int u = 0; u < U; u++)
#pragma unroll
            for (int j = 0; j < R; j++)
                __builtin_nontemporal_store(acc[u] + u32x4{uint32_t(j), 0, 0, 0},
                                            reinterpret_cast<u32x4*>(ob + j * cell +
                                                                      uint64_t(tcol * TILE + u * BS + threadIdx.x) * 16));
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
}

template <int K, int R>
void run_p(int cus, size_t cell, uint32_t stripes, uint32_t P, uint32_t pr, uint32_t gate) {
    constexpr int U = 4, BS = 256;
    const uint32_t chunks = uint32_t(cell / 16), tps = chunks / (BS * U), total = tps * stripes;
    uint8_t *in, *out;
    CK(hipMalloc(&in, size_t(stripes) * K * cell));
    CK(hipMalloc(&out, size_t(stripes) * R * cell));
    CK(hipMemset(in, 1, size_t(stripes) * K * cell));
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    for (int w = 0; w < 5; w++) skelp<K, R, U, BS><<<cus, BS>>>(in, out, chunks, tps, total, 4, P, pr, gate);
    CK(hipDeviceSynchronize());
    float best = 1e30f;
    for (int rep = 0; rep < 3; rep++) {
        CK(hipEventRecord(a));
        for (int it = 0; it < 10; it++) skelp<K, R, U, BS><<<cus, BS>>>(in, out, chunks, tps, total, 4, P, pr, gate);
        CK(hipEventRecord(b));
        CK(hipEventSynchronize(b));
        float t;
        CK(hipEventElapsedTime(&t, a, b));
        best = std::min(best, t / 10);
    }
    const double bytes = double(K + R) * cell * stripes;
    std::printf("phased RS(%d,%d) x %u P %u ticks, reads [0,%u) gate %u: %.4f ms/launch %.1f GB/s = %.3f of 8 TB/s\n", K,
                R, stripes, P, pr, gate, best, bytes / best / 1e6, bytes / best / 1e6 / 8000.0);
    CK(hipFree(in));
    CK(hipFree(out));
}

static bool g_contig = false;  // PROBE_CONTIG=1: physically contiguous allocations

template <int K, int R, bool MIXED = false, int U = 4, int BS = 256>
void run(int cus, size_t cell, uint32_t stripes, int bpc = 1, uint32_t group = 4) {
    const uint32_t chunks = uint32_t(cell / 16), tps = chunks / (BS * U), total = tps * stripes;
    uint8_t *in, *out;
    const unsigned fl = g_contig ? hipDeviceMallocContiguous : hipDeviceMallocDefault;
    CK(hipExtMallocWithFlags(reinterpret_cast<void**>(&in), size_t(stripes) * K * cell, fl));
    CK(hipExtMallocWithFlags(reinterpret_cast<void**>(&out), std::max<size_t>(size_t(stripes) * R * cell, 4096), fl));
    CK(hipMemset(in, 1, size_t(stripes) * K * cell));
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    for (int w = 0; w < 20; w++) skel<K, R, U, BS, MIXED><<<cus * bpc, BS>>>(in, out, chunks, tps, total, group);
    CK(hipDeviceSynchronize());
    std::vector<float> ms;
    for (int rep = 0; rep < 3; rep++) {
        CK(hipEventRecord(a));
        for (int it = 0; it < 20; it++) skel<K, R, U, BS, MIXED><<<cus * bpc, BS>>>(in, out, chunks, tps, total, group);
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
                " (mean writes %.2f)%s\n",
                K, R, MIXED ? " mixed e" : "", cell >> 10, stripes, best, bytes / best / 1e6, bytes / best / 1e6 / 8000.0,
                shards / stripes - K,
                (U == 4 && BS == 256 && bpc == 1 && group == 4)
                    ? ""
                    : (" [U " + std::to_string(U) + ", " + std::to_string(BS) + " threads, " + std::to_string(bpc) +
                       " per CU, group " + std::to_string(group) + "]")
                          .c_str());
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
    if (mode && std::string(mode) == "order") {
        // tile order (stripes interleaved per column group) and chunks per lane
        // for the read-heavy mixes of the mixed-pattern decodes
        for (int rep = 0; rep < 2; rep++) {
            for (uint32_t g : {1u, 2u, 4u, 8u, 16u, 64u}) run<10, 4, true>(cus, 1 << 20, 256, 1, g);
            run<10, 4, true, 2, 256>(cus, 1 << 20, 256, 2);
            run<10, 4, true, 2, 512>(cus, 1 << 20, 256, 1);
            run<10, 4, true, 8, 256>(cus, 1 << 20, 256, 1);
            run<10, 4, true, 4, 256>(cus, 1 << 20, 256, 2);
            run<10, 4, true>(cus, 1 << 20, 1024);
            for (uint32_t g : {1u, 4u, 16u}) run<6, 3, true>(cus, 1 << 20, 1024, 1, g);
            run<6, 3, true, 8, 256>(cus, 1 << 20, 1024, 1);
        }
        return 0;
    }
    if (mode && std::string(mode) == "occupancy") {
        // more waves per SIMD (the write-only stream gains 5 % at 4 blocks per CU)
        for (int rep = 0; rep < 2; rep++) {
            run<6, 3>(cus, 1 << 20, 1024);
            run<6, 3, false, 4, 256>(cus, 1 << 20, 1024, 2);
            run<6, 3, false, 4, 256>(cus, 1 << 20, 1024, 4);
            run<6, 3, false, 2, 256>(cus, 1 << 20, 1024, 2);
            run<6, 3, false, 2, 256>(cus, 1 << 20, 1024, 4);
            run<3, 2>(cus, 1 << 20, 1024);
            run<3, 2, false, 4, 256>(cus, 1 << 20, 1024, 4);
            run<3, 2, false, 2, 256>(cus, 1 << 20, 1024, 4);
            run<10, 4>(cus, 1 << 20, 256);
            run<10, 4, false, 2, 256>(cus, 1 << 20, 256, 4);
        }
        return 0;
    }
    if (mode && std::string(mode) == "writes") {
        // write-only stream shapes: store policy, drain, chunks per lane, block size, blocks per CU
        for (int rep = 0; rep < 2; rep++) {
            run_w<3>(cus, 1 << 20, 2048);
            run_w<3, 4, 256, false>(cus, 1 << 20, 2048);
            run_w<3, 4, 256, true, false>(cus, 1 << 20, 2048);
            run_w<3, 8, 256>(cus, 1 << 20, 2048);
            run_w<3, 4, 512>(cus, 1 << 20, 2048);
            run_w<3, 4, 256>(cus, 1 << 20, 2048, 2);
            run_w<3, 4, 256>(cus, 1 << 20, 2048, 4);
            run_w<3, 4, 256, true, false>(cus, 1 << 20, 2048, 4);
            run_w<1, 4, 256>(cus, 1 << 20, 6144);
        }
        return 0;
    }
    if (mode && std::string(mode) == "phase") {
        // RS(6,3) x 1024: about 640 ticks (6.4 us) per tile per CU at the skeleton's rate
        run<6, 3>(cus, 1 << 20, 1024);
        run_p<6, 3>(cus, 1 << 20, 1024, 640, 400, 0);  // gates off: the clock reads' cost alone
        for (uint32_t P : {160u, 320u, 640u, 1280u})
            for (uint32_t g : {2u, 3u}) run_p<6, 3>(cus, 1 << 20, 1024, P, P * 5 / 8, g);
        run_p<6, 3>(cus, 1 << 20, 1024, 640, 320, 3);
        run_p<6, 3>(cus, 1 << 20, 1024, 640, 480, 3);
        run<6, 3>(cus, 1 << 20, 1024);
        return 0;
    }
    if (mode && std::string(mode) == "pure") {
        // read-only and write-only streams on the same schedule, then the
        // coding mixes between them
        for (int rep = 0; rep < 2; rep++) {
            run<6, 0>(cus, 1 << 20, 1024);
            run<10, 0>(cus, 1 << 20, 512);
            run_w<6>(cus, 1 << 20, 1024);
            run_w<3>(cus, 1 << 20, 2048);
            run<6, 3>(cus, 1 << 20, 1024);
            run<1, 1>(cus, 1 << 20, 4096);
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
