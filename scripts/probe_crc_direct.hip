// probe_crc_direct.hip -- measurement tool (not shipped): does the chunk-CRC
// kernel need its LDS quarter image?
//
// The shipped kernel (checksum.hip, scheme 11) loads a wave's 8-KiB task with
// 8 coalesced 1-KiB loads, writes it into a per-wave LDS image and walks each
// lane's 128-B quarter back out of LDS.  The image costs LDS cycles (a
// ds_write_b128 moves 16 B/lane at ~79 B/clk/CU) in a kernel whose bound is
// the LDS (table lookups).  The "direct" variant has each lane load its own
// quarter (8 x 16 B at a 128-B lane stride: every instruction touches 64
// lines, each line is used whole over the 8 instructions) and checksum it
// from registers; no image, so more blocks fit a CU.
//   build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -Ihdfs-native_amd/csrc \
//            scripts/probe_crc_direct.hip -o scripts/probe_crc_direct
// Output: one line per variant, TB/s of checksummed bytes (median of rounds).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "checksum_device.hpp"
#include "checksum_tables.hpp"

#define CK(x)                                                                                     \
    do {                                                                                          \
        hipError_t e_ = (x);                                                                      \
        if (e_ != hipSuccess) {                                                                   \
            std::fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
            std::exit(1);                                                                         \
        }                                                                                         \
    } while (0)

using namespace hec;
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

__constant__ crc::Tables<crc::kCrc32c> kTab = crc::Tables<crc::kCrc32c>();

constexpr int SCHEME = 11;
using L = crcdev::TableLayout<SCHEME>;

// MODE 0: image (as shipped), 1: direct, 2: image, memory side only,
// 3: direct, memory side only.  NT: non-temporal loads.  The copy kernel
// below measures the same two layouts with stores (the fused kernel writes
// its parity cells in whichever layout it computes them).
template <int MODE, int BPC, bool NT>
__global__ __launch_bounds__(256, BPC) void crc_probe(const uint8_t* __restrict__ in, uint32_t* __restrict__ out,
                                                      uint64_t tasks) {
    constexpr int Q = 128, PITCH = Q + 16, STAGE = 64 * PITCH;
    constexpr bool IMG = MODE == 0 || MODE == 2;
    __shared__ uint32_t s_tab[L::kWords];
    __shared__ __attribute__((aligned(16))) uint8_t s_stage[IMG ? 4 * STAGE : 16];
    crcdev::stage_tables<SCHEME, 256, crc::kCrc32c>(s_tab, kTab);
    __syncthreads();
    const uint32_t kfinal = kTab.final512;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x / 64), lane = threadIdx.x & 63;
    const int qi = lane & 3;
    uint8_t* stage = s_stage + (IMG ? wave * STAGE : 0);
    const uint64_t step = uint64_t(gridDim.x) * 4;

    auto load = [&](uint64_t task, u32x4 (&v)[8]) {
        const uint8_t* base = in + task * 8192u;
#pragma unroll
        for (int t = 0; t < 8; t++) {
            const uint32_t off = IMG ? uint32_t(t) * 1024u + uint32_t(lane) * 16u : uint32_t(lane) * 128u + uint32_t(t) * 16u;
            const u32x4* p = reinterpret_cast<const u32x4*>(base + off);
            if constexpr (NT)
                v[t] = __builtin_nontemporal_load(p);
            else
                v[t] = *p;
        }
    };
    auto run = [&](uint64_t task, u32x4 (&v)[8], uint64_t next) {
        uint32_t val;
        if constexpr (IMG) {
#pragma unroll
            for (int t = 0; t < 8; t++) {
                const uint32_t off = uint32_t(t) * 1024u + uint32_t(lane) * 16u;
                *reinterpret_cast<u32x4*>(stage + (off / Q) * PITCH + (off % Q)) = v[t];
            }
            if (next < tasks) load(next, v);
            __builtin_amdgcn_wave_barrier();
            asm volatile("" ::: "memory");
            if constexpr (MODE == 0) {
                uint32_t r = crcdev::quarter_w11<true>(s_tab, stage + lane * PITCH);
                if (qi < 3) r = crcdev::shift_quarter<SCHEME>(s_tab, qi, r);
                val = r;
            } else {
                val = *reinterpret_cast<const uint32_t*>(stage + lane * PITCH);
            }
            __builtin_amdgcn_wave_barrier();
            asm volatile("" ::: "memory");
        } else {
            u32x4 w[8];
#pragma unroll
            for (int t = 0; t < 8; t++) w[t] = v[t];
            if (next < tasks) load(next, v);
            if constexpr (MODE == 1) {
                uint32_t r = 0;
#pragma unroll
                for (int t = 0; t < 8; t++) {
                    r = crcdev::step8_w11<true>(s_tab, r, w[t].x, w[t].y);
                    r = crcdev::step8_w11<true>(s_tab, r, w[t].z, w[t].w);
                }
                if (qi < 3) r = crcdev::shift_quarter<SCHEME>(s_tab, qi, r);
                val = r;
            } else {
                val = 0;
#pragma unroll
                for (int t = 0; t < 8; t++) val ^= w[t].x ^ w[t].y ^ w[t].z ^ w[t].w;
            }
        }
        val ^= __shfl_xor(val, 1);
        val ^= __shfl_xor(val, 2);
        if (qi == 0) out[task * 16 + (lane >> 2)] = __builtin_bswap32(val ^ kfinal);
    };
    uint64_t task = uint64_t(blockIdx.x) * 4 + wave;
    u32x4 va[8], vb[8];
    if (task < tasks) load(task, va);
    if (task + step < tasks) load(task + step, vb);
    while (task < tasks) {
        run(task, va, task + 2 * step);
        task += step;
        if (task >= tasks) break;
        run(task, vb, task + 2 * step);
        task += step;
    }
}

// DIRECT: lane l copies its 128-B quarter (8 x 16 B at a 128-B lane
// stride); else coalesced 1-KiB wave instructions.
template <bool DIRECT, bool NT>
__global__ __launch_bounds__(256) void copy_probe(const uint8_t* __restrict__ in, uint8_t* __restrict__ out,
                                                  uint64_t tasks) {
    const int wave = threadIdx.x / 64, lane = threadIdx.x & 63;
    for (uint64_t task = uint64_t(blockIdx.x) * 4 + wave; task < tasks; task += uint64_t(gridDim.x) * 4) {
        u32x4 v[8];
#pragma unroll
        for (int t = 0; t < 8; t++) {
            const uint32_t off = DIRECT ? uint32_t(lane) * 128u + uint32_t(t) * 16u : uint32_t(t) * 1024u + uint32_t(lane) * 16u;
            const u32x4* p = reinterpret_cast<const u32x4*>(in + task * 8192u + off);
            v[t] = NT ? __builtin_nontemporal_load(p) : *p;
        }
#pragma unroll
        for (int t = 0; t < 8; t++) {
            const uint32_t off = DIRECT ? uint32_t(lane) * 128u + uint32_t(t) * 16u : uint32_t(t) * 1024u + uint32_t(lane) * 16u;
            u32x4* p = reinterpret_cast<u32x4*>(out + task * 8192u + off);
            if constexpr (NT)
                __builtin_nontemporal_store(v[t], p);
            else
                *p = v[t];
        }
    }
}

__global__ void fill(uint32_t* p, size_t n) {
    for (size_t i = blockIdx.x * size_t(blockDim.x) + threadIdx.x; i < n; i += size_t(gridDim.x) * blockDim.x) {
        uint64_t x = i * 0x9E3779B97F4A7C15ull;
        x ^= x >> 29;
        x *= 0xBF58476D1CE4E5B9ull;
        p[i] = uint32_t(x >> 32);
    }
}

int main(int argc, char** argv) {
    const size_t bytes = size_t(argc > 1 ? atoi(argv[1]) : 2304) << 20;  // 9 x 1 MiB x 256 stripes
    const int rounds = argc > 2 ? atoi(argv[2]) : 5, reps = 10;
    const uint64_t tasks = bytes / 8192;
    int cus = 0;
    CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    uint8_t* in;
    uint32_t *out, *ref;
    CK(hipMalloc(&in, bytes));
    CK(hipMalloc(&out, tasks * 64));
    CK(hipMalloc(&ref, tasks * 64));
    fill<<<2048, 256>>>(reinterpret_cast<uint32_t*>(in), bytes / 4);
    struct V {
        const char* name;
        void (*fn)(const uint8_t*, uint32_t*, uint64_t);
        int bpc;
        bool check;
    };
    std::vector<V> vs = {
        {"image (shipped) 2/CU", crc_probe<0, 2, true>, 2, true},
        {"direct 2/CU", crc_probe<1, 2, false>, 2, true},
        {"direct 3/CU", crc_probe<1, 3, false>, 3, true},
        {"direct nt 2/CU", crc_probe<1, 2, true>, 2, true},
        {"image mem-only 2/CU", crc_probe<2, 2, true>, 2, false},
        {"direct mem-only 2/CU", crc_probe<3, 2, false>, 2, false},
        {"direct mem-only 3/CU", crc_probe<3, 3, false>, 3, false},
        {"direct nt mem-only 2/CU", crc_probe<3, 2, true>, 2, false},
    };
    {
        // copies: half the buffer in, half out; GB/s of read + write
        uint8_t* half = in + bytes / 2;
        const uint64_t ct = tasks / 2;
        void (*cf[4])(const uint8_t*, uint8_t*, uint64_t) = {copy_probe<false, true>, copy_probe<true, false>,
                                                             copy_probe<true, true>, copy_probe<false, false>};
        const char* cn[4] = {"copy coalesced nt", "copy direct", "copy direct nt", "copy coalesced"};
        std::vector<std::vector<float>> ctm(4);
        hipEvent_t c0, c1;
        CK(hipEventCreate(&c0));
        CK(hipEventCreate(&c1));
        for (int r = 0; r < rounds; r++)
            for (int v = 0; v < 4; v++) {
                hipLaunchKernelGGL(cf[v], dim3(cus * 8), dim3(256), 0, 0, in, half, ct);
                CK(hipEventRecord(c0));
                for (int i = 0; i < reps; i++) hipLaunchKernelGGL(cf[v], dim3(cus * 8), dim3(256), 0, 0, in, half, ct);
                CK(hipEventRecord(c1));
                CK(hipEventSynchronize(c1));
                float ms = 0;
                CK(hipEventElapsedTime(&ms, c0, c1));
                ctm[v].push_back(ms / reps);
            }
        for (int v = 0; v < 4; v++) {
            std::sort(ctm[v].begin(), ctm[v].end());
            const float ms = ctm[v][ctm[v].size() / 2];
            std::printf("%-26s median %.3f ms  %.2f TB/s read+write\n", cn[v], ms, double(bytes) / ms / 1e9);
        }
        fill<<<2048, 256>>>(reinterpret_cast<uint32_t*>(in), bytes / 4);
    }
    hipLaunchKernelGGL(vs[0].fn, dim3(cus * 2), dim3(256), 0, 0, in, ref, tasks);
    CK(hipDeviceSynchronize());
    std::vector<std::vector<float>> t(vs.size());
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    std::vector<uint32_t> h_ref(tasks * 16), h_out(tasks * 16);
    CK(hipMemcpy(h_ref.data(), ref, tasks * 64, hipMemcpyDeviceToHost));
    for (int r = 0; r < rounds; r++)
        for (size_t v = 0; v < vs.size(); v++) {
            const dim3 grid(cus * vs[v].bpc);
            hipLaunchKernelGGL(vs[v].fn, grid, dim3(256), 0, 0, in, out, tasks);
            CK(hipEventRecord(e0));
            for (int i = 0; i < reps; i++) hipLaunchKernelGGL(vs[v].fn, grid, dim3(256), 0, 0, in, out, tasks);
            CK(hipEventRecord(e1));
            CK(hipEventSynchronize(e1));
            float ms = 0;
            CK(hipEventElapsedTime(&ms, e0, e1));
            t[v].push_back(ms / reps);
            if (r == 0 && vs[v].check) {
                CK(hipMemcpy(h_out.data(), out, tasks * 64, hipMemcpyDeviceToHost));
                if (h_out != h_ref) {
                    std::printf("MISMATCH %s\n", vs[v].name);
                    return 1;
                }
            }
        }
    for (size_t v = 0; v < vs.size(); v++) {
        std::sort(t[v].begin(), t[v].end());
        const float ms = t[v][t[v].size() / 2];
        std::printf("%-26s median %.3f ms  %.2f TB/s  (min %.3f max %.3f)\n", vs[v].name, ms, bytes / ms / 1e9,
                    t[v].front(), t[v].back());
    }
    return 0;
}
