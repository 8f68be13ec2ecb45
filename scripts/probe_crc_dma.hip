// probe_crc_dma.hip -- measurement tool (not shipped): CRC32C per 512-B chunk
// of 9 x 1 MiB x S cells (the encode + CRC leg's k+m cells), the product
// kernel (hec_crc32c_device) against LDS-DMA variants of the same algorithm
// (the fold + a lookup tail + nibble shift tables, checksum_device.hpp).
//
// LDS-DMA variant: each wave owns NST landing stages of 8 KiB (one task = 16
// chunks of one cell); global_load_lds_dwordx4 lands a task's 8 KiB straight
// in LDS (no staging VGPRs, no ds_write pass), NST-1 tasks in flight while one
// is checksummed.  The landing image is lane-linear (64 x 16 B per
// instruction), so the per-lane quarter walk (lane Q reads the 128 B of
// quarter Q) is made bank-conflict free by an XOR swizzle on the SOURCE
// address: piece i of quarter Q lands in slot 8Q + (i ^ ((Q >> 1) & 7)); each
// instruction still reads one contiguous 1 KiB (lanes permuted inside each
// 128-B line).  TAIL = 1: the fold's 32-B tail through slicing-by-8 tables
// (8 KiB), 2: through the 11-bit tables (40 KiB), 0: no CRC math (the
// schedule's memory ceiling; sums wrong, not checked).
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 scripts/probe_crc_dma.hip -o scripts/probe_crc_dma \
//       -Lhdfs-native_amd/lib -lhdfs_ec_amd -Wl,-rpath,'$ORIGIN/../hdfs-native_amd/lib'
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "../hdfs-native_amd/csrc/checksum_device.hpp"
#include "../hdfs-native_amd/csrc/checksum_tables.hpp"
#include "../include/hdfs_ec_amd.h"

#define CK(x)                                                                                      \
    do {                                                                                           \
        hipError_t e_ = (x);                                                                       \
        if (e_ != hipSuccess) {                                                                    \
            std::fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
            std::exit(1);                                                                          \
        }                                                                                          \
    } while (0)

namespace cd = hec::crcdev;
typedef uint32_t v4u __attribute__((ext_vector_type(4)));

__constant__ hec::crc::Tables<hec::crc::kCrc32c> kT = hec::crc::Tables<hec::crc::kCrc32c>();

constexpr uint32_t kCell = 1u << 20, kGroups = kCell / 8192, kNck = kCell / 512;

template <int TAIL>
struct TabW {
    static constexpr int kMain = TAIL == 2 ? 10240 : TAIL == 1 ? 2048 : 0;
    static constexpr int kWords = kMain + 384;  // + shift_nib[3][8][16]
};

// the fold of checksum_device.hpp quarter_fold, on registers
__device__ __forceinline__ void fold24(uint32_t (&w)[32]) {
    using F = cd::Fold;
#pragma unroll
    for (int i = 2; i < 32; i++) {
        uint32_t acc = w[i], pend = 0;
        bool has = false;
#pragma unroll
        for (int o = 0; o < F::kN; o++) {
            const int hi = i - F::q[o], lo = hi - 1;
            const bool h = hi >= 0 && hi < F::kDwords, l = lo >= 0 && lo < F::kDwords;
            if (!h && !l) continue;
            const uint32_t c = h && l ? __builtin_amdgcn_alignbit(w[hi], w[lo], 32 - F::s[o])
                               : h    ? w[hi] << F::s[o]
                                      : w[lo] >> (32 - F::s[o]);
            if (has) {
                acc = cd::x3(acc, pend, c);
                has = false;
            } else {
                pend = c;
                has = true;
            }
        }
        w[i] = has ? acc ^ pend : acc;
    }
}

// cell (stripe s, shard i) at base[i] + s * stride[i]; sums [s][9][chunk]
struct Cells {
    const uint8_t* base[9];
    uint64_t stride[9];
};

template <int WAVES, int NST, int TAIL>
__global__ __launch_bounds__(WAVES * 64) void crc_dma(Cells cs, uint32_t ncells, uint32_t* __restrict__ out,
                                                      uint32_t inter) {
    using TW = TabW<TAIL>;
    constexpr int STAGE = 8192;
    // one LDS object: stages then tables
    __shared__ __attribute__((aligned(16))) uint8_t s_mem[WAVES * NST * STAGE + TW::kWords * 4];
    uint32_t* s_tab = reinterpret_cast<uint32_t*>(s_mem + WAVES * NST * STAGE);
    if constexpr (TAIL == 2) {
        constexpr int off[6] = {0, 2048, 4096, 5120, 7168, 9216}, len[6] = {2048, 2048, 1024, 2048, 2048, 1024};
#pragma unroll
        for (int f = 0; f < 6; f++)
            for (int t = threadIdx.x; t < len[f]; t += WAVES * 64) s_tab[off[f] + t] = kT.w11[f][t];
    } else if constexpr (TAIL == 1) {
        for (int t = threadIdx.x; t < 2048; t += WAVES * 64) s_tab[t] = (&kT.slice[0][0])[t];
    }
    for (int t = threadIdx.x; t < 384; t += WAVES * 64) s_tab[TW::kMain + t] = (&kT.shift_nib[0][0][0])[t];
    __syncthreads();
    const uint32_t kfinal = kT.final512;

    const int wave = __builtin_amdgcn_readfirstlane(int(threadIdx.x / 64)), lane = threadIdx.x & 63;
    uint8_t* st = s_mem + wave * NST * STAGE;
    const uint32_t tasks = ncells * kGroups;
    const uint32_t nw = gridDim.x * WAVES;
    uint32_t task = blockIdx.x * WAVES + wave;

    // instruction t, lane l: quarter q = 8t + l/8, piece (l%8) ^ ((q>>1)&7)
    uint32_t loff[8];
#pragma unroll
    for (int t = 0; t < 8; t++) {
        const uint32_t q = 8u * t + uint32_t(lane) / 8u;
        loff[t] = 1024u * t + 128u * (uint32_t(lane) / 8u) + 16u * ((uint32_t(lane) & 7u) ^ ((q >> 1) & 7u));
    }
    // task order: `inter` cells interleaved -- consecutive tasks take group g
    // of cells c0 .. c0+inter-1, then group g+1 (inter = 1: cell-major)
    auto cell_of = [&](uint32_t tk, uint32_t& cell, uint32_t& g) {
        const uint32_t span = inter * kGroups, blk = tk / span, r = tk - blk * span;
        cell = blk * inter + r % inter;
        g = r / inter;
    };
    auto issue = [&](uint32_t tk, int s) {
        uint32_t cell, g;
        cell_of(tk, cell, g);
        const uint32_t stripe = cell / 9u, shard = cell % 9u;
        const uint8_t* src = cs.base[shard] + uint64_t(stripe) * cs.stride[shard] + uint64_t(g) * 8192u;
#pragma unroll
        for (int t = 0; t < 8; t++)
            __builtin_amdgcn_global_load_lds(reinterpret_cast<const void*>(src + loff[t]),
                                             (__attribute__((address_space(3))) void*)(st + s * STAGE + t * 1024),
                                             16, 0, 2 /* nt */);
    };
#pragma unroll
    for (int s = 0; s < NST - 1; s++)
        if (task + uint32_t(s) * nw < tasks) issue(task + uint32_t(s) * nw, s);
    const int qi = lane & 3, c = lane >> 2;
    int s = 0;
    for (int k = 0; task < tasks; k++, task += nw) {
        const uint32_t nt = task + uint32_t(NST - 1) * nw;
        __builtin_amdgcn_sched_barrier(0);
        if (nt < tasks) {
            issue(nt, s == 0 ? NST - 1 : s - 1);
            // younger than this task's 8 DMAs: the NST-1 newer tasks' DMAs and,
            // from iteration NST-1 on, the NST-1 sums stores issued since
            if (k >= NST - 1)
                asm volatile("s_waitcnt vmcnt(%0)" ::"n"(9 * (NST - 1)) : "memory");
            else
                asm volatile("s_waitcnt vmcnt(%0)" ::"n"(8 * (NST - 1)) : "memory");
        } else {
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
        __builtin_amdgcn_sched_barrier(0);
        const uint8_t* sb = st + s * STAGE;
        uint32_t w[32];
#pragma unroll
        for (int i = 0; i < 8; i++) {
            const v4u v = *reinterpret_cast<const v4u*>(sb + 16 * (lane * 8 + (i ^ ((lane >> 1) & 7))));
            w[4 * i] = v.x, w[4 * i + 1] = v.y, w[4 * i + 2] = v.z, w[4 * i + 3] = v.w;
        }
        uint32_t r = 0;
        if constexpr (TAIL == 0) {
#pragma unroll
            for (int i = 0; i < 32; i++) r ^= w[i];
        } else {
            fold24(w);
#pragma unroll
            for (int i = 24; i < 32; i += 2) {
                if constexpr (TAIL == 2)
                    r = cd::step8_w11<true>(s_tab, r, w[i], w[i + 1]);
                else
                    r = cd::step8<true>(reinterpret_cast<const uint32_t(*)[256]>(s_tab), r, w[i], w[i + 1]);
            }
            if (qi < 3) r = cd::apply_shift_nib(reinterpret_cast<const uint32_t(*)[8][16]>(s_tab + TW::kMain)[qi], r);
        }
        r ^= __shfl_xor(r, 1);
        r ^= __shfl_xor(r, 2);
        uint32_t cell, g;
        cell_of(task, cell, g);
        if (qi == 0) out[uint64_t(cell) * kNck + g * 16 + c] = __builtin_bswap32(r ^ kfinal);
        s = s == NST - 1 ? 0 : s + 1;
    }
}

// The product's register-staged kernel (checksum.hip checksum_chunks512<
// CRC32C, fold, one task of prefetch>: 256 threads, 2 blocks per CU, a
// padded 9-KiB image per wave) restated over Cells with the task order
// interleaved over `inter` cells, as crc_dma.
__global__ __launch_bounds__(256) void crc_reg(Cells cs, uint32_t ncells, uint32_t* __restrict__ out,
                                               uint32_t inter) {
    constexpr int Q = 128, PITCH = Q + 16, STAGE = 64 * PITCH;
    __shared__ uint32_t s_tab[10240 + 384];
    __shared__ __attribute__((aligned(16))) uint8_t s_stage[4 * STAGE];
    {
        constexpr int off[6] = {0, 2048, 4096, 5120, 7168, 9216}, len[6] = {2048, 2048, 1024, 2048, 2048, 1024};
#pragma unroll
        for (int f = 0; f < 6; f++)
            for (int t = threadIdx.x; t < len[f]; t += 256) s_tab[off[f] + t] = kT.w11[f][t];
        for (int t = threadIdx.x; t < 384; t += 256) s_tab[10240 + t] = (&kT.shift_nib[0][0][0])[t];
    }
    __syncthreads();
    const uint32_t kfinal = kT.final512;
    const int wave = __builtin_amdgcn_readfirstlane(int(threadIdx.x / 64)), lane = threadIdx.x & 63;
    const int qi = lane & 3, c = lane >> 2;
    uint8_t* stage = s_stage + wave * STAGE;
    const uint32_t tasks = ncells * kGroups, step = gridDim.x * 4;
    auto cell_of = [&](uint32_t tk, uint32_t& cell, uint32_t& g) {
        const uint32_t span = inter * kGroups, blk = tk / span, r = tk - blk * span;
        cell = blk * inter + r % inter;
        g = r / inter;
    };
    auto load = [&](uint32_t tk, v4u (&v)[8]) {
        uint32_t cell, g;
        cell_of(tk, cell, g);
        const uint8_t* b = cs.base[cell % 9u] + uint64_t(cell / 9u) * cs.stride[cell % 9u] + uint64_t(g) * 8192u;
#pragma unroll
        for (int t = 0; t < 8; t++)
            v[t] = __builtin_nontemporal_load(reinterpret_cast<const v4u*>(b + t * 1024 + lane * 16));
    };
    uint32_t task = blockIdx.x * 4 + wave;
    v4u v[8];
    if (task < tasks) load(task, v);
    for (; task < tasks; task += step) {
#pragma unroll
        for (int t = 0; t < 8; t++) {
            const uint32_t off = uint32_t(t) * 1024u + uint32_t(lane) * 16u;
            *reinterpret_cast<v4u*>(stage + (off / Q) * PITCH + (off % Q)) = v[t];
        }
        if (task + step < tasks) load(task + step, v);
        __builtin_amdgcn_wave_barrier();
        asm volatile("" ::: "memory");
        uint32_t r = cd::quarter_fold<true>(s_tab, stage + lane * PITCH);
        if (qi < 3) r = cd::apply_shift_nib(reinterpret_cast<const uint32_t(*)[8][16]>(s_tab + 10240)[qi], r);
        r ^= __shfl_xor(r, 1);
        r ^= __shfl_xor(r, 2);
        uint32_t cell, g;
        cell_of(task, cell, g);
        if (qi == 0) out[uint64_t(cell) * kNck + g * 16 + c] = __builtin_bswap32(r ^ kfinal);
        __builtin_amdgcn_wave_barrier();
        asm volatile("" ::: "memory");
    }
}

struct Variant {
    std::string name;
    const void* fn;  // null: the product (hec_crc32c_device)
    int waves, per_cu;
    bool check;
    uint32_t inter;
};

template <int W, int N, int T>
Variant make(int per_cu, uint32_t inter) {
    return {"dma w" + std::to_string(W) + " st" + std::to_string(N) + (T == 2 ? " w11" : T == 1 ? " s8" : " mem") +
                " x" + std::to_string(per_cu) + "/CU inter " + std::to_string(inter),
            reinterpret_cast<const void*>(&crc_dma<W, N, T>), W, per_cu, T != 0, inter};
}

static uint32_t host_crc32c(const uint8_t* p, size_t n) {
    static uint32_t t[256];
    static bool init = false;
    if (!init) {
        for (uint32_t i = 0; i < 256; i++) {
            uint32_t c = i;
            for (int b = 0; b < 8; b++) c = (c >> 1) ^ (0x82F63B78u & (0u - (c & 1u)));
            t[i] = c;
        }
        init = true;
    }
    uint32_t r = 0xFFFFFFFFu;
    for (size_t i = 0; i < n; i++) r = t[(r ^ p[i]) & 0xFF] ^ (r >> 8);
    return r ^ 0xFFFFFFFFu;
}

static void fill(uint8_t* dst, size_t n, uint64_t x) {  // deterministic, 64 MiB at a time
    std::vector<uint8_t> h(64u << 20);
    for (size_t off = 0; off < n; off += h.size()) {
        for (size_t i = 0; i < h.size(); i += 8) {
            x ^= x << 13, x ^= x >> 7, x ^= x << 17;
            std::memcpy(&h[i], &x, 8);
        }
        CK(hipMemcpy(dst + off, h.data(), std::min(h.size(), n - off), hipMemcpyHostToDevice));
    }
}

// PROBE_SETS fresh buffer sets in one process (earlier sets stay allocated,
// so each gets new memory); per set every variant, rounds alternated.
// PROBE_LAYOUT: contig = one [S][9][cell] allocation; split = data
// [S][6][cell] + parity [S][3][cell] (bench.py's layout).
int main() {
    const uint32_t S = uint32_t(std::atoi(std::getenv("PROBE_STRIPES") ? std::getenv("PROBE_STRIPES") : "1024"));
    const int rounds = std::atoi(std::getenv("PROBE_ROUNDS") ? std::getenv("PROBE_ROUNDS") : "4");
    const int reps = std::atoi(std::getenv("PROBE_REPS") ? std::getenv("PROBE_REPS") : "8");
    const int nsets = std::atoi(std::getenv("PROBE_SETS") ? std::getenv("PROBE_SETS") : "3");
    const std::string layout = std::getenv("PROBE_LAYOUT") ? std::getenv("PROBE_LAYOUT") : "contig";
    const uint32_t ncells = S * 9;
    const size_t bytes = size_t(ncells) * kCell;
    hipDeviceProp_t prop;
    CK(hipGetDeviceProperties(&prop, 0));
    const int cus = prop.multiProcessorCount;
    hec_coder_t* coder = nullptr;
    if (hec_coder_create(6, 3, 0, &coder) != 0) {
        std::fprintf(stderr, "coder: %s\n", hec_last_error());
        return 1;
    }
    uint32_t *o_ref = nullptr, *o = nullptr;
    CK(hipMalloc(&o_ref, size_t(ncells) * kNck * 4));
    CK(hipMalloc(&o, size_t(ncells) * kNck * 4));
    auto reg = [](uint32_t inter) {
        return Variant{"reg (product restated) inter " + std::to_string(inter),
                       reinterpret_cast<const void*>(&crc_reg), 4, 2, true, inter};
    };
    std::vector<Variant> vs = {
        {"product hec_crc32c_device", nullptr, 0, 0, true, 1},
        reg(1), reg(2), reg(4), reg(8), reg(16),
        make<4, 3, 1>(1, 1), make<4, 3, 1>(1, 8), make<4, 4, 1>(1, 8),
    };
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    const uint32_t tasks = ncells * kGroups;
    for (int set = 0; set < nsets; set++) {
        uint8_t* d = nullptr;
        uint8_t* dpar = nullptr;
        if (layout == "split") {
            CK(hipMalloc(&d, size_t(S) * 6 * kCell));
            CK(hipMalloc(&dpar, size_t(S) * 3 * kCell));
            fill(d, size_t(S) * 6 * kCell, 0x9E3779B97F4A7C15ull + set);
            fill(dpar, size_t(S) * 3 * kCell, 0x1234567887654321ull + set);
        } else {
            CK(hipMalloc(&d, bytes));
            fill(d, bytes, 0x9E3779B97F4A7C15ull + set);
        }
        std::vector<const uint8_t*> bases(9);
        std::vector<size_t> strides(9, size_t(9) * kCell);
        Cells cs;
        for (int i = 0; i < 9; i++) {
            if (layout == "split") {
                bases[i] = i < 6 ? d + size_t(i) * kCell : dpar + size_t(i - 6) * kCell;
                strides[i] = (i < 6 ? 6 : 3) * size_t(kCell);
            } else {
                bases[i] = d + size_t(i) * kCell;
            }
            cs.base[i] = bases[i];
            cs.stride[i] = strides[i];
        }
        auto run_ref = [&](uint32_t* dst) {
            const int rc = hec_crc32c_device(coder, bases.data(), strides.data(), 9, kCell, S, 512,
                                             reinterpret_cast<uint8_t*>(dst), nullptr);
            if (rc != 0) {
                std::fprintf(stderr, "hec_crc32c_device %d %s\n", rc, hec_last_error());
                std::exit(1);
            }
        };
        run_ref(o_ref);
        CK(hipDeviceSynchronize());
        {  // the product against a host CRC on sampled chunks
            std::vector<uint32_t> got(kNck);
            std::vector<uint8_t> cellh(kCell);
            for (uint32_t cidx : {0u, 1u, 7u, ncells / 2, ncells - 1}) {
                CK(hipMemcpy(cellh.data(), bases[cidx % 9] + size_t(cidx / 9) * strides[cidx % 9], kCell,
                             hipMemcpyDeviceToHost));
                CK(hipMemcpy(got.data(), o_ref + size_t(cidx) * kNck, kNck * 4, hipMemcpyDeviceToHost));
                for (uint32_t ch = 0; ch < kNck; ch += 37) {
                    const uint32_t want = __builtin_bswap32(host_crc32c(cellh.data() + ch * 512, 512));
                    if (got[ch] != want) {
                        std::fprintf(stderr, "product mismatch cell %u chunk %u\n", cidx, ch);
                        return 1;
                    }
                }
            }
        }
        auto launch = [&](const Variant& v) {
            if (!v.fn) return run_ref(o);
            uint64_t grid = (tasks + v.waves - 1) / v.waves;
            grid = std::min<uint64_t>(grid, uint64_t(cus) * v.per_cu);
            uint32_t inter = v.inter;
            void* args[] = {&cs, const_cast<uint32_t*>(&ncells), &o, &inter};
            CK(hipLaunchKernel(v.fn, dim3(uint32_t(grid)), dim3(v.waves * 64), args, 0, nullptr));
        };
        for (const Variant& v : vs) {  // correctness first
            CK(hipMemset(o, 0, size_t(ncells) * kNck * 4));
            launch(v);
            CK(hipDeviceSynchronize());
            if (v.check) {
                std::vector<uint32_t> h1(size_t(ncells) * kNck), h2(size_t(ncells) * kNck);
                CK(hipMemcpy(h1.data(), o_ref, h1.size() * 4, hipMemcpyDeviceToHost));
                CK(hipMemcpy(h2.data(), o, h2.size() * 4, hipMemcpyDeviceToHost));
                if (h1 != h2) {
                    size_t bad = 0;
                    while (h1[bad] == h2[bad]) bad++;
                    std::printf("%s: MISMATCH at sum %zu\n", v.name.c_str(), bad);
                    return 2;
                }
            }
        }
        std::vector<std::vector<float>> ms(vs.size());
        for (int r = 0; r < rounds; r++)
            for (size_t i = 0; i < vs.size(); i++) {
                launch(vs[i]);
                CK(hipEventRecord(a));
                for (int k = 0; k < reps; k++) launch(vs[i]);
                CK(hipEventRecord(b));
                CK(hipEventSynchronize(b));
                float t = 0;
                CK(hipEventElapsedTime(&t, a, b));
                ms[i].push_back(t / reps);
            }
        const double algo = double(bytes) + double(ncells) * kNck * 4;
        std::printf("set %d (%s, base %p):\n", set, layout.c_str(), static_cast<void*>(d));
        for (size_t i = 0; i < vs.size(); i++) {
            auto v = ms[i];
            std::sort(v.begin(), v.end());
            const double med = v[v.size() / 2];
            std::printf("  %-40s median %.4f ms (min %.4f max %.4f) %.4f of 8 TB/s%s\n", vs[i].name.c_str(), med,
                        v.front(), v.back(), algo / (med * 1e-3) / 8e12, vs[i].check ? "" : " [no CRC math]");
        }
        std::fflush(stdout);
    }
    hec_coder_destroy(coder);
    return 0;
}
