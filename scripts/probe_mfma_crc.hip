// probe_mfma_crc.hip -- measurement tool (not shipped): CRC32C per 512-B
// chunk with the GF(2)-linear map on the matrix cores instead of LDS table
// lookups.  Checks the idea and the i8 MFMA operand layout before it goes
// into checksum.hip.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 scripts/probe_mfma_crc.hip -o scripts/probe_mfma_crc
//
// The linear part of the CRC of a 128-B quarter is L(q) = XOR over set bits
// (p, b) of column vectors L(e_pb).  As an integer matmul on
// v_mfma_i32_32x32x32_i8: rows = 32 quarters, k = 32 byte positions of one
// 32-B segment, one bit plane b per MFMA, n = 32 CRC bits.
//   A_b[row][k] = byte & (1 << b)            in {0, 2^b}   (one v_and per dword)
//   B_b[k][n]   = bit n of L(e_pb) ? 2^(7-b) : 0 (int8: 2^7 wraps to -128)
// Every product is 0 or +-2^7, so summing all 8 planes and 4 segments into one
// int32 accumulator leaves bit n of L(q) in bit 7 (the parity of the count).
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#define CK(x)                                                                                        \
    do {                                                                                             \
        hipError_t e = (x);                                                                          \
        if (e != hipSuccess) {                                                                       \
            std::fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e));    \
            std::exit(1);                                                                            \
        }                                                                                            \
    } while (0)

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef int8_t i8x16 __attribute__((ext_vector_type(16)));
typedef int32_t i32x16 __attribute__((ext_vector_type(16)));

constexpr uint32_t kPoly = 0x82F63B78u;

static uint32_t host_tab[256];
static void host_init() {
    for (int i = 0; i < 256; i++) {
        uint32_t c = i;
        for (int b = 0; b < 8; b++) c = (c >> 1) ^ (kPoly & (0u - (c & 1u)));
        host_tab[i] = c;
    }
}
static uint32_t host_crc(const uint8_t* p, size_t n, uint32_t r = 0xFFFFFFFFu) {
    for (size_t i = 0; i < n; i++) r = host_tab[(r ^ p[i]) & 0xFF] ^ (r >> 8);
    return r;
}
static uint32_t host_zero(uint32_t r, int n) {
    for (int i = 0; i < n; i++) r = host_tab[r & 0xFF] ^ (r >> 8);
    return r;
}

// B tiles: [seg 0..3][plane 0..7][lane 0..63][16 B]; lane l = (col c = l&31,
// half h = l>>5), byte j = B[k = 16h + j][c]
static std::vector<int8_t> make_btiles() {
    std::vector<int8_t> t(4 * 8 * 64 * 16);
    for (int s = 0; s < 4; s++)
        for (int b = 0; b < 8; b++)
            for (int l = 0; l < 64; l++)
                for (int j = 0; j < 16; j++) {
                    const int c = l & 31, h = l >> 5, p = 32 * s + 16 * h + j;
                    uint8_t q[128] = {};
                    q[p] = uint8_t(1u << b);
                    const uint32_t lin = host_crc(q, 128, 0);  // linear part from state 0
                    const int v = ((lin >> c) & 1) ? (1 << (7 - b)) : 0;
                    t[((s * 8 + b) * 64 + l) * 16 + j] = int8_t(uint8_t(v));
                }
    return t;
}

struct ShiftTabs {
    uint32_t t[3][4][256];  // append 384 / 256 / 128 zero bytes
    uint32_t final512;
    uint32_t slice[8][256];  // slicing-by-8 (hybrid mode)
};
static ShiftTabs make_shift() {
    ShiftTabs s;
    for (int k = 0; k < 3; k++) {
        const int n = 128 * (3 - k);
        uint32_t col[32];
        for (int j = 0; j < 32; j++) col[j] = host_zero(1u << j, n);
        for (int b = 0; b < 4; b++)
            for (int x = 0; x < 256; x++) {
                uint32_t v = 0;
                for (int j = 0; j < 8; j++)
                    if (x & (1 << j)) v ^= col[8 * b + j];
                s.t[k][b][x] = v;
            }
    }
    s.final512 = host_zero(0xFFFFFFFFu, 512) ^ 0xFFFFFFFFu;
    for (int i = 0; i < 256; i++) s.slice[0][i] = host_tab[i];
    for (int k = 1; k < 8; k++)
        for (int i = 0; i < 256; i++) s.slice[k][i] = host_tab[s.slice[k - 1][i] & 0xFF] ^ (s.slice[k - 1][i] >> 8);
    return s;
}

// One wave = one task of 16 chunks (8 KiB) at a time: 8 coalesced 1-KiB loads
// -> LDS quarter image (64 rows x 144 B) -> 2 row groups x 4 segments x 8
// planes of MFMA -> ballots put quarter q's 32 bits in lane q -> zero-append
// shifts + 2 xor shuffles -> one CRC per chunk.
// MODE 0: full; 1: no MFMA (memory + staging side); 2: no global loads
// after the first task (compute side); 3: hybrid -- quarters 0-31 by
// slicing-by-8 LDS lookups (lanes 0-31), quarters 32-63 on the MFMA;
// 4: hybrid without global loads.  PF: tasks of register prefetch.
template <int BS, bool BREG, int PF = 1, int MODE = 0>
__global__ __launch_bounds__(BS) void crc_mfma(const uint8_t* __restrict__ data, size_t tasks,
                                               uint32_t* __restrict__ out, const int8_t* __restrict__ btiles,
                                               const ShiftTabs* __restrict__ sh, uint32_t* dbg) {
    constexpr int WAVES = BS / 64, PITCH = 144, STAGE = 64 * PITCH;
    __shared__ uint32_t s_shift[3][4][256];
    __shared__ __attribute__((aligned(16))) uint8_t s_stage[WAVES * STAGE];
    __shared__ __attribute__((aligned(16))) int8_t s_b[BREG ? 16 : 32 * 1024];
    __shared__ uint32_t s_slice[MODE >= 3 ? 8 : 1][256];
    if constexpr (MODE >= 3)
        for (int t = threadIdx.x; t < 8 * 256; t += BS) (&s_slice[0][0])[t] = (&sh->slice[0][0])[t];
    for (int t = threadIdx.x; t < 3 * 4 * 256; t += BS) (&s_shift[0][0][0])[t] = (&sh->t[0][0][0])[t];
    if constexpr (!BREG)
        for (int t = threadIdx.x; t < 32 * 1024 / 16; t += BS)
            reinterpret_cast<u32x4*>(s_b)[t] = reinterpret_cast<const u32x4*>(btiles)[t];
    __syncthreads();
    const uint32_t kfinal = sh->final512;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x / 64), lane = threadIdx.x & 63;
    uint8_t* stage = s_stage + wave * STAGE;
    u32x4 breg[BREG ? 32 : 1];
    if constexpr (BREG)
        for (int t = 0; t < 32; t++) breg[t] = reinterpret_cast<const u32x4*>(btiles)[t * 64 + lane];

    const size_t step = size_t(gridDim.x) * WAVES;
    size_t task = size_t(blockIdx.x) * WAVES + wave;
    u32x4 va[8], vb[8];
    auto load = [&](size_t t, u32x4 (&v)[8]) {
        const uint8_t* base = data + t * 8192;
#pragma unroll
        for (int i = 0; i < 8; i++) v[i] = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(base + i * 1024 + lane * 16));
    };
    if (task < tasks) load(task, va);
    if (PF == 2 && task + step < tasks) load(task + step, vb);
    auto process = [&](size_t task, u32x4 (&v)[8]) {
#pragma unroll
        for (int i = 0; i < 8; i++) {
            const uint32_t off = uint32_t(i) * 1024u + uint32_t(lane) * 16u;
            *reinterpret_cast<u32x4*>(stage + (off / 128) * PITCH + (off % 128)) = v[i];
        }
        if (MODE != 2 && MODE != 4 && task + PF * step < tasks) load(task + PF * step, v);
        __builtin_amdgcn_wave_barrier();
        asm volatile("" ::: "memory");
        uint32_t qv = 0;  // lane q: linear part of quarter q
        constexpr int G0 = MODE >= 3 ? 1 : 0;  // hybrid: MFMA on row group 1 only
        if constexpr (MODE >= 3) {
            if (lane < 32) {
                const uint8_t* row = stage + lane * PITCH;
                uint32_t r = 0;
#pragma unroll
                for (int t = 0; t < 8; t++) {
                    const u32x4 w = *reinterpret_cast<const u32x4*>(row + t * 16);
#pragma unroll
                    for (int h = 0; h < 2; h++) {
                        const uint32_t lo = (h ? w.z : w.x) ^ r, hi = h ? w.w : w.y;
                        r = s_slice[7][lo & 0xFF] ^ s_slice[6][(lo >> 8) & 0xFF] ^ s_slice[5][(lo >> 16) & 0xFF] ^
                            s_slice[4][lo >> 24] ^ s_slice[3][hi & 0xFF] ^ s_slice[2][(hi >> 8) & 0xFF] ^
                            s_slice[1][(hi >> 16) & 0xFF] ^ s_slice[0][hi >> 24];
                    }
                }
                qv = r;
            }
        }
        // both row groups at once: two independent accumulation chains share
        // each B tile
        i32x16 acc[2] = {};
#pragma unroll
        for (int s = 0; s < 4; s++) {
            u32x4 a[2];
#pragma unroll
            for (int g = G0; g < 2; g++)
                a[g] = *reinterpret_cast<const u32x4*>(stage + (32 * g + (lane & 31)) * PITCH + 32 * s + 16 * (lane >> 5));
#pragma unroll
            for (int b = 0; b < 8; b++) {
                const uint32_t m = 0x01010101u << b;
                u32x4 bb;
                if constexpr (BREG)
                    bb = breg[s * 8 + b];
                else
                    bb = *reinterpret_cast<const u32x4*>(s_b + ((s * 8 + b) * 64 + lane) * 16);
#pragma unroll
                for (int g = G0; g < 2; g++) {
                    const u32x4 am = u32x4{a[g].x & m, a[g].y & m, a[g].z & m, a[g].w & m};
                    if constexpr (MODE == 1)
                        acc[g][b] ^= am.x ^ bb.y;
                    else
                        acc[g] = __builtin_amdgcn_mfma_i32_32x32x32_i8(__builtin_bit_cast(i8x16, am),
                                                                       __builtin_bit_cast(i8x16, bb), acc[g], 0, 0, 0);
                }
            }
        }
#pragma unroll
        for (int g = G0; g < 2; g++) {
            // D[row][col]: col = lane&31 = CRC bit, row = (i&3) + 8*(i>>2) + 4*(lane>>5).
            // Ballots -> SGPRs; v_writelane reads an SGPR a VALU (v_cmp) just
            // wrote, which needs wait states that hipcc does not add inside asm
#pragma unroll
            for (int i0 = 0; i0 < 16; i0 += 4) {
                uint64_t bal[4];
#pragma unroll
                for (int t = 0; t < 4; t++) bal[t] = __builtin_amdgcn_ballot_w64((acc[g][i0 + t] & 0x80) != 0);
                asm volatile(
                    "s_nop 4\n"
                    "v_writelane_b32 %0, %1, %9\n v_writelane_b32 %0, %2, %10\n"
                    "v_writelane_b32 %0, %3, %11\n v_writelane_b32 %0, %4, %12\n"
                    "v_writelane_b32 %0, %5, %13\n v_writelane_b32 %0, %6, %14\n"
                    "v_writelane_b32 %0, %7, %15\n v_writelane_b32 %0, %8, %16\n"
                    : "+v"(qv)
                    : "s"(uint32_t(bal[0])), "s"(uint32_t(bal[0] >> 32)), "s"(uint32_t(bal[1])),
                      "s"(uint32_t(bal[1] >> 32)), "s"(uint32_t(bal[2])), "s"(uint32_t(bal[2] >> 32)),
                      "s"(uint32_t(bal[3])), "s"(uint32_t(bal[3] >> 32)), "n"(32 * g + 8 * (i0 >> 2) + 0),
                      "n"(32 * g + 8 * (i0 >> 2) + 4), "n"(32 * g + 8 * (i0 >> 2) + 1), "n"(32 * g + 8 * (i0 >> 2) + 5),
                      "n"(32 * g + 8 * (i0 >> 2) + 2), "n"(32 * g + 8 * (i0 >> 2) + 6), "n"(32 * g + 8 * (i0 >> 2) + 3),
                      "n"(32 * g + 8 * (i0 >> 2) + 7));
            }
        }
        if (dbg && task == 0) dbg[lane] = qv;
        const int qi = lane & 3;
        uint32_t r = qv;
        if (qi < 3) r = s_shift[qi][0][r & 0xFF] ^ s_shift[qi][1][(r >> 8) & 0xFF] ^ s_shift[qi][2][(r >> 16) & 0xFF] ^
                        s_shift[qi][3][r >> 24];
        r ^= __shfl_xor(r, 1);
        r ^= __shfl_xor(r, 2);
        if (qi == 0) out[task * 16 + (lane >> 2)] = r ^ kfinal;
        __builtin_amdgcn_wave_barrier();
        asm volatile("" ::: "memory");
    };
    while (task < tasks) {
        process(task, va);
        task += step;
        if constexpr (PF == 2) {
            if (task >= tasks) break;
            process(task, vb);
            task += step;
        }
    }
}

template <int BS, bool BREG, int PF = 1, int MODE = 0>
static void run(const char* name, const uint8_t* d, size_t tasks, uint32_t* o, const int8_t* bt, const ShiftTabs* st,
                int grid, const std::vector<uint8_t>& host, std::vector<uint32_t>& hout) {
    CK(hipMemset(o, 0, tasks * 16 * 4));
    uint32_t* dbg;
    CK(hipMalloc(&dbg, 256));
    hipLaunchKernelGGL((crc_mfma<BS, BREG, PF, MODE>), dim3(grid), dim3(BS), 0, 0, d, tasks, o, bt, st, dbg);
    CK(hipDeviceSynchronize());
    uint32_t hd[64];
    CK(hipMemcpy(hd, dbg, 256, hipMemcpyDeviceToHost));
    for (int l = 0; l < 64; l++) {
        int match = -1;
        for (int q = 0; q < 64; q++)
            if (host_crc(host.data() + q * 128, 128, 0) == hd[l]) match = q;
        std::printf("%d:%d ", l, match);
    }
    std::printf("\n");
    CK(hipMemcpy(hout.data(), o, hout.size() * 4, hipMemcpyDeviceToHost));
    int bad = 0;
    for (size_t c = 0; c < hout.size(); c++)
        if (hout[c] != (host_crc(host.data() + c * 512, 512) ^ 0xFFFFFFFFu)) bad++;
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    const int reps = 10;
    CK(hipEventRecord(e0));
    for (int i = 0; i < reps; i++) hipLaunchKernelGGL((crc_mfma<BS, BREG, PF, MODE>), dim3(grid), dim3(BS), 0, 0, d, tasks, o, bt, st, nullptr);
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, e0, e1));
    ms /= reps;
    std::printf("%s grid=%d: %.3f ms  %.1f GB/s  mismatches(first %zu chunks)=%d\n", name, grid, ms,
                tasks * 8192.0 / ms / 1e6, hout.size(), bad);
}

int main() {
    host_init();
    const size_t tasks = size_t(1) << 18;  // 2 GiB
    const size_t bytes = tasks * 8192;
    uint8_t* d;
    uint32_t* o;
    int8_t* bt;
    ShiftTabs* st;
    CK(hipMalloc(&d, bytes));
    CK(hipMalloc(&o, tasks * 16 * 4));
    CK(hipMalloc(&bt, 32 * 1024));
    CK(hipMalloc(&st, sizeof(ShiftTabs)));
    std::vector<uint8_t> host(size_t(8) << 20);
    uint64_t x = 0x9E3779B97F4A7C15ull;
    for (auto& b : host) {
        x ^= x << 13;
        x ^= x >> 7;
        x ^= x << 17;
        b = uint8_t(x >> 24);
    }
    for (size_t off = 0; off < bytes; off += host.size()) CK(hipMemcpy(d + off, host.data(), host.size(), hipMemcpyHostToDevice));
    const auto btiles = make_btiles();
    const ShiftTabs shs = make_shift();
    CK(hipMemcpy(bt, btiles.data(), btiles.size(), hipMemcpyHostToDevice));
    CK(hipMemcpy(st, &shs, sizeof(shs), hipMemcpyHostToDevice));
    std::vector<uint32_t> hout(host.size() / 512);
    int cus = 256;
    for (int rep = 0; rep < 2; rep++) {
        run<256, true, 1, 0>("breg pf1 full", d, tasks, o, bt, st, cus * 2, host, hout);
        run<256, true, 1, 2>("breg pf1 no-loads", d, tasks, o, bt, st, cus * 2, host, hout);
        run<256, true, 1, 3>("breg pf1 hybrid", d, tasks, o, bt, st, cus * 2, host, hout);
        run<256, true, 2, 3>("breg pf2 hybrid", d, tasks, o, bt, st, cus * 2, host, hout);
        run<256, true, 1, 4>("breg pf1 hybrid no-loads", d, tasks, o, bt, st, cus * 2, host, hout);
        run<256, false, 2, 3>("blds pf2 hybrid", d, tasks, o, bt, st, cus * 2, host, hout);
        run<512, false, 2, 3>("blds bs512 pf2 hybrid", d, tasks, o, bt, st, cus * 1, host, hout);
    }
    return 0;
}
