// host_gf.cpp -- host-side GF(2^8) stripe multiply (see host_gf.hpp): the
// per-call drop-in's path for rows below the coder's host limit, where one
// PCIe round trip and a launch (tens of microseconds) cost more than the
// whole row on a CPU core.
#include "host_gf.hpp"

#include <immintrin.h>
#include <pthread.h>
#include <sys/types.h>
#include <unistd.h>

#include <algorithm>
#include <condition_variable>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <mutex>
#include <new>
#include <thread>

#include "gf256.hpp"

namespace hec {
namespace host {

uint64_t affine_matrix(uint8_t c) {
    // column b of the bit matrix = c * x^b; row i = bit i of every column
    uint8_t col[8];
    for (int b = 0; b < 8; b++) col[b] = gf_mul(c, uint8_t(1u << b));
    uint64_t q = 0;
    for (int i = 0; i < 8; i++) {
        uint8_t row = 0;
        for (int b = 0; b < 8; b++) row |= uint8_t(((col[b] >> i) & 1u) << b);
        q |= uint64_t(row) << (8 * (7 - i));
    }
    return q;
}

std::vector<uint64_t> affine_matrices(const uint8_t* mat, size_t n_entries) {
    std::vector<uint64_t> a(n_entries);
    for (size_t x = 0; x < n_entries; x++) a[x] = affine_matrix(mat[x]);
    return a;
}

namespace {

// ---- scalar: log / antilog ------------------------------------------------
void matmul_scalar(const uint8_t* mat, size_t rows, size_t cols, const uint8_t* const* in, uint8_t* const* out,
                   size_t n) {
    for (size_t j = 0; j < rows; j++) {
        uint8_t* o = out[j];
        std::memset(o, 0, n);
        for (size_t i = 0; i < cols; i++) {
            const uint8_t c = mat[j * cols + i];
            if (c == 0) continue;
            const unsigned lc = kGf.log[c];
            const uint8_t* x = in[i];
            for (size_t b = 0; b < n; b++)
                if (x[b]) o[b] ^= kGf.exp[lc + kGf.log[x[b]]];
        }
    }
}

// ---- AVX2: split-nibble vpshufb tables --------------------------------------
struct NibbleTables {
    alignas(32) uint8_t lo[32], hi[32];  // c*x and c*(x<<4) for x < 16, repeated per 128-bit lane
};

__attribute__((target("avx2"))) void matmul_avx2(const uint8_t* mat, size_t rows, size_t cols,
                                                 const uint8_t* const* in, uint8_t* const* out, size_t n) {
    NibbleTables tab[4 * 16];
    const __m256i mask = _mm256_set1_epi8(0x0F);
    const size_t whole = n / 32 * 32;
    // rows in groups of up to 4 accumulators, their tables built per group
    for (size_t r0 = 0; r0 < rows; r0 += 4) {
        const size_t nr = std::min<size_t>(4, rows - r0);
        for (size_t i0 = 0; i0 < cols; i0 += 16) {
            const size_t ni = std::min<size_t>(16, cols - i0);
            for (size_t j = 0; j < nr; j++)
                for (size_t i = 0; i < ni; i++) {
                    const uint8_t c = mat[(r0 + j) * cols + i0 + i];
                    NibbleTables& t = tab[j * 16 + i];
                    for (int x = 0; x < 16; x++) {
                        t.lo[x] = t.lo[x + 16] = gf_mul(c, uint8_t(x));
                        t.hi[x] = t.hi[x + 16] = gf_mul(c, uint8_t(x << 4));
                    }
                }
            for (size_t o = 0; o < whole; o += 32) {
                __m256i acc[4];
                for (size_t j = 0; j < nr; j++)
                    acc[j] = i0 == 0 ? _mm256_setzero_si256()
                                     : _mm256_loadu_si256(reinterpret_cast<const __m256i*>(out[r0 + j] + o));
                for (size_t i = 0; i < ni; i++) {
                    const __m256i x = _mm256_loadu_si256(reinterpret_cast<const __m256i*>(in[i0 + i] + o));
                    const __m256i xl = _mm256_and_si256(x, mask);
                    const __m256i xh = _mm256_and_si256(_mm256_srli_epi64(x, 4), mask);
                    for (size_t j = 0; j < nr; j++) {
                        const NibbleTables& t = tab[j * 16 + i];
                        const __m256i pl = _mm256_shuffle_epi8(_mm256_load_si256(reinterpret_cast<const __m256i*>(t.lo)), xl);
                        const __m256i ph = _mm256_shuffle_epi8(_mm256_load_si256(reinterpret_cast<const __m256i*>(t.hi)), xh);
                        acc[j] = _mm256_xor_si256(acc[j], _mm256_xor_si256(pl, ph));
                    }
                }
                for (size_t j = 0; j < nr; j++) _mm256_storeu_si256(reinterpret_cast<__m256i*>(out[r0 + j] + o), acc[j]);
            }
            for (size_t o = whole; o < n; o++)  // tail bytes
                for (size_t j = 0; j < nr; j++) {
                    uint8_t acc = i0 == 0 ? 0 : out[r0 + j][o];
                    for (size_t i = 0; i < ni; i++) acc ^= gf_mul(mat[(r0 + j) * cols + i0 + i], in[i0 + i][o]);
                    out[r0 + j][o] = acc;
                }
        }
    }
}

// ---- AVX-512BW + GFNI: one affine transform per 64 bytes per coefficient ---
#define HEC_GFNI_TARGET __attribute__((target("avx512f,avx512bw,gfni,bmi2")))

// One 64-B column of NR outputs (FULL: all 64 bytes; else the bytes of mask
// m, masked loads / stores: any length, no out-of-bounds access).  A: NR x
// cols affine qwords (row-major); inputs two at a time folded into the
// accumulators with a 3-input XOR (vpternlogq 0x96).
template <int NR, bool FULL>
HEC_GFNI_TARGET inline void gfni_column(const uint64_t* A, size_t cols, const uint8_t* const* in,
                                        uint8_t* const* out, size_t o, __mmask64 m) {
    __m512i acc[NR];
    for (int j = 0; j < NR; j++) acc[j] = _mm512_setzero_si512();
    size_t i = 0;
    for (; i + 2 <= cols; i += 2) {
        const __m512i x0 = FULL ? _mm512_loadu_si512(in[i] + o) : _mm512_maskz_loadu_epi8(m, in[i] + o);
        const __m512i x1 = FULL ? _mm512_loadu_si512(in[i + 1] + o) : _mm512_maskz_loadu_epi8(m, in[i + 1] + o);
        for (int j = 0; j < NR; j++) {
            const __m512i p0 = _mm512_gf2p8affine_epi64_epi8(x0, _mm512_set1_epi64(int64_t(A[j * cols + i])), 0);
            const __m512i p1 = _mm512_gf2p8affine_epi64_epi8(x1, _mm512_set1_epi64(int64_t(A[j * cols + i + 1])), 0);
            acc[j] = _mm512_ternarylogic_epi64(acc[j], p0, p1, 0x96);
        }
    }
    if (i < cols) {
        const __m512i x0 = FULL ? _mm512_loadu_si512(in[i] + o) : _mm512_maskz_loadu_epi8(m, in[i] + o);
        for (int j = 0; j < NR; j++)
            acc[j] = _mm512_xor_si512(acc[j],
                                      _mm512_gf2p8affine_epi64_epi8(x0, _mm512_set1_epi64(int64_t(A[j * cols + i])), 0));
    }
    for (int j = 0; j < NR; j++) {
        if (FULL)
            _mm512_storeu_si512(out[j] + o, acc[j]);
        else
            _mm512_mask_storeu_epi8(out[j] + o, m, acc[j]);
    }
}

template <int NR>
HEC_GFNI_TARGET void gfni_rows(const uint64_t* A, size_t cols, const uint8_t* const* in, uint8_t* const* out,
                               size_t n) {
    size_t o = 0;
    for (; o + 64 <= n; o += 64) gfni_column<NR, true>(A, cols, in, out, o, ~__mmask64(0));
    if (o < n) gfni_column<NR, false>(A, cols, in, out, o, _bzhi_u64(~uint64_t(0), unsigned(n - o)));
}

// aff: rows x cols affine qwords (precomputed), or null (built here from mat)
HEC_GFNI_TARGET void matmul_gfni(const uint8_t* mat, const uint64_t* aff, size_t rows, size_t cols,
                                 const uint8_t* const* in, uint8_t* const* out, size_t n) {
    uint64_t Abuf[8 * 32];
    for (size_t r0 = 0; r0 < rows; r0 += 8) {
        const size_t nr = std::min<size_t>(8, rows - r0);
        const uint64_t* A = aff ? aff + r0 * cols : Abuf;
        if (!aff)
            for (size_t j = 0; j < nr; j++)
                for (size_t i = 0; i < cols; i++) Abuf[j * cols + i] = affine_matrix(mat[(r0 + j) * cols + i]);
        uint8_t* const* o = out + r0;
        switch (nr) {
            case 1: gfni_rows<1>(A, cols, in, o, n); break;
            case 2: gfni_rows<2>(A, cols, in, o, n); break;
            case 3: gfni_rows<3>(A, cols, in, o, n); break;
            case 4: gfni_rows<4>(A, cols, in, o, n); break;
            case 5: gfni_rows<5>(A, cols, in, o, n); break;
            case 6: gfni_rows<6>(A, cols, in, o, n); break;
            case 7: gfni_rows<7>(A, cols, in, o, n); break;
            default: gfni_rows<8>(A, cols, in, o, n); break;
        }
    }
}

Isa detect() {
    __builtin_cpu_init();
    if (__builtin_cpu_supports("avx512f") && __builtin_cpu_supports("avx512bw") && __builtin_cpu_supports("gfni") &&
        __builtin_cpu_supports("bmi2"))
        return kAvx512Gfni;
    if (__builtin_cpu_supports("avx2")) return kAvx2;
    return kScalar;
}

}  // namespace

Isa best_isa() {
    static const Isa isa = detect();
    return isa;
}

const char* isa_name(Isa isa) {
    switch (isa) {
        case kAvx512Gfni: return "avx512bw+gfni";
        case kAvx2: return "avx2";
        default: return "scalar";
    }
}

void gf_matmul(Isa isa, const uint8_t* mat, const uint64_t* aff, size_t rows, size_t cols, const uint8_t* const* in,
               uint8_t* const* out, size_t n) {
    isa = std::min(isa, best_isa());
    if (n == 0 || rows == 0 || cols == 0) return;
    if (isa == kAvx512Gfni && cols <= 32)
        matmul_gfni(mat, aff, rows, cols, in, out, n);
    else if (isa >= kAvx2)
        matmul_avx2(mat, rows, cols, in, out, n);
    else
        matmul_scalar(mat, rows, cols, in, out, n);
}

namespace {

// Column-split helpers for long rows (gf_matmul_split): a process-wide pool
// of worker threads, started on first use.  One split call at a time owns it
// (try-lock): a concurrent caller codes its row on its own thread instead of
// queueing behind another's.
struct SplitPool {
    std::mutex own;          // held by the call that is using the workers
    std::mutex mu;
    std::condition_variable go, done;
    std::vector<std::thread> workers;
    uint64_t gen = 0;        // job generation (workers run each generation once)
    size_t pending = 0;      // worker pieces not finished
    bool stop = false;
    std::function<void(size_t)> job;  // piece index 1..workers.size()

    explicit SplitPool(size_t n) {
        for (size_t w = 0; w < n; w++)
            workers.emplace_back([this, w] {
                uint64_t seen = 0;
                for (;;) {
                    std::function<void(size_t)> f;
                    {
                        std::unique_lock<std::mutex> lk(mu);
                        go.wait(lk, [&] { return stop || gen != seen; });
                        if (stop) return;
                        seen = gen;
                        f = job;
                    }
                    f(w + 1);
                    std::lock_guard<std::mutex> lk(mu);
                    if (--pending == 0) done.notify_one();
                }
            });
    }
    ~SplitPool() {
        {
            std::lock_guard<std::mutex> lk(mu);
            stop = true;
        }
        go.notify_all();
        for (auto& t : workers) t.join();
    }
};

size_t split_threads() {
    static const size_t n = [] {
        const char* v = std::getenv("HEC_HOST_THREADS");
        long t = v && *v ? std::strtol(v, nullptr, 10) : 4;
        const long hw = long(std::thread::hardware_concurrency());
        if (hw > 0) t = std::min(t, hw);
        return size_t(std::max(1L, std::min(t, 64L)));
    }();
    return n;
}

// The process-wide pool, owned by the process that created it.  A fork()ed
// child (Python multiprocessing's default start method) inherits the pool's
// memory but not its worker threads, and a mutex another parent thread held
// at fork time stays locked in the child: posting a job there would wait for
// workers that do not exist.  So the child drops the inherited
// pool (leaked, never touched) and builds its own on first use; the pid check
// covers a fork before the handler was registered.
std::mutex g_pool_mu;
SplitPool* g_pool = nullptr;  // never destroyed: workers may outlive static destruction order
pid_t g_pool_pid = 0;

void pool_after_fork_child() {
    new (&g_pool_mu) std::mutex();  // the child runs only the forking thread
    g_pool = nullptr;
    g_pool_pid = 0;
}

SplitPool* split_pool() {
    if (split_threads() <= 1) return nullptr;
    static const int registered = pthread_atfork(nullptr, nullptr, pool_after_fork_child);
    (void)registered;
    std::lock_guard<std::mutex> lk(g_pool_mu);
    const pid_t me = getpid();
    if (!g_pool || g_pool_pid != me) {
        g_pool = new SplitPool(split_threads() - 1);
        g_pool_pid = me;
    }
    return g_pool;
}

}  // namespace

size_t split_min_bytes() { return size_t(256) << 10; }

void gf_matmul_split(Isa isa, const uint8_t* mat, const uint64_t* aff, size_t rows, size_t cols,
                     const uint8_t* const* in, uint8_t* const* out, size_t n) {
    const size_t T = split_threads();
    // the pieces' pointer arrays below hold up to kMaxSplitShards rows / cols
    // (the C ABI bounds cols only): larger matrices run unsplit
    constexpr size_t kMaxSplitShards = 64;
    SplitPool* pool = n >= split_min_bytes() && T > 1 && rows <= kMaxSplitShards && cols <= kMaxSplitShards
                          ? split_pool()
                          : nullptr;
    std::unique_lock<std::mutex> own;
    if (pool) own = std::unique_lock<std::mutex>(pool->own, std::try_to_lock);
    if (!pool || !own.owns_lock()) {
        gf_matmul(isa, mat, aff, rows, cols, in, out, n);
        return;
    }
    // T column ranges, 4 KiB aligned (no two threads write one cache line or page)
    const size_t piece = ((n + T - 1) / T + 4095) & ~size_t(4095);
    auto run = [&](size_t p) {
        const size_t a = p * piece;
        if (a >= n) return;
        const size_t len = std::min(piece, n - a);
        const uint8_t* pin[kMaxSplitShards];
        uint8_t* pout[kMaxSplitShards];
        for (size_t i = 0; i < cols; i++) pin[i] = in[i] + a;
        for (size_t j = 0; j < rows; j++) pout[j] = out[j] + a;
        gf_matmul(isa, mat, aff, rows, cols, pin, pout, len);
    };
    {
        std::lock_guard<std::mutex> lk(pool->mu);
        pool->job = run;
        pool->pending = pool->workers.size();
        pool->gen++;
    }
    pool->go.notify_all();
    run(0);  // the caller's own piece
    std::unique_lock<std::mutex> lk(pool->mu);
    pool->done.wait(lk, [&] { return pool->pending == 0; });
    pool->job = nullptr;
}

}  // namespace host
}  // namespace hec
