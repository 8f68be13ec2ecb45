// host_gf_check.cpp -- the engine's host-side GF(2^8) multiply
// (hdfs-native_amd/csrc/host_gf.cpp: AVX-512BW+GFNI affine, AVX2 split-nibble
// vpshufb, scalar) against the CPU oracle's restatement of the reference hot
// loop (oracle/ec_oracle.c orc_matmul_shards, rust/src/ec/matrix.rs:204-231),
// bit-exact, for every ISA this CPU supports: RS encode / decode matrices and
// random matrices up to 16 x 32, lengths 1 .. 65543 (all tails).  `bench`
// as argv[1] also prints GiB/s per ISA and row size.  Run by
// tests/test_host_gf.py (CPU).
#include <chrono>
#include <cstdio>
#include <cstring>
#include <random>
#include <vector>

#include "../../hdfs-native_amd/csrc/gf256.hpp"
#include "../../hdfs-native_amd/csrc/host_gf.hpp"

extern "C" void orc_matmul_shards(const uint8_t* M, size_t r, size_t k, const uint8_t* const* in, size_t n,
                                  uint8_t* const* out);

using hec::host::Isa;

static int failures = 0;

static bool run_case(Isa isa, const std::vector<uint8_t>& mat, size_t rows, size_t cols, size_t n, std::mt19937& rng) {
    std::vector<std::vector<uint8_t>> in(cols, std::vector<uint8_t>(n)), got(rows), want(rows);
    for (auto& v : in)
        for (auto& b : v) b = uint8_t(rng());
    std::vector<const uint8_t*> ip;
    std::vector<uint8_t*> gp, wp;
    for (auto& v : in) ip.push_back(v.data());
    for (size_t j = 0; j < rows; j++) {
        got[j].assign(n + 64, 0xA5);  // guard bytes past n must stay untouched
        want[j].assign(n, 0);
        gp.push_back(got[j].data());
        wp.push_back(want[j].data());
    }
    // half the cases with the affine matrices precomputed (the coder's path)
    const std::vector<uint64_t> aff = hec::host::affine_matrices(mat.data(), mat.size());
    hec::host::gf_matmul(isa, mat.data(), (n & 1) ? aff.data() : nullptr, rows, cols, ip.data(), gp.data(), n);
    orc_matmul_shards(mat.data(), rows, cols, ip.data(), n, wp.data());
    for (size_t j = 0; j < rows; j++) {
        if (std::memcmp(got[j].data(), want[j].data(), n) != 0) return false;
        for (size_t b = n; b < n + 64; b++)
            if (got[j][b] != 0xA5) return false;
    }
    return true;
}

int main(int argc, char** argv) {
    const Isa best = hec::host::best_isa();
    std::printf("best isa: %s\n", hec::host::isa_name(best));
    std::mt19937 rng(0x5EEDEC00u);
    const size_t lens[] = {1, 2, 15, 16, 17, 31, 32, 33, 63, 64, 65, 127, 128, 129, 1000, 4093, 4096, 65536 + 7};
    size_t cases = 0;
    for (int isa_i = 0; isa_i <= int(best); isa_i++) {
        const Isa isa = Isa(isa_i);
        // the RS encode matrices and one decode matrix of each code
        for (auto km : {std::pair<size_t, size_t>{3, 2}, {6, 3}, {10, 4}, {32, 16}, {1, 1}}) {
            const size_t k = km.first, m = km.second;
            const std::vector<uint8_t> enc = hec::gen_rs_matrix(k, m);
            std::vector<uint8_t> par(enc.begin() + k * k, enc.end());
            std::vector<uint8_t> sub(k * k);
            for (size_t r = 0; r < k; r++) std::memcpy(&sub[r * k], &enc[(r + std::min(m, k)) * k], k);
            hec::invert(sub.data(), k);
            std::vector<uint8_t> dec(sub.begin(), sub.begin() + std::min(m, k) * k);
            for (size_t n : lens) {
                for (auto* mm : {&par, &dec}) {
                    const size_t rows = mm->size() / k;
                    if (!run_case(isa, *mm, rows, k, n, rng)) {
                        std::fprintf(stderr, "FAIL isa %s RS(%zu,%zu) rows %zu n %zu\n", hec::host::isa_name(isa), k, m,
                                     rows, n);
                        failures++;
                    }
                    cases++;
                }
            }
        }
        // random matrices (zeros included)
        for (int t = 0; t < 60; t++) {
            const size_t rows = 1 + rng() % 16, cols = 1 + rng() % 32, n = lens[rng() % (sizeof(lens) / sizeof(lens[0]))];
            std::vector<uint8_t> mat(rows * cols);
            for (auto& c : mat) c = (rng() % 5 == 0) ? 0 : uint8_t(rng());
            if (!run_case(isa, mat, rows, cols, n, rng)) {
                std::fprintf(stderr, "FAIL isa %s random %zux%zu n %zu\n", hec::host::isa_name(isa), rows, cols, n);
                failures++;
            }
            cases++;
        }
    }
    // the affine matrix of c, applied bit by bit, is multiplication by c
    for (int c = 0; c < 256; c++) {
        const uint64_t q = hec::host::affine_matrix(uint8_t(c));
        for (int x = 0; x < 256; x++) {
            uint8_t y = 0;
            for (int i = 0; i < 8; i++) {
                const uint8_t row = uint8_t(q >> (8 * (7 - i)));
                y |= uint8_t((__builtin_popcount(row & x) & 1) << i);
            }
            if (y != hec::gf_mul(uint8_t(c), uint8_t(x))) {
                failures++;
                std::fprintf(stderr, "FAIL affine c=%d x=%d\n", c, x);
                break;
            }
        }
    }
    if (argc > 1 && std::strcmp(argv[1], "bench") == 0) {
        const std::vector<uint8_t> enc = hec::gen_rs_matrix(6, 3);
        for (size_t n : {size_t(16), size_t(512), size_t(4096), size_t(16384), size_t(65536), size_t(1) << 20}) {
            std::vector<std::vector<uint8_t>> in(6, std::vector<uint8_t>(n, 7)), out(3, std::vector<uint8_t>(n));
            std::vector<const uint8_t*> ip;
            std::vector<uint8_t*> op;
            for (auto& v : in) ip.push_back(v.data());
            for (auto& v : out) op.push_back(v.data());
            const std::vector<uint64_t> aff = hec::host::affine_matrices(enc.data() + 36, 18);
            for (int isa_i = 0; isa_i <= int(best); isa_i++) {
                const size_t reps = std::max<size_t>(4, (size_t(64) << 20) / (6 * n) / (isa_i == 0 ? 16 : 1));
                const auto t0 = std::chrono::steady_clock::now();
                for (size_t r = 0; r < reps; r++)
                    hec::host::gf_matmul(Isa(isa_i), enc.data() + 36, aff.data(), 3, 6, ip.data(), op.data(), n);
                const double s = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
                std::printf("bench RS(6,3) encode n=%zu isa=%s %.3f us/call %.2f GiB/s\n", n,
                            hec::host::isa_name(Isa(isa_i)), s / reps * 1e6, 6.0 * n * reps / s / (1 << 30));
            }
        }
    }
    if (failures) {
        std::fprintf(stderr, "%d failure(s) in %zu cases\n", failures, cases);
        return 1;
    }
    std::printf("host gf ok: %zu cases\n", cases);
    return 0;
}
