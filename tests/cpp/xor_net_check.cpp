// xor_net_check.cpp -- the plan-time XOR networks of the JIT-specialised
// decode + verify kernel (hdfs-native_amd/csrc/xor_net.hpp, jit.cpp), on the
// host: for EVERY decode plan of RS(3,2), RS(6,3) and RS(10,4) (every
// presence mask with 1..m data shards missing and >= k shards present), the
// plan's matrix (oracle orc_decode_matrix, gf256.rs:84-126 restated) is
// turned into per-input networks, run on bit-sliced survivor data
// (bitslice.hpp transpose8) exactly as the kernel runs them (input 0
// initialises the accumulators), transposed back, and compared with the
// oracle's decode of the same 32-byte cells.  Also random 1..4-row matrices
// for k = 2, 3, 6, 10.  Run by tests/test_host_gf.py (CPU).
#include <cstdio>
#include <cstring>
#include <random>
#include <vector>

#define __host__
#define __device__
#define __forceinline__ inline
#include "../../hdfs-native_amd/csrc/bitslice.hpp"
#include "../../hdfs-native_amd/csrc/gf256.hpp"
#include "../../hdfs-native_amd/csrc/xor_net.hpp"

extern "C" int orc_decode_matrix(size_t k, size_t m, const int* present, uint8_t* dm, size_t* e_out,
                                 size_t* surv_out);
extern "C" void orc_matmul_shards(const uint8_t* M, size_t r, size_t k, const uint8_t* const* in, size_t n,
                                  uint8_t* const* out);

using namespace hec;

// the network of matrix (r x k) on k random 32-byte cells vs the oracle multiply
static int run(const uint8_t* mat, int r, int k, std::mt19937& rng, long* ops_total, int restarts = 32) {
    const auto nets = xornet::matrix_network(mat, r, k, restarts);
    *ops_total += xornet::network_ops(nets);
    int bad = 0;
    for (int trial = 0; trial < 4; trial++) {
        std::vector<std::array<uint32_t, 8>> in(k);
        for (auto& v : in)
            for (auto& w : v) w = trial == 0 ? 0xFFFFFFFFu : uint32_t(rng());
        std::vector<uint32_t> acc(8 * r);
        for (int i = 0; i < k; i++) {
            uint32_t p[8];
            std::memcpy(p, in[i].data(), 32);
            bitslice::transpose8(p);
            xornet::eval_input(nets[i], i == 0, p, acc.data());
        }
        std::vector<const uint8_t*> ip(k);
        for (int i = 0; i < k; i++) ip[i] = reinterpret_cast<const uint8_t*>(in[i].data());
        std::vector<std::array<uint8_t, 32>> want(r);
        std::vector<uint8_t*> op(r);
        for (int j = 0; j < r; j++) op[j] = want[j].data();
        orc_matmul_shards(mat, r, k, ip.data(), 32, op.data());
        for (int j = 0; j < r; j++) {
            uint32_t q[8];
            std::memcpy(q, &acc[8 * j], 32);
            bitslice::transpose8(q);
            if (std::memcmp(q, want[j].data(), 32) != 0) bad++;
        }
    }
    return bad;
}

int main() {
    std::mt19937 rng(11);
    int bad = 0;
    for (auto [k, m] : {std::pair<int, int>{3, 2}, {6, 3}, {10, 4}}) {
        long plans = 0, ops = 0;
        for (unsigned mask = 0; mask < (1u << (k + m)); mask++) {
            int present[16], n_present = 0, lost_data = 0;
            for (int i = 0; i < k + m; i++) {
                present[i] = (mask >> i) & 1;
                n_present += present[i];
                lost_data += i < k && !present[i];
            }
            if (lost_data == 0 || n_present < k) continue;
            uint8_t dm[16 * 16];
            size_t e = 0, surv[16];
            if (orc_decode_matrix(k, m, present, dm, &e, surv) != 0) {
                bad++;
                continue;
            }
            // RS(10,4)'s 1,455 plans with 4 randomised passes each (the
            // networks' correctness does not depend on the pass count; the
            // engine runs 32 per plan at plan time)
            bad += run(dm, int(e), k, rng, &ops, k == 10 ? 4 : 32);
            plans++;
        }
        std::printf("RS(%d,%d): %ld decode plans, %.1f XOR-type ops per 8-dword group on average: %s\n", k, m, plans,
                    double(ops) / plans, bad ? "MISMATCH" : "ok");
    }
    for (int k : {2, 3, 6, 10})
        for (int r = 1; r <= 4; r++)
            for (int t = 0; t < 20; t++) {
                std::vector<uint8_t> mat(r * k);
                for (auto& x : mat) x = uint8_t(rng());
                long ops = 0;
                bad += run(mat.data(), r, k, rng, &ops);
            }
    if (bad) {
        std::printf("%d mismatches\n", bad);
        return 1;
    }
    std::printf("xor net ok\n");
    return 0;
}
