// bitslice_check.cpp -- the bit-sliced RS parity path of the fused encode +
// CRC kernel, on the host: transpose8 (hdfs-native_amd/csrc/bitslice.hpp) is
// an involution that turns 8 dwords into bit planes, and the generated XOR
// networks (csrc/xor_networks.hpp, scripts/gen_xor_networks.py) fed one input
// shard at a time, then transposed back, equal the RS parity of every byte
// (gf256.rs:40-80 restated by the oracle, oracle/ec_oracle.c) for RS(2,1),
// RS(3,2), RS(6,3) and RS(10,4).  Run by tests/test_host_gf.py (CPU).
#include <cstdio>
#include <cstring>
#include <random>

#define __host__
#define __device__
#define __forceinline__ inline
#include "../../hdfs-native_amd/csrc/bitslice.hpp"
#include "../../hdfs-native_amd/csrc/gf256.hpp"
#include "../../hdfs-native_amd/csrc/xor_networks.hpp"

extern "C" int orc_encode(size_t k, size_t m, const uint8_t* const* data, size_t n, uint8_t* const* parity);

using namespace hec::bitslice;

template <int K, int R>
int check(std::mt19937& rng) {
    int bad = 0;
    for (int trial = 0; trial < 200; trial++) {
        uint32_t in[K][8], acc[R * 8];
        for (int i = 0; i < K; i++)
            for (int w = 0; w < 8; w++) in[i][w] = trial == 0 ? 0xFFFFFFFFu : trial == 1 ? 0u : uint32_t(rng());
        for (int i = 0; i < K; i++) {
            uint32_t p[8];
            std::memcpy(p, in[i], sizeof(p));
            transpose8(p);
            rs_absorb_at<K, R>(i, p, acc);
        }
        // oracle: the 32 bytes of each shard as one shard of 32 bytes
        uint8_t data[K][32], want[R][32];
        const uint8_t* dp[K];
        uint8_t* wp[R];
        for (int i = 0; i < K; i++) {
            std::memcpy(data[i], in[i], 32);
            dp[i] = data[i];
        }
        for (int j = 0; j < R; j++) wp[j] = want[j];
        orc_encode(K, R, dp, 32, wp);
        for (int j = 0; j < R; j++) {
            uint32_t q[8];
            std::memcpy(q, acc + 8 * j, sizeof(q));
            transpose8(q);
            if (std::memcmp(q, want[j], 32) != 0) bad++;
        }
    }
    std::printf("RS(%d,%d): %s\n", K, R, bad ? "MISMATCH" : "ok");
    return bad;
}

int main() {
    std::mt19937 rng(7);
    int bad = 0;
    // transpose8 is an involution, and plane b byte y bit w = bit b of byte y of row w
    for (int t = 0; t < 1000; t++) {
        uint32_t d[8], e[8];
        for (auto& x : d) x = uint32_t(rng());
        std::memcpy(e, d, sizeof(d));
        transpose8(e);
        for (int b = 0; b < 8; b++)
            for (int y = 0; y < 4; y++)
                for (int w = 0; w < 8; w++)
                    if (((e[b] >> (8 * y + w)) & 1u) != ((d[w] >> (8 * y + b)) & 1u)) bad++;
        transpose8(e);
        if (std::memcmp(d, e, sizeof(d)) != 0) bad++;
    }
    std::printf("transpose8: %s\n", bad ? "MISMATCH" : "ok");
    bad += check<2, 1>(rng);
    bad += check<3, 2>(rng);
    bad += check<6, 3>(rng);
    bad += check<10, 4>(rng);
    if (bad) return 1;
    std::printf("bitslice ok\n");
    return 0;
}
