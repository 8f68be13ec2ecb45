// xor_net.hpp -- plan-time bit-sliced XOR networks for an arbitrary GF(2^8)
// coefficient matrix (host code).  The run-time counterpart of
// scripts/gen_xor_networks.py, which generates xor_networks.hpp for the fixed
// RS parity rows at build time: the decode + verify kernel's matrix is the
// decode plan's (rows of inverse(select_rows(encode_matrix, survivors)),
// gf256.rs:113-122), known only when the erasure pattern is, so jit.cpp
// builds its network here and compiles the fused kernel with it (hiprtc).
//
// Multiplication by c in GF(2^8)/0x11D is GF(2)-linear on a byte: output bit
// t = XOR over input bits b with bit t of c * x^b set.  With the data
// bit-sliced (plane b of an 8-dword group = bit b of each of its 32 bytes,
// bitslice.hpp), an r-row matrix is a fixed XOR network over the k * 8 input
// planes.  The kernel streams one input shard at a time, so the network is
// built per input: pairs of input planes that several outputs share are
// XORed once first (greedy common-subexpression pairing, Paar's heuristic,
// as the Python generator, extended to triples: a 3-input XOR temp removes two
// terms per output for one op), then every output plane absorbs its terms two
// at a time through a 3-input XOR; input 0 initialises the accumulators.  A
// few randomised greedy passes are tried and the cheapest network kept.
#pragma once

#include <algorithm>
#include <array>
#include <random>
#include <cstdint>
#include <map>
#include <set>
#include <string>
#include <utility>
#include <vector>

#include "gf256.hpp"

namespace hec {
namespace xornet {

// Operand ids: 0..7 = input plane p[b]; 8 + t = temporary t.
struct InputNet {
    std::vector<std::array<int, 3>> temps;  // temp t = a ^ b (^ c when c >= 0); operands < 8 + t
    std::vector<std::vector<int>> absorb;   // per output plane 8*j + t: the operands it takes in
};

// bit t of c * x^b, as the set of input bits b feeding output bit t
inline std::vector<std::set<int>> bit_rows(uint8_t c) {
    uint8_t cols[8];
    for (int b = 0; b < 8; b++) cols[b] = gf_mul(c, uint8_t(1u << b));
    std::vector<std::set<int>> rows(8);
    for (int t = 0; t < 8; t++)
        for (int b = 0; b < 8; b++)
            if ((cols[b] >> t) & 1) rows[t].insert(b);
    return rows;
}

// VALU ops to fold n terms into an output plane with 3-input XORs; input 0
// initialises the plane (one op takes up to three terms, a single term is a move)
inline int absorb_cost(int n, bool first) {
    if (first) return n <= 1 ? 0 : 1 + (std::max(0, n - 3) + 1) / 2;
    return (n + 1) / 2;
}

// One greedy pass: repeatedly factor out the pair or triple of operands whose
// shared XOR saves the most ops over the outputs that contain it (a temp
// costs one op; a triple removes two terms per output, a pair one), ties and
// near-ties broken by `rng` (temperature `temp`); stops when nothing saves.
inline InputNet greedy_network(std::vector<std::set<int>> outs, bool first, std::mt19937* rng, double temp) {
    InputNet net;
    for (;;) {
        std::map<std::array<int, 3>, int> cnt;  // {a, b, c} (c = -1: pair) -> outputs holding it
        for (auto& o : outs) {
            const std::vector<int> v(o.begin(), o.end());
            for (size_t a = 0; a < v.size(); a++)
                for (size_t b = a + 1; b < v.size(); b++) {
                    cnt[{v[a], v[b], -1}]++;
                    for (size_t c = b + 1; c < v.size(); c++) cnt[{v[a], v[b], v[c]}]++;
                }
        }
        std::vector<std::pair<int, std::array<int, 3>>> scored;
        int best = 0;
        for (auto& [t, n] : cnt) {
            if (n < 2) continue;
            const int len = t[2] < 0 ? 2 : 3;
            int save = -1;
            for (auto& o : outs)
                if (o.count(t[0]) && o.count(t[1]) && (t[2] < 0 || o.count(t[2])))
                    save += absorb_cost(int(o.size()), first) - absorb_cost(int(o.size()) - len + 1, first);
            if (save > 0) {
                scored.push_back({save, t});
                best = std::max(best, save);
            }
        }
        if (scored.empty()) break;
        const int floor = (rng && std::uniform_real_distribution<double>(0, 1)(*rng) < temp) ? best - 1 : best;
        std::vector<std::array<int, 3>> pool;
        for (auto& [sv, t] : scored)
            if (sv >= floor && sv > 0) pool.push_back(t);
        const auto pick = rng ? pool[std::uniform_int_distribution<size_t>(0, pool.size() - 1)(*rng)] : pool.front();
        const int name = 8 + int(net.temps.size());
        net.temps.push_back(pick);
        for (auto& o : outs)
            if (o.count(pick[0]) && o.count(pick[1]) && (pick[2] < 0 || o.count(pick[2]))) {
                o.erase(pick[0]);
                o.erase(pick[1]);
                if (pick[2] >= 0) o.erase(pick[2]);
                o.insert(name);
            }
    }
    for (auto& o : outs) net.absorb.emplace_back(o.begin(), o.end());
    return net;
}

inline int input_cost(const InputNet& net, bool first) {
    int ops = int(net.temps.size());
    for (auto& terms : net.absorb) ops += absorb_cost(int(terms.size()), first);
    return ops;
}

// coefs[j] = this input's coefficient in output row j (r rows).  The
// deterministic greedy plus `restarts` randomised passes (fixed seed); the
// cheapest network wins.
inline InputNet input_network(const uint8_t* coefs, int r, bool first, int restarts = 32) {
    std::vector<std::set<int>> outs;
    for (int j = 0; j < r; j++)
        for (auto& s : bit_rows(coefs[j])) outs.push_back(s);
    InputNet best = greedy_network(outs, first, nullptr, 0.0);
    int best_cost = input_cost(best, first);
    std::mt19937 rng(0x5EED + r);
    for (int t = 0; t < restarts; t++) {
        InputNet n = greedy_network(outs, first, &rng, 0.3);
        const int c = input_cost(n, first);
        if (c < best_cost) {
            best = std::move(n);
            best_cost = c;
        }
    }
    return best;
}

// The k inputs' networks of an r x k matrix (row-major).
inline std::vector<InputNet> matrix_network(const uint8_t* matrix, int r, int k, int restarts = 32) {
    std::vector<InputNet> nets;
    std::vector<uint8_t> col(r);
    for (int i = 0; i < k; i++) {
        for (int j = 0; j < r; j++) col[j] = matrix[j * k + i];
        nets.push_back(input_network(col.data(), r, i == 0, restarts));
    }
    return nets;
}

// XOR-type VALU ops per 8-dword group over all inputs (the kernel's cost).
inline int network_ops(const std::vector<InputNet>& nets) {
    int ops = 0;
    for (size_t i = 0; i < nets.size(); i++) ops += input_cost(nets[i], i == 0);
    return ops;
}

// Host evaluation of input i's network on its 8 planes (checks, tests).
inline void eval_input(const InputNet& net, bool first, const uint32_t (&p)[8], uint32_t* acc) {
    std::vector<uint32_t> v(8 + net.temps.size());
    for (int b = 0; b < 8; b++) v[b] = p[b];
    for (size_t t = 0; t < net.temps.size(); t++) {
        const auto& q = net.temps[t];
        v[8 + t] = v[q[0]] ^ v[q[1]] ^ (q[2] >= 0 ? v[q[2]] : 0u);
    }
    for (size_t o = 0; o < net.absorb.size(); o++) {
        uint32_t x = first ? 0u : acc[o];
        for (int id : net.absorb[o]) x ^= v[id];
        acc[o] = x;
    }
}

// The device source of input i's network: a specialisation of
// `Net::absorb<I>` (the struct the JIT source declares) in the style of
// xor_networks.hpp.
inline std::string emit_input(const InputNet& net, int i, int r) {
    auto opnd = [](int id) { return id < 8 ? "p[" + std::to_string(id) + "]" : "t" + std::to_string(id - 8); };
    std::string s = "template <> __device__ __forceinline__ void Net::absorb<" + std::to_string(i) +
                    ">(const uint32_t (&p)[8], uint32_t (&acc)[" + std::to_string(8 * r) + "]) {\n";
    for (size_t t = 0; t < net.temps.size(); t++) {
        const auto& q = net.temps[t];
        s += "    const uint32_t t" + std::to_string(t) + " = " +
             (q[2] >= 0 ? "bitslice::x3(" + opnd(q[0]) + ", " + opnd(q[1]) + ", " + opnd(q[2]) + ")"
                        : opnd(q[0]) + " ^ " + opnd(q[1])) +
             ";\n";
    }
    for (size_t o = 0; o < net.absorb.size(); o++) {
        std::vector<int> terms = net.absorb[o];
        const std::string a = "acc[" + std::to_string(o) + "]";
        size_t q = 0;
        if (i == 0) {
            if (terms.empty()) {
                s += "    " + a + " = 0u;\n";
                continue;
            }
            if (terms.size() == 1) {
                s += "    " + a + " = " + opnd(terms[0]) + ";\n";
                q = 1;
            } else if (terms.size() == 2) {
                s += "    " + a + " = " + opnd(terms[0]) + " ^ " + opnd(terms[1]) + ";\n";
                q = 2;
            } else {
                s += "    " + a + " = bitslice::x3(" + opnd(terms[0]) + ", " + opnd(terms[1]) + ", " + opnd(terms[2]) +
                     ");\n";
                q = 3;
            }
        }
        while (q < terms.size()) {
            if (terms.size() - q >= 2) {
                s += "    " + a + " = bitslice::x3(" + a + ", " + opnd(terms[q]) + ", " + opnd(terms[q + 1]) + ");\n";
                q += 2;
            } else {
                s += "    " + a + " ^= " + opnd(terms[q]) + ";\n";
                q++;
            }
        }
    }
    s += "}\n";
    return s;
}

}  // namespace xornet
}  // namespace hec
