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
// as the Python generator), then every output plane absorbs its terms two at
// a time through a 3-input XOR; input 0 initialises the accumulators.
#pragma once

#include <algorithm>
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
    std::vector<std::pair<int, int>> temps;  // temp t = a ^ b (operands < 8 + t)
    std::vector<std::vector<int>> absorb;    // per output plane 8*j + t: the operands it takes in
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

// coefs[j] = this input's coefficient in output row j (r rows)
inline InputNet input_network(const uint8_t* coefs, int r) {
    std::vector<std::set<int>> outs;
    for (int j = 0; j < r; j++)
        for (auto& s : bit_rows(coefs[j])) outs.push_back(s);
    InputNet net;
    for (;;) {
        std::map<std::pair<int, int>, int> cnt;
        for (auto& o : outs)
            for (auto a = o.begin(); a != o.end(); ++a)
                for (auto b = std::next(a); b != o.end(); ++b) cnt[{*a, *b}]++;
        std::pair<int, int> best{-1, -1};
        int n = 1;
        for (auto& [pr, c] : cnt)
            if (c > n) {
                n = c;
                best = pr;
            }
        if (best.first < 0) break;  // no pair shared by two outputs
        const int name = 8 + int(net.temps.size());
        net.temps.push_back(best);
        for (auto& o : outs)
            if (o.count(best.first) && o.count(best.second)) {
                o.erase(best.first);
                o.erase(best.second);
                o.insert(name);
            }
    }
    for (auto& o : outs) net.absorb.emplace_back(o.begin(), o.end());
    return net;
}

// The k inputs' networks of an r x k matrix (row-major).
inline std::vector<InputNet> matrix_network(const uint8_t* matrix, int r, int k) {
    std::vector<InputNet> nets;
    std::vector<uint8_t> col(r);
    for (int i = 0; i < k; i++) {
        for (int j = 0; j < r; j++) col[j] = matrix[j * k + i];
        nets.push_back(input_network(col.data(), r));
    }
    return nets;
}

// XOR-type VALU ops per 8-dword group over all inputs (the kernel's cost).
inline int network_ops(const std::vector<InputNet>& nets) {
    int ops = 0;
    for (size_t i = 0; i < nets.size(); i++) {
        ops += int(nets[i].temps.size());
        for (auto& terms : nets[i].absorb) {
            int n = int(terms.size());
            if (i == 0) {  // initialisation: one op folds up to three terms
                if (n <= 1) continue;
                ops++;
                n -= 3;
            }
            if (n > 0) ops += (n + 1) / 2;
        }
    }
    return ops;
}

// Host evaluation of input i's network on its 8 planes (checks, tests).
inline void eval_input(const InputNet& net, bool first, const uint32_t (&p)[8], uint32_t* acc) {
    std::vector<uint32_t> v(8 + net.temps.size());
    for (int b = 0; b < 8; b++) v[b] = p[b];
    for (size_t t = 0; t < net.temps.size(); t++) v[8 + t] = v[net.temps[t].first] ^ v[net.temps[t].second];
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
    for (size_t t = 0; t < net.temps.size(); t++)
        s += "    const uint32_t t" + std::to_string(t) + " = " + opnd(net.temps[t].first) + " ^ " +
             opnd(net.temps[t].second) + ";\n";
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
