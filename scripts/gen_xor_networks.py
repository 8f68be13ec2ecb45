#!/usr/bin/env python3
"""Generates hdfs-native_amd/csrc/xor_networks.hpp: the bit-sliced XOR
networks of the Hadoop RS parity rows (Coder::gen_rs_matrix,
rust/src/ec/gf256.rs:40-57) for RS(2,1), RS(3,2), RS(6,3) and RS(10,4).

Multiplication by a constant c in GF(2^8)/0x11D is GF(2)-linear on a byte:
output bit t = XOR over input bits b of M_c[t][b], with M_c[t][b] = bit t of
c * x^b.  With the data bit-sliced -- plane b of an 8-dword group holds bit b
of each of its 32 bytes -- a parity row is a fixed XOR network over the k*8
input planes, and the engine's fused encode + CRC kernel (ec_fused.hip) runs
it instead of the v_perm product tables.  The kernel streams one input shard
at a time, so the network is emitted per input: input i's 8 planes are folded
into the r*8 accumulator planes; pairs of input planes that several outputs
share are XORed once first (greedy common-subexpression pairing, Paar's
heuristic, extended to triples: a 3-input XOR temp removes two terms per
output for one op; seeded randomised greedy passes, the cheapest kept), then
every accumulator absorbs its terms two at a time through a 3-input XOR.
Input 0 initialises the accumulators.

usage: python3 scripts/gen_xor_networks.py > hdfs-native_amd/csrc/xor_networks.hpp
"""
import collections
import itertools
import random


def gf_mul(a, b):
    r = 0
    for i in range(8):
        if b & (1 << i):
            r ^= a
        a <<= 1
        if a & 0x100:
            a ^= 0x11D
    return r


def gf_inv(a):
    return next(x for x in range(1, 256) if gf_mul(a, x) == 1)


def rs_parity_rows(k, m):
    # gf256.rs:40-57: row r >= k, col c: 1 / (r ^ c) (0 when r == c)
    return [[0 if (r ^ c) == 0 else gf_inv(r ^ c) for c in range(k)] for r in range(k, k + m)]


def bit_rows(c):
    # M_c[t] as a set of input bits b
    cols = [gf_mul(c, 1 << b) for b in range(8)]
    return [{b for b in range(8) if (cols[b] >> t) & 1} for t in range(8)]


def absorb_cost(n, first):
    """VALU ops to fold n terms into an output plane with 3-input XORs; input
    0 initialises the plane (one op takes up to three terms)."""
    if first:
        return 0 if n <= 1 else 1 + (max(0, n - 3) + 1) // 2
    return (n + 1) // 2


def greedy_network(outs, first, rng=None, temp=0.0):
    """Repeatedly factor out the pair or triple of operands whose shared XOR
    saves the most ops over the outputs holding it (a temp costs one op; a
    triple removes two terms per output, a pair one); ties and near-ties
    broken by rng.  Returns (temps, absorb)."""
    outs = [set(o) for o in outs]
    temps = []
    while True:
        cnt = collections.Counter()
        for o in outs:
            so = sorted(o)
            for t in itertools.combinations(so, 2):
                cnt[t] += 1
            for t in itertools.combinations(so, 3):
                cnt[t] += 1
        scored = []
        for t, n in cnt.items():
            if n < 2:
                continue
            save = -1
            for o in outs:
                if all(x in o for x in t):
                    save += absorb_cost(len(o), first) - absorb_cost(len(o) - len(t) + 1, first)
            if save > 0:
                scored.append((save, t))
        if not scored:
            break
        best = max(sv for sv, _ in scored)
        floor = best - 1 if rng is not None and rng.random() < temp else best
        pool = sorted(t for sv, t in scored if sv >= floor)
        pick = rng.choice(pool) if rng is not None else pool[0]
        name = f"t{len(temps)}"
        temps.append((name,) + tuple(pick))
        for o in outs:
            if all(x in o for x in pick):
                o.difference_update(pick)
                o.add(name)
    return temps, [sorted(o) for o in outs]


def input_cost(temps, absorb, first):
    return len(temps) + sum(absorb_cost(len(t), first) for t in absorb)


def input_network(coefs, first, restarts=48):
    """coefs[j] = coefficient of this input in parity row j.  Returns
    (temps, absorb): temps = [(name, a, b[, c])] 2- or 3-input XORs of
    planes / earlier temps; absorb[o] = the operands output plane o = 8*j + t
    takes in.  The deterministic greedy plus seeded randomised passes; the
    cheapest network wins (the plan-time generator, csrc/xor_net.hpp, does the
    same for decode matrices)."""
    outs = []
    for c in coefs:
        outs.extend(set(f"p[{b}]" for b in s) for s in bit_rows(c))
    best = greedy_network(outs, first)
    rng = random.Random(0x5EED + len(coefs))
    for _ in range(restarts):
        cand = greedy_network(outs, first, rng, 0.3)
        if input_cost(*cand, first) < input_cost(*best, first):
            best = cand
    return best


def emit_input(k, m, i, coefs):
    temps, absorb = input_network(coefs, i == 0)
    n = 8 * m
    lines = [f"template <> __host__ __device__ __forceinline__ void rs_absorb<{k}, {m}, {i}>("
             f"const uint32_t (&p)[8], uint32_t (&acc)[{n}]) {{"]
    ops = 0
    for name, *ops_in in temps:
        expr = f"x3({ops_in[0]}, {ops_in[1]}, {ops_in[2]})" if len(ops_in) == 3 else f"{ops_in[0]} ^ {ops_in[1]}"
        lines.append(f"    const uint32_t {name} = {expr};")
        ops += 1
    for o, terms in enumerate(absorb):
        terms = list(terms)
        if i == 0:
            if not terms:
                lines.append(f"    acc[{o}] = 0u;")
                continue
            if len(terms) == 1:
                cur = terms.pop(0)
            elif len(terms) == 2:
                cur = f"{terms.pop(0)} ^ {terms.pop(0)}"
                ops += 1
            else:
                cur = f"x3({terms.pop(0)}, {terms.pop(0)}, {terms.pop(0)})"
                ops += 1
            lines.append(f"    acc[{o}] = {cur};")
        while terms:
            if len(terms) >= 2:
                lines.append(f"    acc[{o}] = x3(acc[{o}], {terms.pop(0)}, {terms.pop(0)});")
            else:
                lines.append(f"    acc[{o}] ^= {terms.pop(0)};")
            ops += 1
    lines.append("}")
    return lines, ops


def main():
    out = ['// xor_networks.hpp -- GENERATED by scripts/gen_xor_networks.py; do not edit.',
           '// Bit-sliced XOR networks of the RS parity rows (gf256.rs:40-57) per input',
           '// shard: rs_absorb<K, R, I>(p, acc) folds input I\'s 8 bit planes p into the',
           '// R*8 accumulator planes (plane 8*j + t = bit t of parity row j); I = 0',
           '// initialises them.  See the generator for the construction.',
           '#pragma once', '', '#include <cstdint>', '', 'namespace hec {', 'namespace bitslice {', '',
           '__host__ __device__ __forceinline__ uint32_t x3(uint32_t a, uint32_t b, uint32_t c) {',
           '#if defined(__HIP_DEVICE_COMPILE__)',
           '    return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);',
           '#else',
           '    return a ^ b ^ c;',
           '#endif',
           '}', '',
           'template <int K, int R, int I>',
           '__host__ __device__ void rs_absorb(const uint32_t (&p)[8], uint32_t (&acc)[R * 8]);', '',
           '// (K, R) with a generated network',
           'template <int K, int R>',
           'constexpr bool rs_net_available() {',
           '    return (K == 2 && R == 1) || (K == 3 && R == 2) || (K == 6 && R == 3) || (K == 10 && R == 4);',
           '}', '']
    summary = []
    for k, m in [(2, 1), (3, 2), (6, 3), (10, 4)]:
        rows = rs_parity_rows(k, m)
        total = 0
        out.append(f"// ---- RS({k},{m}): parity rows {rows}")
        for i in range(k):
            lines, ops = emit_input(k, m, i, [rows[j][i] for j in range(m)])
            total += ops
            out.extend(lines)
            out.append("")
        out.append(f"constexpr int kRsNetOps_{k}_{m} = {total};  // XOR-type ops per 8-dword group, all inputs")
        out.append("")
        summary.append((k, m, total))
    out += ['// rs_absorb<K, R, i> for a loop index i that is constant after unrolling',
            'template <int K, int R, int I = 0>',
            '__host__ __device__ __forceinline__ void rs_absorb_at(int i, const uint32_t (&p)[8], uint32_t (&acc)[R * 8]) {',
            '    if constexpr (I < K) {',
            '        if (i == I)',
            '            rs_absorb<K, R, I>(p, acc);',
            '        else',
            '            rs_absorb_at<K, R, I + 1>(i, p, acc);',
            '    }',
            '}', '',
            '}  // namespace bitslice', '}  // namespace hec']
    print("\n".join(out))
    import sys
    for k, m, t in summary:
        print(f"RS({k},{m}): {t} ops per 8-dword group", file=sys.stderr)


if __name__ == "__main__":
    main()
