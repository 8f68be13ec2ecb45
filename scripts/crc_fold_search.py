"""Searches sparse multiples of the CRC32C polynomial for the fold (DESIGN.md
§3.5, checksum_device.hpp quarter_fold): weight-6 polynomials sum_{t in T}
x^t = 0 mod P with degree <= argv[1], by colliding XORs of the residues
x^t mod P over triples (numpy sort).  Prints the shortest, with the fold
offsets D - t and their bit shifts mod 32.  CPU only; about 30 s at 300.
usage: python3 scripts/crc_fold_search.py 300"""
import numpy as np, itertools, sys
P = (1 << 32) | 0x1EDC6F41
def mulx(r):
    r <<= 1
    if r >> 32: r ^= P
    return r
Dmax = int(sys.argv[1])
res = [1]
for t in range(1, Dmax + 1): res.append(mulx(res[-1]))
res = np.array(res, dtype=np.uint64)
idx = np.array(list(itertools.combinations(range(Dmax + 1), 3)), dtype=np.int32)
v = res[idx[:, 0]] ^ res[idx[:, 1]] ^ res[idx[:, 2]]
o = np.argsort(v, kind="stable"); vs = v[o]
dup = np.nonzero(vs[1:] == vs[:-1])[0]
found = set()
for d in dup:
    a = idx[o[d]]; b = idx[o[d + 1]]
    T = set(a.tolist()) ^ set(b.tolist())
    if len(T) != 6: continue
    T = sorted(T); m = T[0]; T = tuple(t - m for t in T)
    found.add(T)
good = sorted(found, key=lambda T: (T[-1], -(T[-1] - T[-2])))
print(len(found))
for T in good[:12]:
    D = T[-1]; offs = [D - t for t in T[:-1]]
    print(D, T, "offsets", offs, "min gap", D - T[-2], "s", [o % 32 for o in offs])
