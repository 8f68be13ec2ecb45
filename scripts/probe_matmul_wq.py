"""Measurement probe (GPU box): the register kernel's fixed tile order (tune
key 27 = 3; the default before round 5) against its work queue of wave-tiles
(key 27 = 1 / 2 rounds per atomic over 8 launch counters; the default is 2 for
k <= 3, 1 for k = 6, 10), measurement build, on the bench's uniform step: encode, then decode with data shards 0..m-1 lost.  Same process, same
buffers, rounds alternated, HIP events around REPS back-to-back steps
(median); two fresh buffer sets per config; outputs checked against the
fixed order's.
  python3 scripts/probe_matmul_wq.py
"""
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "hdfs-native_amd"))

import torch  # noqa: E402

import hdfs_native_ec as H  # noqa: E402

CELL = 1 << 20
CONFIGS = [(6, 3, 1024), (10, 4, 256), (3, 2, 1024)]
SETS = int(os.environ.get("PROBE_SETS", "2"))
ROUNDS = int(os.environ.get("PROBE_ROUNDS", "5"))
REPS = int(os.environ.get("PROBE_REPS", "6"))
VARIANTS = [("fixed order", 3), ("queue x1", 1), ("queue x2", 2)]
# PROBE_C64K=1: RS(6,3) 64 KiB cells x 65536 (BASELINE configs[4]): the LDS-DMA
# kernel (the small-cell default, fixed order) against the register kernel on the
# queue (tune key 5 = 1) and in the fixed order (5 = 1, 27 = 3)
C64K = os.environ.get("PROBE_C64K") == "1"
if C64K:
    CONFIGS = [(6, 3, 65536, 1 << 16)]
    if os.environ.get("PROBE_CELLS"):  # e.g. "8192:131072,262144:8192": cell:stripes, one set each
        CONFIGS = [(6, 3, int(x.split(":")[1]), int(x.split(":")[0])) for x in os.environ["PROBE_CELLS"].split(",")]
        SETS = 1
    VARIANTS = [("LDS-DMA", [(5, 0)]), ("register queue", [(5, 1)]), ("register fixed", [(5, 1), (27, 3)])]
# PROBE_BPC=1: RS(6,3) / RS(3,2) on the queue at 1 block per CU (the default)
# against 2 (key 3 = 2: two waves per SIMD)
if os.environ.get("PROBE_BPC") == "1":
    CONFIGS = [(6, 3, 1024), (3, 2, 1024)]
    VARIANTS = [("queue 1/CU", [(27, 0)]), ("queue 2/CU", [(27, 0), (3, 2)]), ("queue x2 2/CU", [(27, 2), (3, 2)])]
# PROBE_GROUP=1: the tile-order group (tune key 8: stripes interleaved
# column-major; default 4) on the queue
if os.environ.get("PROBE_GROUP") == "1":
    CONFIGS = [(6, 3, 1024), (10, 4, 256)]
    VARIANTS = [("group 4", [(27, 0)]), ("group 1", [(27, 0), (8, 1)]), ("group 2", [(27, 0), (8, 2)]),
                ("group 8", [(27, 0), (8, 8)]), ("group 16", [(27, 0), (8, 16)])]
# PROBE_K10=1: RS(10,4) only, its 512-thread shape against 256-thread blocks
# (tune keys 4 = 256, 1 = 2) at 1 and 2 blocks per CU (key 3), all on the queue
K10 = os.environ.get("PROBE_K10") == "1"
if K10:
    CONFIGS = [(10, 4, 256), (10, 4, 1024)]
    VARIANTS = [("512 x1/CU", [(27, 1)]), ("256 U4 x1/CU", [(27, 1), (4, 256), (1, 4)]),
                ("256 U4 x2/CU", [(27, 1), (4, 256), (1, 4), (3, 2)]), ("256 x2/CU", [(27, 1), (4, 256), (1, 2), (3, 2)])]

# PROBE_PAIR=1 (round 6): RS(10,4) on the wave-pair kernel (tune key 32 = 1:
# two waves per wave-tile, 5 inputs x 4 KiB each, partials exchanged in LDS)
# at 4 and 2 blocks of 128 threads per CU against the 512-thread default
if os.environ.get("PROBE_PAIR") == "1":
    CONFIGS = [(10, 4, 256), (10, 4, 1024)]
    VARIANTS = [("512 x1/CU", [(27, 0)]), ("pair x4/CU", [(32, 1)]), ("pair x2/CU", [(32, 1), (3, 2)]),
                ("pair x3/CU", [(32, 1), (3, 3)])]

# PROBE_BSL=1 (round 6): RS(10,4) encode with the RS parity rows as bit-
# sliced XOR networks (tune key 23 = 1, gf_encode_bsl, fixed tile order; the
# decode keeps the v_perm tables) against the v_perm encode on the queue
# (default) and in the fixed order (key 27 = 3)
if os.environ.get("PROBE_BSL") == "1":
    CONFIGS = [(10, 4, 256), (10, 4, 1024), (6, 3, 1024)]
    VARIANTS = [("v_perm queue", [(27, 0)]), ("v_perm fixed", [(27, 3)]), ("bsl fixed", [(23, 1)])]

# PROBE_K10OCC=1 (round 6): RS(10,4) register kernel (76 VGPRs) on the queue
# at more resident waves: 512-thread blocks at 2 / 3 per CU (4 / 6 waves per
# SIMD) and 256-thread blocks at 4 / 6 per CU, against the default 1 x 512
if os.environ.get("PROBE_K10OCC") == "1":
    CONFIGS = [(10, 4, 256), (10, 4, 1024)]
    VARIANTS = [("512 x1/CU", [(27, 0)]), ("512 x2/CU", [(3, 2)]), ("512 x3/CU", [(3, 3)]),
                ("256 x4/CU", [(4, 256), (1, 2), (3, 4)]), ("256 x6/CU", [(4, 256), (1, 2), (3, 6)])]


def main():
    dev = torch.device("cuda:0")
    stream = torch.cuda.current_stream()
    lib = H.experimental_lib()
    g = torch.Generator(device=dev)
    g.manual_seed(9)
    cases = []
    for cfg in CONFIGS:
        k, m, S = cfg[:3]
        cell = cfg[3] if len(cfg) > 3 else CELL
        coder = H.Coder(k, m, 0, lib=lib)
        for si in range(SETS):
            d = torch.empty((S, k, cell), dtype=torch.uint8, device=dev)
            d.random_(0, 256, generator=g)
            ps = [torch.empty((S, m, cell), dtype=torch.uint8, device=dev) for _ in VARIANTS]
            rs = [torch.empty((S, k, cell), dtype=torch.uint8, device=dev) for _ in VARIANTS]
            cases.append(dict(name=f"RS({k},{m}) {cell >> 10} KiB x {S} set {si}", coder=coder, d=d, ps=ps, rs=rs,
                              m=m, bytes=2 * (k + m) * S * cell, t={v: [] for v, _ in VARIANTS}))
    torch.cuda.synchronize()

    def step(c, i, wq):
        pairs = wq if isinstance(wq, list) else [(27, wq)]
        for key, val in pairs:
            H.tune_set(key, val, lib)
        H.encode_batch(c["coder"], c["d"], c["ps"][i], stream)
        H.decode_batch(c["coder"], c["d"], c["ps"][i], list(range(c["m"])), c["rs"][i], stream)
        for key, _ in pairs:
            H.tune_set(key, -1 if key == 2 else 0, lib)

    for c in cases:
        for i, (_, wq) in enumerate(VARIANTS):
            step(c, i, wq)
        torch.cuda.synchronize()
        m = c["m"]
        for i in range(len(VARIANTS)):
            assert torch.equal(c["ps"][i], c["ps"][0]), (c["name"], VARIANTS[i][0])
            assert torch.equal(c["rs"][i][:, :m], c["d"][:, :m]), (c["name"], VARIANTS[i][0])
    for _ in range(ROUNDS):
        for c in cases:
            for i, (v, wq) in enumerate(VARIANTS):
                step(c, i, wq)
                a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                a.record(stream)
                for _ in range(REPS):
                    step(c, i, wq)
                b.record(stream)
                torch.cuda.synchronize()
                c["t"][v].append(a.elapsed_time(b) / REPS)
    for c in cases:
        parts = []
        for v, ts in c["t"].items():
            med = statistics.median(ts)
            parts.append(f"{v} {med:.4f} ms/step ({c['bytes'] / (med * 1e-3) / 8e12:.3f})")
        print(f"{c['name']:22s} " + "  ".join(parts), flush=True)


if __name__ == "__main__":
    main()
