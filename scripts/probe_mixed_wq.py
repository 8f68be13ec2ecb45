"""Measurement probe (GPU box): the mixed-pattern decode's fixed tile order
(tune key 26 = 3; the default before round 5) against its work queue of
wave-tiles (key 26 = 1 / 2 / 4 rounds per atomic; the default is 1 for k >= 6,
4 below), measurement build, same process, same buffers, rounds alternated, HIP events
around REPS back-to-back launches (median).  Masks as bench.py
--decode-mode mixed: 1..m random data shards lost per stripe.  Per config two
fresh buffer sets.  Every variant's output is checked against the fixed
order's.
  python3 scripts/probe_mixed_wq.py
"""
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "hdfs-native_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

import hdfs_native_ec as H  # noqa: E402

CELL = 1 << 20
CONFIGS = [(10, 4, 256), (6, 3, 1024), (3, 2, 1024)]
SETS = int(os.environ.get("PROBE_SETS", "2"))
ROUNDS = int(os.environ.get("PROBE_ROUNDS", "5"))
REPS = int(os.environ.get("PROBE_REPS", "8"))
VARIANTS = [("fixed order", 3), ("queue x1", 1), ("queue x2", 2), ("queue x4", 4)]


def main():
    dev = torch.device("cuda:0")
    stream = torch.cuda.current_stream()
    lib = H.experimental_lib()
    g = torch.Generator(device=dev)
    g.manual_seed(7)
    cases = []
    for k, m, S in CONFIGS:
        coder = H.Coder(k, m, 0, lib=lib)
        rng = np.random.default_rng(0x5EED_EC00 + k)
        full = (1 << (k + m)) - 1
        masks, erased = [], 0
        for _ in range(S):
            e = int(rng.integers(1, m + 1))
            lost = rng.choice(k, size=e, replace=False)
            masks.append(full & ~sum(1 << int(i) for i in lost))
            erased += e
        for si in range(SETS):
            d = torch.empty((S, k, CELL), dtype=torch.uint8, device=dev)
            d.random_(0, 256, generator=g)
            p = torch.empty((S, m, CELL), dtype=torch.uint8, device=dev)
            H.encode_batch(coder, d, p)
            outs = [torch.zeros((S, k, CELL), dtype=torch.uint8, device=dev) for _ in VARIANTS]
            ws = torch.empty(coder.decode_mixed_workspace_size(S), dtype=torch.uint8, device=dev)
            cases.append(dict(name=f"RS({k},{m}) x {S} set {si}", coder=coder, d=d, p=p, outs=outs, ws=ws,
                              masks=masks, bytes=(k * S + erased) * CELL, t={v: [] for v, _ in VARIANTS}))
    torch.cuda.synchronize()

    def run(c, i, wq):
        H.tune_set(26, wq, lib)
        H.decode_batch_mixed(c["coder"], c["d"], c["p"], c["masks"], c["outs"][i], stream, c["ws"])
        H.tune_set(26, 0, lib)

    for c in cases:  # correctness: every variant rebuilds the same cells
        for i, (_, wq) in enumerate(VARIANTS):
            run(c, i, wq)
        torch.cuda.synchronize()
        for i in range(1, len(VARIANTS)):
            assert torch.equal(c["outs"][i], c["outs"][0]), (c["name"], VARIANTS[i][0])
        lost = torch.tensor([[not (mk >> j) & 1 for j in range(c["d"].shape[1])] for mk in c["masks"]], device=dev)
        assert bool(((c["outs"][0] == c["d"]) | ~lost[:, :, None]).all()), c["name"]
    for _ in range(ROUNDS):
        for c in cases:
            for i, (v, wq) in enumerate(VARIANTS):
                run(c, i, wq)
                a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                a.record(stream)
                for _ in range(REPS):
                    run(c, i, wq)
                b.record(stream)
                torch.cuda.synchronize()
                c["t"][v].append(a.elapsed_time(b) / REPS)
    for c in cases:
        parts = []
        for v, ts in c["t"].items():
            med = statistics.median(ts)
            parts.append(f"{v} {med:.4f} ms ({c['bytes'] / (med * 1e-3) / 8e12:.3f})")
        print(f"{c['name']:22s} " + "  ".join(parts), flush=True)


if __name__ == "__main__":
    main()
