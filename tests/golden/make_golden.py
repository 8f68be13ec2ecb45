"""Generates tests/golden/*.npz -- committed golden vectors for the EC path.

The reference (Rust) cannot be built or run in this image (no cargo/rustc;
the g2p crate is not vendored), so the vectors come from the two CPU
restatements in oracle/ (C and pure Python), which must agree byte for byte
and which are themselves pinned by the reference's KATs
(rust/src/ec/gf256.rs:144-202, rust/src/ec/mod.rs:152-160) in
tests/test_oracle.py.  Re-run:  python tests/golden/make_golden.py
"""
from __future__ import annotations

import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
sys.path.insert(0, os.path.join(ROOT, "hdfs-native_amd"))

import ec_oracle as O  # noqa: E402
from hdfs_native_ec.synth import bench_counter_shards, splitmix64_bytes, SEED_BASE  # noqa: E402

OUT = os.path.dirname(os.path.abspath(__file__))

SCHEMES = [(3, 2), (6, 3), (10, 4)]
LENGTHS = [1, 15, 16, 17, 4093, 4096]


def main() -> None:
    clib = O.load_c_oracle()
    manifest = {"generator": "tests/golden/make_golden.py", "cases": []}
    arrays = {}
    for k, m in SCHEMES:
        for n in LENGTHS:
            data = splitmix64_bytes(SEED_BASE + 1000 * k + n, k * n).reshape(k, n)
            par_py = O.encode(k, m, list(data))
            par_c = O.c_encode(clib, k, m, list(data))
            for a, b in zip(par_py, par_c):
                assert np.array_equal(a, b), (k, m, n)
            key = f"rs{k}_{m}_n{n}"
            arrays[key + "_data"] = data
            arrays[key + "_parity"] = np.stack(par_py)
            manifest["cases"].append({"key": key, "k": k, "m": m, "n": n, "fill": "splitmix64",
                                      "seed": SEED_BASE + 1000 * k + n})
        # reference bench fill (benches/ec.rs:19-27), 4 KiB slices
        n = 4096
        data = bench_counter_shards(k, n)
        par = O.encode(k, m, list(data))
        assert all(np.array_equal(a, b) for a, b in zip(par, O.c_encode(clib, k, m, list(data))))
        key = f"rs{k}_{m}_counter"
        arrays[key + "_data"] = data
        arrays[key + "_parity"] = np.stack(par)
        manifest["cases"].append({"key": key, "k": k, "m": m, "n": n, "fill": "bench_counter_be_i32"})
        # decode matrices for every erasure pattern of up to m data shards
        # (worst case) -- e x k rows, survivors = first k present
        plans = []
        import itertools
        for e in range(1, m + 1):
            for miss in itertools.combinations(range(k), e):
                present = [i not in miss for i in range(k + m)]
                surv, inval, dm = O.decode_plan(k, m, present)
                plans.append({"missing": list(miss), "survivors": surv, "matrix": dm})
        manifest[f"rs{k}_{m}_decode_plans"] = plans
    np.savez(os.path.join(OUT, "ec_vectors.npz"), **arrays)
    with open(os.path.join(OUT, "ec_vectors.json"), "w") as f:
        json.dump(manifest, f, indent=0, separators=(",", ":"))
    print("wrote", len(arrays), "arrays")


if __name__ == "__main__":
    main()
