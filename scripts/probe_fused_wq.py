"""Measurement probe (GPU box): the fused encode + CRC32C kernel with its
block tiles (tune key 28 = 2; the default at k = 6) against the work queue
of wave-tiles (key 28 = 1; the default at k = 3 and 10), measurement build;
and the plan-specialised decode {0..m-1} + verify the same two ways (key 28
= 1 compiles its work-queue form, the default since round 5; 2 its block-tile
form).  Same process, same buffers, rounds
alternated, HIP events around REPS back-to-back launches (median), two fresh
buffer sets per config; parity and sums checked equal.
  python3 scripts/probe_fused_wq.py
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
VARIANTS = [("block tiles", 2), ("queue", 1)]
# PROBE_ENC4=1: encode + CRC only, adds the queue at 4 slabs with input pairs
# (tune keys 28 = 1, 10 = 4) where the default is 8 slabs
ENC4 = os.environ.get("PROBE_ENC4") == "1"
if ENC4:
    VARIANTS = [("block tiles", [(28, 2)]), ("queue", [(28, 1)]), ("queue 4 slabs", [(28, 1), (10, 4)]),
                ("block 4 slabs", [(28, 2), (10, 4)])]
# PROBE_NT=1: encode + CRC only, the sums stored non-temporal (tune key 30)
if os.environ.get("PROBE_NT") == "1":
    ENC4 = True
    CONFIGS = [(6, 3, 1024)]
    VARIANTS = [("default", [(28, 0)]), ("sums nt", [(30, 1)]), ("queue sums nt", [(28, 1), (30, 1)])]


def main():
    dev = torch.device("cuda:0")
    stream = torch.cuda.current_stream()
    sp = stream.cuda_stream
    lib = H.experimental_lib()
    g = torch.Generator(device=dev)
    g.manual_seed(11)
    cases = []
    for k, m, S in CONFIGS:
        coder = H.Coder(k, m, 0, lib=lib)
        nck = CELL // 512
        for si in range(SETS):
            d = torch.empty((S, k, CELL), dtype=torch.uint8, device=dev)
            d.random_(0, 256, generator=g)
            dp, ds = H.stripe_layout_ptrs(d, k)
            outs = []
            for _ in VARIANTS:
                p = torch.empty((S, m, CELL), dtype=torch.uint8, device=dev)
                sums = torch.empty((S, k + m, nck, 4), dtype=torch.uint8, device=dev)
                pp, ps = H.stripe_layout_ptrs(p, m)
                outs.append((p, sums, pp, ps))
            rec = torch.empty((S, m, CELL), dtype=torch.uint8, device=dev)
            rp, rsd = H.stripe_layout_ptrs(rec, m)
            bad = torch.zeros((S, k + m), dtype=torch.uint8, device=dev)
            cases.append(dict(name=f"RS({k},{m}) x {S} set {si}", coder=coder, d=d, dp=dp, ds=ds, outs=outs, S=S,
                              k=k, m=m, rec=rec, rp=rp, rsd=rsd, bad=bad,
                              bytes=(k + m) * S * CELL + 4 * nck * (k + m) * S,
                              vbytes=(k + m) * S * CELL + 4 * nck * k * S,
                              t={v: [] for v, _ in VARIANTS}, tv={v: [] for v, _ in VARIANTS}))
    torch.cuda.synchronize()

    def run(c, i, wq):
        p, sums, pp, ps = c["outs"][i]
        pairs = wq if isinstance(wq, list) else [(28, wq)]
        for key, val in pairs:
            H.tune_set(key, val, lib)
        c["coder"].encode_crc_device(c["dp"], c["ds"], pp, ps, CELL, c["S"], 512, sums.data_ptr(), sp)
        for key, _ in pairs:
            H.tune_set(key, 0, lib)

    def run_verify(c, wq):
        # decode data 0..m-1 + verify the k survivors against the sums the
        # default encode + CRC wrote (outs[0]); rebuilt rows into rec
        k, m = c["k"], c["m"]
        p, sums, pp, ps = c["outs"][0]
        surv = [None] * m + c["dp"][m:] + pp
        out = [c["rp"][i] if i < m else c["dp"][i] for i in range(k)]
        ost = [c["rsd"][0] if i < m else c["ds"][i] for i in range(k)]
        H.tune_set(28, wq, lib)
        c["coder"].decode_verify_device(H.CHECKSUM_CRC32C, surv, c["ds"] + ps, out, ost, CELL, c["S"], 512,
                                        sums.data_ptr(), c["bad"].data_ptr(), sp)
        H.tune_set(28, 0, lib)

    if ENC4:
        for c in cases:
            for i, (_, wq) in enumerate(VARIANTS):
                run(c, i, wq)
            torch.cuda.synchronize()
            for i in range(1, len(VARIANTS)):
                assert torch.equal(c["outs"][i][0], c["outs"][0][0]), (c["name"], "parity")
                assert torch.equal(c["outs"][i][1], c["outs"][0][1]), (c["name"], "sums")
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
            print(f"{c['name']:22s} " + "  ".join(
                f"{v} {statistics.median(ts):.4f} ms ({c['bytes'] / (statistics.median(ts) * 1e-3) / 8e12:.3f})"
                for v, ts in c["t"].items()), flush=True)
        return
    for c in cases:
        for _, wq in VARIANTS:  # compile both specialised decode + verify kernels now
            H.tune_set(28, wq, lib)
            assert c["coder"].prepare_decode(list(range(c["m"])), H.CHECKSUM_CRC32C)
            H.tune_set(28, 0, lib)
        for i, (_, wq) in enumerate(VARIANTS):
            run(c, i, wq)
        torch.cuda.synchronize()
        for _, wq in VARIANTS:
            c["rec"].zero_()
            run_verify(c, wq)
            torch.cuda.synchronize()
            assert torch.equal(c["rec"], c["d"][:, :c["m"]]), (c["name"], "rebuilt", wq)
            assert not bool(c["bad"].any()), (c["name"], "flagged", wq)
        for i in range(1, len(VARIANTS)):
            assert torch.equal(c["outs"][i][0], c["outs"][0][0]), (c["name"], "parity")
            assert torch.equal(c["outs"][i][1], c["outs"][0][1]), (c["name"], "sums")
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
                run_verify(c, wq)
                a.record(stream)
                for _ in range(REPS):
                    run_verify(c, wq)
                b.record(stream)
                torch.cuda.synchronize()
                c["tv"][v].append(a.elapsed_time(b) / REPS)
    for c in cases:
        parts = []
        for v, ts in c["t"].items():
            med = statistics.median(ts)
            parts.append(f"enc+crc {v} {med:.4f} ms ({c['bytes'] / (med * 1e-3) / 8e12:.3f})")
        for v, ts in c["tv"].items():
            med = statistics.median(ts)
            parts.append(f"dec+verify {v} {med:.4f} ms ({c['vbytes'] / (med * 1e-3) / 8e12:.3f})")
        print(f"{c['name']:22s} " + "  ".join(parts), flush=True)


if __name__ == "__main__":
    main()
