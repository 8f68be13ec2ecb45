"""Measurement probe (GPU box, measurement build): small batches on the
register kernel's work queue at one 256-thread block per CU (the default: one
wave per SIMD) against 2 and 4 per CU (tune key 3).  A batch of a few
thousand wave-tiles gives each of the 1024 waves only a handful, so the
launch's ramp-up and tail are a large part of it.  The first config is the
reference's own Criterion exercise (`rust/benches/ec.rs`: one RS(6,3) stripe
of 16 MiB cells, encode and decode with 3 data slices missing).  Two timings
per variant: iterations each followed by a synchronise (as Criterion's
`b.iter` with `GpuCoder::synchronize`), wall clock; and REPS launches back to
back between HIP events (the kernel's own rate).  Same process, same
buffers, rounds alternated, medians; outputs checked equal to the default's.
  python3 scripts/probe_small_batch.py
"""
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "hdfs-native_amd"))

import torch  # noqa: E402

import hdfs_native_ec as H  # noqa: E402

CONFIGS = [(6, 3, 16 << 20, 1), (6, 3, 1 << 20, 16), (6, 3, 1 << 20, 128), (10, 4, 1 << 20, 32)]
VARIANTS = [("1/CU", []), ("2/CU", [(3, 2)]), ("4/CU", [(3, 4)])]
ROUNDS = int(os.environ.get("PROBE_ROUNDS", "5"))
REPS = int(os.environ.get("PROBE_REPS", "20"))


def main():
    dev = torch.device("cuda:0")
    stream = torch.cuda.current_stream()
    sp = stream.cuda_stream
    lib = H.experimental_lib()
    g = torch.Generator(device=dev)
    g.manual_seed(7)
    cases = []
    for k, m, cell, S in CONFIGS:
        coder = H.Coder(k, m, 0, lib=lib)
        d = torch.randint(0, 256, (S, k, cell), dtype=torch.uint8, device=dev, generator=g)
        p = torch.empty((S, m, cell), dtype=torch.uint8, device=dev)
        r = torch.empty((S, m, cell), dtype=torch.uint8, device=dev)
        dp, ds = H.stripe_layout_ptrs(d, k)
        pp, ps = H.stripe_layout_ptrs(p, m)
        rp, rs = H.stripe_layout_ptrs(r, m)
        surv = [None] * m + dp[m:] + pp
        outs = rp + [0] * (k - m)

        def enc(coder=coder, dp=dp, ds=ds, pp=pp, ps=ps, cell=cell, S=S):
            coder.encode_device(dp, ds, pp, ps, cell, S, sp)

        def dec(coder=coder, surv=surv, ds=ds, ps=ps, outs=outs, rs=rs, cell=cell, S=S, k=k):
            coder.decode_device(surv, ds + ps, outs, [rs[0]] * k, cell, S, sp)

        cases.append(dict(name=f"RS({k},{m}) {cell >> 20} MiB x {S}", d=d, p=p, r=r, m=m, enc=enc, dec=dec,
                          bytes_enc=(k + m) * cell * S, data=k * cell * S,
                          t={(op, v): {"sync": [], "events": []} for op in ("encode", "decode") for v, _ in VARIANTS}))

    def with_knobs(knobs, fn):
        for key, val in knobs:
            H.tune_set(key, val, lib)
        fn()
        for key, _ in knobs:
            H.tune_set(key, 0, lib)

    for c in cases:
        ref = None
        for v, kn in VARIANTS:
            c["p"].zero_()
            c["r"].zero_()
            with_knobs(kn, c["enc"])
            with_knobs(kn, c["dec"])
            torch.cuda.synchronize()
            assert torch.equal(c["r"], c["d"][:, :c["m"]]), (c["name"], v, "decode")
            if ref is None:
                ref = c["p"].clone()
            assert torch.equal(c["p"], ref), (c["name"], v, "parity")
        del ref
    for _ in range(ROUNDS):
        for c in cases:
            for op in ("encode", "decode"):
                fn = c["enc"] if op == "encode" else c["dec"]
                for v, kn in VARIANTS:
                    for key, val in kn:
                        H.tune_set(key, val, lib)
                    fn()
                    torch.cuda.synchronize()
                    t0 = time.perf_counter()
                    for _ in range(REPS):
                        fn()
                        torch.cuda.synchronize()
                    c["t"][(op, v)]["sync"].append((time.perf_counter() - t0) / REPS * 1e3)
                    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    a.record(stream)
                    for _ in range(REPS):
                        fn()
                    b.record(stream)
                    torch.cuda.synchronize()
                    c["t"][(op, v)]["events"].append(a.elapsed_time(b) / REPS)
                    for key, _ in kn:
                        H.tune_set(key, 0, lib)
    GIB = float(1 << 30)
    for c in cases:
        for op in ("encode", "decode"):
            parts = []
            for v, _ in VARIANTS:
                ts, te = (statistics.median(c["t"][(op, v)][x]) for x in ("sync", "events"))
                parts.append(f"{v} sync {ts * 1e3:.1f} us ({c['data'] / (ts * 1e-3) / GIB:.0f} GiB/s) "
                             f"back-to-back {te * 1e3:.1f} us")
            print(f"{c['name']:22s} {op:6s} " + "  ".join(parts), flush=True)


if __name__ == "__main__":
    main()
