"""Measurement probe (GPU box): the product kernels over three HBM layouts of
the same RS(6,3) 1 MiB x S batch, two fresh buffer sets per layout, rounds
alternated so drift hits every set alike (HIP events, median of REPS):
  split  : data [S][k][cell] + parity [S][m][cell] (+ rebuilt [S][m][cell]):
           bench.py's layout
  stripe : one [S][k+m][cell] tensor (a stripe's cells contiguous); rebuilt
           rows go to the stripe's own slots of the lost shards
  shard  : k+m tensors [S][cell] (+ rebuilt [S][m][cell])
Kernels: checksum_chunks512 (CRC32C of all k+m cells), gf_matmul_v16
(encode), the fused encode + CRC32C and the plan-specialised fused decode
{0,1,2} + verify.  Prints one line per (layout, set).
PROBE_CRC_AB=1: the measurement build instead, CRC32C of all k+m cells by the
default register-staged kernel, the same with non-temporal sum stores (tune
key 30 = 1) and on the work queue (key 29 = 4 tasks per unit), compute and
verify mode, same buffers,
rounds alternated (round 5 also ran the LDS-DMA kernel here, key 11 = 13,
removed in round 6: profiles/r05n); PROBE_CRC_768=1 (round 6) the default kernel
against one 768-thread block per CU (key 33) and the memory side alone (key
11 = 9, WRONG sums), compute and verify mode; PROBE_CRC_PF2=1 (round 6) the
default against two tasks of register prefetch (key 12 = 2).
  python3 scripts/probe_layout.py
"""
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "hdfs-native_amd"))

import torch  # noqa: E402

import hdfs_native_ec as H  # noqa: E402

K, M, CELL = 6, 3, 1 << 20
S = int(os.environ.get("PROBE_S", "1024"))
SETS = int(os.environ.get("PROBE_SETS", "2"))
ROUNDS = int(os.environ.get("PROBE_ROUNDS", "4"))
REPS = int(os.environ.get("PROBE_REPS", "6"))
LAYOUTS = os.environ.get("PROBE_LAYOUTS", "split,stripe,shard").split(",")
CRC_AB = os.environ.get("PROBE_CRC_AB") == "1"
BPC, NCH = 512, CELL // 512
MISS = [0, 1, 2]


def make_set(layout, dev, g):
    """-> dict of pointer lists / strides for one fresh buffer set."""
    keep = []
    if layout == "split":
        d = torch.randint(0, 256, (S, K, CELL), dtype=torch.uint8, device=dev, generator=g)
        p = torch.empty((S, M, CELL), dtype=torch.uint8, device=dev)
        r = torch.empty((S, M, CELL), dtype=torch.uint8, device=dev)
        keep += [d, p, r]
        dp, ds = H.stripe_layout_ptrs(d, K)
        pp, ps = H.stripe_layout_ptrs(p, M)
        rp, rs = H.stripe_layout_ptrs(r, M)
        out = [rp[i] if i in MISS else dp[i] for i in range(K)]
        ost = [rs[0] if i in MISS else ds[i] for i in range(K)]
    elif layout == "stripe":
        t = torch.empty((S, K + M, CELL), dtype=torch.uint8, device=dev)
        t[:, :K].random_(0, 256, generator=g)
        keep += [t]
        ap, ast = H.stripe_layout_ptrs(t, K + M)
        dp, ds, pp, ps = ap[:K], ast[:K], ap[K:], ast[K:]
        out, ost = dp, ds  # rebuilt rows into the lost shards' own slots
    else:
        ts = [torch.empty((S, CELL), dtype=torch.uint8, device=dev) for _ in range(K + M)]
        for x in ts[:K]:
            x.random_(0, 256, generator=g)
        r = torch.empty((S, M, CELL), dtype=torch.uint8, device=dev)
        keep += ts + [r]
        dp, ds = [x.data_ptr() for x in ts[:K]], [CELL] * K
        pp, ps = [x.data_ptr() for x in ts[K:]], [CELL] * M
        rp, rs = H.stripe_layout_ptrs(r, M)
        out = [rp[i] if i in MISS else dp[i] for i in range(K)]
        ost = [rs[0] if i in MISS else ds[i] for i in range(K)]
    sums = torch.empty((S, K + M, NCH, 4), dtype=torch.uint8, device=dev)
    bad = torch.zeros((S, K + M), dtype=torch.uint8, device=dev)
    keep += [sums, bad]
    return dict(keep=keep, dp=dp, ds=ds, pp=pp, ps=ps, out=out, ost=ost, sums=sums, bad=bad)


def main():
    dev = torch.device("cuda:0")
    stream = torch.cuda.current_stream()
    sp = stream.cuda_stream
    lib = H.experimental_lib() if CRC_AB else None
    coder = H.Coder(K, M, 0, lib=lib)
    print("jit prepared:", coder.prepare_decode(MISS, H.CHECKSUM_CRC32C), flush=True)
    g = torch.Generator(device=dev)
    g.manual_seed(5)
    sets = [(lay, i, make_set(lay, dev, g)) for i in range(SETS) for lay in LAYOUTS]
    kernels = {}
    for lay, i, st in sets:
        cells, cstr = st["dp"] + st["pp"], st["ds"] + st["ps"]
        surv = [None if x in MISS else st["dp"][x] for x in range(K)] + st["pp"]

        def crc(st=st, cells=cells, cstr=cstr):
            coder.crc32c_device(cells, cstr, CELL, S, BPC, st["sums"].data_ptr(), sp)

        def enc(st=st):
            coder.encode_device(st["dp"], st["ds"], st["pp"], st["ps"], CELL, S, sp)

        def enc_crc(st=st):
            coder.encode_crc_device(st["dp"], st["ds"], st["pp"], st["ps"], CELL, S, BPC, st["sums"].data_ptr(), sp)

        def dec_ver(st=st, surv=surv):
            coder.decode_verify_device(H.CHECKSUM_CRC32C, surv, st["ds"] + st["ps"], st["out"], st["ost"], CELL, S,
                                       BPC, st["sums"].data_ptr(), st["bad"].data_ptr(), sp)

        enc_crc()
        torch.cuda.synchronize()
        if CRC_AB:
            def tuned(fn, v, key=11):
                def run():
                    H.tune_set(key, v, lib)
                    fn()
                    H.tune_set(key, 0, lib)
                return run

            def ver(st=st, cells=cells, cstr=cstr):
                coder.checksum_verify_device(H.CHECKSUM_CRC32C, cells, cstr, CELL, S, BPC, st["sums"].data_ptr(),
                                             st["bad"].data_ptr(), sp)

            kernels[(lay, i)] = {"crc_reg": crc, "crc_runs4": tuned(crc, 4, 31), "crc_runs8": tuned(crc, 8, 31),
                                 "crc_runs16": tuned(crc, 16, 31), "verify_reg": ver, "verify_runs8": tuned(ver, 8, 31)}
            if os.environ.get("PROBE_CRC_768") == "1":  # round 6: 3 waves per SIMD (key 33), the skeleton (key 11 = 9)
                # the memory side first: its WRONG sums are rewritten before the verify legs
                kernels[(lay, i)] = {"crc_mem": tuned(crc, 9), "crc_reg": crc, "crc_768": tuned(crc, 768, 33),
                                     "verify_reg": ver, "verify_768": tuned(ver, 768, 33)}
            if os.environ.get("PROBE_CRC_PF2") == "1":  # round 6: two tasks of prefetch (key 12 = 2)
                kernels[(lay, i)] = {"crc_reg": crc, "crc_pf2": tuned(crc, 2, 12), "verify_reg": ver,
                                     "verify_pf2": tuned(ver, 2, 12)}
            continue
        kernels[(lay, i)] = {"crc_only": crc, "encode": enc, "encode_crc": enc_crc, "decode_verify": dec_ver}
    times = {key: {n: [] for n in fns} for key, fns in kernels.items()}
    for _ in range(ROUNDS):
        for key, fns in kernels.items():
            for name, fn in fns.items():
                fn()
                a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                a.record(stream)
                for _ in range(REPS):
                    fn()
                b.record(stream)
                torch.cuda.synchronize()
                times[key][name].append(a.elapsed_time(b) / REPS)
    for lay, i, st in sets:
        assert not bool(st["bad"].any()), f"{lay} {i}: verify flagged a clean cell"
    algo = {"crc_only": (K + M) * CELL * S + 4 * NCH * (K + M) * S, "encode": (K + M) * CELL * S,
            "encode_crc": (K + M) * CELL * S + 4 * NCH * (K + M) * S,
            "decode_verify": (K + len(MISS)) * CELL * S + 4 * NCH * K * S}
    for n in ("crc_dma", "crc_reg", "verify_dma", "verify_reg", "crc_wq1", "crc_wq2", "crc_wq4", "verify_wq2", "crc_nt", "crc_wq8", "crc_wq16", "verify_wq8", "crc_runs2", "crc_runs4", "verify_runs2", "crc_runs8", "crc_runs16", "verify_runs8", "crc_768", "verify_768", "crc_mem", "crc_pf2", "verify_pf2"):
        algo[n] = algo["crc_only"]
    for key, per in times.items():
        parts = []
        for name, ts in per.items():
            med = statistics.median(ts)
            parts.append(f"{name} {med:.4f} ms ({algo[name] / (med * 1e-3) / 8e12:.3f})")
        print(f"{key[0]:6s} set {key[1]}: " + "  ".join(parts), flush=True)


if __name__ == "__main__":
    main()
