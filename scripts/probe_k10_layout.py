"""Measurement probe (GPU box, product library): the plain encode
(gf_matmul_v16 on the work queue) of RS(10,4) 1 MiB x 256 and RS(6,3) 1 MiB
x 1024 over HBM layouts that move the shards' cells against each other:
  pad P  : data [S][k][cell + P], parity [S][m][cell + P] (P = 0 is bench.py's
           split layout; a cell of shard i then starts i * (cell + P) after
           shard 0's)
  shard  : k + m tensors [S][cell] (every shard its own allocation)
Round 6: the k = 10 PMC passes show the TCP's L2 request interface stalled 16 %
of cycles (TCP_TCR_TCP_STALL_CYCLES) against 1 % at k = 6; a cell pitch off
the power of two spreads one wave's 14 streams over other L2 channels if the
channel hash keeps them together.  Same process, rounds alternated, HIP events
around REPS back-to-back launches (median), outputs checked equal to pad 0's.
  python3 scripts/probe_k10_layout.py
"""
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "hdfs-native_amd"))

import torch  # noqa: E402

import hdfs_native_ec as H  # noqa: E402

CELL = 1 << 20
CONFIGS = [(10, 4, 256), (6, 3, 1024)]
PADS = [int(x) for x in os.environ.get("PROBE_PADS", "0,256,2048,4352,65536").split(",")]
ROUNDS = int(os.environ.get("PROBE_ROUNDS", "5"))
# PROBE_CFG=10 / 6: that k only; PROBE_ONLY="pad 0,shard": those layouts only
# (scripts/pmc_layout.sh profiles one (config, layout) per process)
if os.environ.get("PROBE_CFG"):
    CONFIGS = [c for c in CONFIGS if c[0] == int(os.environ["PROBE_CFG"])]
ONLY = os.environ.get("PROBE_ONLY", "").split(",") if os.environ.get("PROBE_ONLY") else None
REPS = int(os.environ.get("PROBE_REPS", "6"))


def main():
    dev = torch.device("cuda:0")
    stream = torch.cuda.current_stream()
    sp = stream.cuda_stream
    g = torch.Generator(device=dev)
    g.manual_seed(3)
    cases = []
    for k, m, S in CONFIGS:
        coder = H.Coder(k, m, 0)
        ref = torch.randint(0, 256, (S, k, CELL), dtype=torch.uint8, device=dev, generator=g)
        lays = []
        for pad in PADS:
            d = torch.empty((S, k, CELL + pad), dtype=torch.uint8, device=dev)
            d[:, :, :CELL].copy_(ref)
            p = torch.empty((S, m, CELL + pad), dtype=torch.uint8, device=dev)
            dp, ds = H.stripe_layout_ptrs(d, k)
            pp, ps = H.stripe_layout_ptrs(p, m)
            lays.append((f"pad {pad}", (d, p), dp, ds, pp, ps, lambda p=p: p[:, :, :CELL]))
        ts = [ref[:, i].contiguous() for i in range(k)]
        tp = [torch.empty((S, CELL), dtype=torch.uint8, device=dev) for _ in range(m)]
        lays.append(("shard", (ts, tp), [x.data_ptr() for x in ts], [CELL] * k, [x.data_ptr() for x in tp],
                     [CELL] * m, lambda tp=tp: torch.stack(tp, 1)))
        del ref
        if ONLY:
            lays = [x for x in lays if x[0] in ONLY]
        cases.append(dict(name=f"RS({k},{m}) x {S}", k=k, m=m, S=S, coder=coder, lays=lays,
                          t={x[0]: [] for x in lays}, bytes=(k + m) * S * CELL))
    torch.cuda.synchronize()

    def run(c, lay):
        _, _, dp, ds, pp, ps, _ = lay
        c["coder"].encode_device(dp, ds, pp, ps, CELL, c["S"], sp)

    for c in cases:
        for lay in c["lays"]:
            run(c, lay)
        torch.cuda.synchronize()
        want = c["lays"][0][6]()
        for lay in c["lays"][1:]:  # (PROBE_ONLY: against the first layout kept)
            assert torch.equal(lay[6](), want), (c["name"], lay[0])
    for _ in range(ROUNDS):
        for c in cases:
            for lay in c["lays"]:
                run(c, lay)
                a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                a.record(stream)
                for _ in range(REPS):
                    run(c, lay)
                b.record(stream)
                torch.cuda.synchronize()
                c["t"][lay[0]].append(a.elapsed_time(b) / REPS)
    for c in cases:
        print(f"{c['name']:16s} " + "  ".join(
            f"{n} {statistics.median(ts):.4f} ms ({c['bytes'] / (statistics.median(ts) * 1e-3) / 8e12:.3f})"
            for n, ts in c["t"].items()), flush=True)


if __name__ == "__main__":
    main()
