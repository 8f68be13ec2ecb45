"""Measurement probe (GPU box, measurement build): the fused kernels' launch
shapes compared on the SAME buffers.  Kernel speed depends on where a
process's buffers land (scripts/probe_placement.py), so an A/B across
processes mixes placement into the result; here PROBE_SETS buffer sets are
allocated once and every configuration (tune keys, include/hdfs_ec_amd_exp.h)
is timed on every set, alternating, PROBE_ROUNDS times.  RS(6,3) 1 MiB x 1024:
the specialised decode + verify ({0,1,2} lost, prepared per configuration)
and the encode + CRC32C.  One line per (configuration, set): best of 6.
  python3 scripts/probe_fused_sweep.py
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "hdfs-native_amd"))

import torch  # noqa: E402

import hdfs_native_ec as H  # noqa: E402

# name -> tune pairs; every key not named is reset to 0 before a configuration
CONFIGS = {
    "default": [],
    "grp16": [(8, 16)],
    "grid32": [(7, 32 * 256)],
    "grp8grid32": [(8, 8), (7, 32 * 256)],
    "enc4": [(10, 4)],
    "grid8": [(7, 8 * 256)],
    "grid64": [(7, 64 * 256)],
    "grp8grid16": [(8, 8), (7, 16 * 256)],
    "grp1": [(8, 1)],
    "grp2": [(8, 2)],
    "grp8": [(8, 8)],
    "grid4": [(7, 4 * 256)],
    "grid16": [(7, 16 * 256)],
    "slabs8": [(10, 8)],
}
KEYS = (7, 8, 10)


def main():
    k, m, cell, S = 6, 3, 1 << 20, 1024
    sets, rounds, reps = int(os.environ.get("PROBE_SETS", "3")), int(os.environ.get("PROBE_ROUNDS", "2")), 6
    names = os.environ.get("PROBE_CONFIGS", ",".join(CONFIGS)).split(",")
    xlib = H.experimental_lib()
    dev = torch.device("cuda:0")
    stream = torch.cuda.current_stream()
    sp = stream.cuda_stream
    bpc, nch = 512, cell // 512
    miss = [0, 1, 2]
    bufs = []
    for s in range(sets):
        d = torch.randint(0, 256, (S, k, cell), dtype=torch.uint8, device=dev)
        p = torch.empty((S, m, cell), dtype=torch.uint8, device=dev)
        out = torch.empty((S, k, cell), dtype=torch.uint8, device=dev)
        sums = torch.empty((S, k + m, nch, 4), dtype=torch.uint8, device=dev)
        bad = torch.empty((S, k + m), dtype=torch.uint8, device=dev)
        bufs.append((d, p, out, sums, bad))
    results = {}
    for rnd in range(rounds):
        for name in names:
            for key in KEYS:
                H.tune_set(key, 0, xlib)
            for key, val in CONFIGS[name]:
                H.tune_set(key, val, xlib)
            coder = H.Coder(k, m, 0, lib=xlib)
            assert coder.prepare_decode(miss, H.CHECKSUM_CRC32C), "specialised kernel not ready"
            for si, (d, p, out, sums, bad) in enumerate(bufs):
                dp, ds = H.stripe_layout_ptrs(d, k)
                pp, ps = H.stripe_layout_ptrs(p, m)
                op, os_ = H.stripe_layout_ptrs(out, k)
                shard_ptrs = [None if i in miss else dp[i] for i in range(k)] + pp
                vo = [op[i] if i in miss else dp[i] for i in range(k)]
                vs = [os_[0] if i in miss else ds[i] for i in range(k)]

                def ec():
                    coder.encode_crc_device(dp, ds, pp, ps, cell, S, bpc, sums.data_ptr(), sp)

                def dv():
                    coder.decode_verify_device(H.CHECKSUM_CRC32C, shard_ptrs, ds + ps, vo, vs, cell, S, bpc,
                                               sums.data_ptr(), bad.data_ptr(), sp)

                row = {}
                for leg, fn in (("encode_crc", ec), ("decode_verify", dv)):
                    fn()
                    torch.cuda.synchronize()
                    best = 1e9
                    for _ in range(reps):
                        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                        a.record(stream)
                        fn()
                        b.record(stream)
                        torch.cuda.synchronize()
                        best = min(best, a.elapsed_time(b))
                    row[leg] = best
                    results.setdefault((name, leg), []).append(best)
                print(f"round {rnd} {name:8s} set {si}: encode_crc {row['encode_crc']:.4f} ms  "
                      f"decode_verify {row['decode_verify']:.4f} ms", flush=True)
            coder.close()
    for key in KEYS:
        H.tune_set(key, 0, xlib)
    print("mean over sets and rounds (ms):")
    for name in names:
        e = results[(name, "encode_crc")]
        v = results[(name, "decode_verify")]
        print(f"  {name:8s} encode_crc {sum(e) / len(e):.4f}  decode_verify {sum(v) / len(v):.4f}", flush=True)


if __name__ == "__main__":
    main()
