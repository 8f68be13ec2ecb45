"""Measurement probe (GPU box): is the fused decode + verify kernel's speed a
property of where its buffers land?  In ONE process, PROBE_SETS times: fresh
RS(6,3) 1 MiB x 1024 data / parity / output tensors (the earlier sets stay
allocated, so every set gets new memory), encode + CRC32C sums, the
{0,1,2}-lost plan prepared (the specialised kernel), then the fused decode +
verify and the fused encode + CRC timed with HIP events.  One line per set.
PROBE_CROSS=1 then times decode + verify for every (input set, output set)
pair: does the speed follow where the survivors or the rebuilt rows land?
  python3 scripts/probe_placement.py
"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "hdfs-native_amd"))

import torch  # noqa: E402

import hdfs_native_ec as H  # noqa: E402


def main():
    k, m, cell, S = 6, 3, 1 << 20, int(os.environ.get("PROBE_S", "1024"))
    sets, reps = int(os.environ.get("PROBE_SETS", "5")), 8
    dev = torch.device("cuda:0")
    stream = torch.cuda.current_stream()
    sp = stream.cuda_stream
    coder = H.Coder(k, m, 0)
    miss = [0, 1, 2]
    print("jit prepared:", coder.prepare_decode(miss, H.CHECKSUM_CRC32C), flush=True)
    keep = []
    bpc, nch = 512, cell // 512
    for s in range(sets):
        d = torch.randint(0, 256, (S, k, cell), dtype=torch.uint8, device=dev)
        p = torch.empty((S, m, cell), dtype=torch.uint8, device=dev)
        out = torch.empty((S, k, cell), dtype=torch.uint8, device=dev)
        sums = torch.empty((S, k + m, nch, 4), dtype=torch.uint8, device=dev)
        bad = torch.empty((S, k + m), dtype=torch.uint8, device=dev)
        keep.append((d, p, out, sums, bad))
        dp, ds = H.stripe_layout_ptrs(d, k)
        pp, ps = H.stripe_layout_ptrs(p, m)
        op, os_ = H.stripe_layout_ptrs(out, k)
        coder.encode_crc_device(dp, ds, pp, ps, cell, S, bpc, sums.data_ptr(), sp)
        shard_ptrs = [None if i in miss else dp[i] for i in range(k)] + pp
        vo = [op[i] if i in miss else dp[i] for i in range(k)]
        vs = [os_[0] if i in miss else ds[i] for i in range(k)]

        def dv():
            coder.decode_verify_device(H.CHECKSUM_CRC32C, shard_ptrs, ds + ps, vo, vs, cell, S, bpc,
                                       sums.data_ptr(), bad.data_ptr(), sp)

        def ec():
            coder.encode_crc_device(dp, ds, pp, ps, cell, S, bpc, sums.data_ptr(), sp)

        res = {}
        for name, fn in (("decode_verify", dv), ("encode_crc", ec)):
            fn()
            torch.cuda.synchronize()
            ts = []
            for _ in range(reps):
                a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                a.record(stream)
                fn()
                b.record(stream)
                torch.cuda.synchronize()
                ts.append(a.elapsed_time(b))
            res[name] = (min(ts), sorted(ts)[len(ts) // 2])
        base = d.data_ptr()
        print(f"set {s}: data base 0x{base:x}  decode_verify min {res['decode_verify'][0]:.4f} "
              f"med {res['decode_verify'][1]:.4f} ms  encode_crc min {res['encode_crc'][0]:.4f} "
              f"med {res['encode_crc'][1]:.4f} ms", flush=True)
        time.sleep(0.2)
    if os.environ.get("PROBE_CROSS") == "1":
        print("decode + verify, best of 8 (ms): rows = input set, columns = output set", flush=True)
        for i, (d, p, _o, sums, bad) in enumerate(keep):
            dp, ds = H.stripe_layout_ptrs(d, k)
            pp, ps = H.stripe_layout_ptrs(p, m)
            shard_ptrs = [None if x in miss else dp[x] for x in range(k)] + pp
            row = []
            for j in range(len(keep)):
                op, os_ = H.stripe_layout_ptrs(keep[j][2], k)
                vo = [op[x] if x in miss else dp[x] for x in range(k)]
                vs = [os_[0] if x in miss else ds[x] for x in range(k)]

                def dv():
                    coder.decode_verify_device(H.CHECKSUM_CRC32C, shard_ptrs, ds + ps, vo, vs, cell, S, bpc,
                                               sums.data_ptr(), bad.data_ptr(), sp)
                dv()
                torch.cuda.synchronize()
                best = 1e9
                for _ in range(reps):
                    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    a.record(stream)
                    dv()
                    b.record(stream)
                    torch.cuda.synchronize()
                    best = min(best, a.elapsed_time(b))
                row.append(best)
            print(f"in {i}: " + "  ".join(f"{t:.4f}" for t in row), flush=True)


if __name__ == "__main__":
    main()
