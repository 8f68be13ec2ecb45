"""Measurement tool (GPU box): fused encode + CRC32C (hec_encode_crc_device)
and fused decode + verify (hec_decode_verify_device) across CRC lookup
schemes (tune key 11: 0/1 = slicing-by-8, 2 = bank-replicated (encode only, exp
library), 5 = 11-bit slicing; suffix w = tune key 16 = 3, one 768-thread
block per CU (exp library); suffix p = tune key 19 = 2, inputs two at a
time; suffix q = tune key 10 = 4, 4 slabs per wave; suffix s / S = tune key 21
= 2 / 3, role-split GF / CRC waves, S with the CRC waves at raised priority),
interleaved rounds, median per variant.  Every variant's
sums are checked against the default's.

  PROBE_K=6 PROBE_M=3 PROBE_S=1024 python scripts/probe_fused.py
"""
import os
import statistics
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "hdfs-native_amd"))
import torch  # noqa: E402

import hdfs_native_ec as H  # noqa: E402

K = int(os.environ.get("PROBE_K", "6"))
M = int(os.environ.get("PROBE_M", "3"))
S = int(os.environ.get("PROBE_S", "1024"))
CELL = 1 << 20
REPS = int(os.environ.get("PROBE_REPS", "10"))
ROUNDS = int(os.environ.get("PROBE_ROUNDS", "5"))
ENC = os.environ.get("PROBE_ENC", "1,5,5w").split(",")  # "<key 11 value>[w]": w = key 16 = 3 (768-thread blocks, 3 waves per SIMD)
VER = os.environ.get("PROBE_VER", "1,5,5w").split(",")
BPC = 512
dev = torch.device("cuda:0")
g = torch.Generator(device=dev).manual_seed(3)
data = torch.randint(0, 256, (S, K, CELL), dtype=torch.uint8, device=dev, generator=g)
parity = torch.empty((S, M, CELL), dtype=torch.uint8, device=dev)
rec = torch.empty((S, M, CELL), dtype=torch.uint8, device=dev)
nch = CELL // BPC
sums = torch.empty((S, K + M, nch, 4), dtype=torch.uint8, device=dev)
bad = torch.zeros((S, K + M), dtype=torch.uint8, device=dev)
coder = H.Coder(K, M, 0)
sp = torch.cuda.current_stream(dev).cuda_stream
dp, ds = H.stripe_layout_ptrs(data, K)
pp, ps = H.stripe_layout_ptrs(parity, M)
rp, rs = H.stripe_layout_ptrs(rec, M)
miss = list(range(M))
shard_ptrs = [None if i in miss else dp[i] for i in range(K)] + pp
out_ptrs = [rp[i] if i in miss else dp[i] for i in range(K)]
out_strides = [rs[0] if i in miss else ds[i] for i in range(K)]


def enc():
    coder.encode_crc_device(dp, ds, pp, ps, CELL, S, BPC, sums.data_ptr(), sp)


def ver():
    coder.decode_verify_device(H.CHECKSUM_CRC32C, shard_ptrs, ds + ps, out_ptrs, out_strides, CELL, S, BPC,
                               sums.data_ptr(), bad.data_ptr(), sp)


for kv in filter(None, os.environ.get("PROBE_TUNE", "").split(",")):  # extra hec_tune_set keys, e.g. 7=2048
    H.tune_set(*(int(v) for v in kv.split("=")))
H.tune_set(11, 0)
enc()
torch.cuda.synchronize()
ref = sums.clone()
variants = [("encode+crc", v, enc) for v in ENC] + [("decode+verify", v, ver) for v in VER]
times = {(n, v): [] for n, v, _ in variants}
for _ in range(ROUNDS):
    for name, v, fn in variants:
        H.tune_set(11, int(v.rstrip("wpqsS")))
        H.tune_set(21, 3 if "S" in v else 2 if "s" in v else 0)
        H.tune_set(16, 3 if "w" in v else 0)
        H.tune_set(19, 2 if "p" in v else 0)
        H.tune_set(10, 4 if "q" in v else 0)
        fn()
        torch.cuda.synchronize()
        if name == "encode+crc":
            assert torch.equal(sums, ref), f"scheme {v} sums differ"
        else:
            assert not bad.any() and torch.equal(rec, data[:, :M]), f"scheme {v} verify"
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
        ev[0].record()
        for _ in range(REPS):
            fn()
        ev[1].record()
        torch.cuda.synchronize()
        times[(name, v)].append(ev[0].elapsed_time(ev[1]) / REPS)
H.tune_set(11, 0)
H.tune_set(16, 0)
H.tune_set(19, 0)
H.tune_set(10, 0)
H.tune_set(21, 0)
print(f"RS({K},{M}) S={S} cell={CELL}")
for (name, v), t in times.items():
    ms = statistics.median(t)
    cells = K + M if name == "encode+crc" else K + M  # encode: k read + m written; verify: k read + e=m written
    print(f"{name} scheme-key {v}: median {ms:.3f} ms  {cells * CELL * S / ms / 1e9:.2f} TB/s of cells  "
          f"data {K * CELL * S / ms / 1e6 / 1.073741824:.1f} GiB/s  (min {min(t):.3f} max {max(t):.3f})")
