"""Measurement tool (GPU box): pinned-host <-> device copy ceilings and the
engine's pipelined host batch (hec_encode_host_batch) across chunk sizes."""
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "hdfs-native_amd"))
import torch  # noqa: E402

import hdfs_native_ec as H  # noqa: E402

GIB = float(1 << 30)
dev = torch.device("cuda:0")
n = 1536 << 20
h = torch.empty(n, dtype=torch.uint8).pin_memory()
h2 = torch.empty(n, dtype=torch.uint8).pin_memory()
d = torch.empty(n, dtype=torch.uint8, device=dev)
d2 = torch.empty(n, dtype=torch.uint8, device=dev)
s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()


def timed(fn, reps=5):
    fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / reps


t = timed(lambda: d.copy_(h, non_blocking=True))
print(f"H2D pinned: {n / t / 1e9:.1f} GB/s")
t = timed(lambda: h.copy_(d, non_blocking=True))
print(f"D2H pinned: {n / t / 1e9:.1f} GB/s")


def both():
    with torch.cuda.stream(s1):
        d.copy_(h, non_blocking=True)
    with torch.cuda.stream(s2):
        h2.copy_(d2, non_blocking=True)


t = timed(both)
print(f"H2D+D2H concurrent: {2 * n / t / 1e9:.1f} GB/s total")


def split4():
    q = n // 4
    for i in range(4):
        st = s1 if i % 2 == 0 else s2
        with torch.cuda.stream(st):
            d[i * q:(i + 1) * q].copy_(h[i * q:(i + 1) * q], non_blocking=True)


t = timed(split4)
print(f"H2D split over 2 streams: {n / t / 1e9:.1f} GB/s")

k, m, cell = 6, 3, 1 << 20
S = 256
coder = H.Coder(k, m, 0)
hin = torch.randint(0, 256, (S, k, cell), dtype=torch.uint8).pin_memory()
hout = torch.empty((S, m, cell), dtype=torch.uint8).pin_memory()
del d, d2
torch.cuda.empty_cache()
for chunk in (2, 4, 8, 16, 32, 64):
    t = timed(lambda: coder.encode_host_batch(hin.data_ptr(), hout.data_ptr(), cell, S, chunk), reps=3)
    print(f"host batch chunk={chunk}: {k * cell * S / t / GIB:.1f} GiB/s data "
          f"(H2D {k * cell * S / t / 1e9:.1f} GB/s, D2H {m * cell * S / t / 1e9:.1f} GB/s)")

# decode straight to file order: vertical shard buffers (data 0..2 lost)
vert = [None] * (k + m)
for i in range(3, k):
    vert[i] = hin[:, i, :].contiguous().pin_memory()
for j in range(m):
    vert[k + j] = hout[:, j, :].contiguous().pin_memory()
hfile = torch.empty(S * k * cell, dtype=torch.uint8).pin_memory()
addrs = [None if v is None else v.data_ptr() for v in vert]
for chunk in (8, 16, 32):
    t = timed(lambda: coder.decode_host_batch(addrs, cell, S, hfile.data_ptr(), chunk), reps=3)
    print(f"host decode->file chunk={chunk}: {k * cell * S / t / GIB:.1f} GiB/s data "
          f"(H2D {k * cell * S / t / 1e9:.1f} GB/s, D2H {k * cell * S / t / 1e9:.1f} GB/s)")
assert torch.equal(hfile.view(S, k, cell), hin), "decode_host_batch mismatch"
print("decode_host_batch bit-exact")
