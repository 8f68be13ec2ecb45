"""Measurement tool (GPU box): the rate of a batch whose layout is not
16-B aligned -- the dword-realigning kernel (gf_matmul_dw)
and, with tune key 18 = 1, the one-thread-per-byte kernel alone -- next to
the same bytes aligned.
RS(6,3) encode, 1 MiB cells; shard i of stripe s at buf + OFF + (s*K + i) *
PITCH.  OFF = 0 with PITCH = cell is the aligned vector path; OFF = 1, 4, 8
moves every base off the 16-B grid; OFF = 0 with PITCH = cell + 4 moves
every stripe's stride off it.  Each variant's parity is checked against the
aligned run's.

  PROBE_S=64 python scripts/probe_unaligned.py
"""
import os
import statistics
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "hdfs-native_amd"))
import torch  # noqa: E402

import hdfs_native_ec as H  # noqa: E402

K, M = 6, 3
CELL = int(os.environ.get("PROBE_CELL", str(1 << 20)))
S = int(os.environ.get("PROBE_S", "64"))
REPS = int(os.environ.get("PROBE_REPS", "5"))
ROUNDS = int(os.environ.get("PROBE_ROUNDS", "3"))
VARIANTS = [(0, CELL, 0), (1, CELL, 0), (4, CELL, 0), (8, CELL, 0), (0, CELL + 4, 0), (2, CELL + 2, 0),
            (1, CELL, 1)]  # (base offset, shard pitch, tune key 18)
dev = torch.device("cuda:0")
coder = H.Coder(K, M, 0)
sp = torch.cuda.current_stream(dev).cuda_stream
src = torch.randint(0, 256, (S, K, CELL), dtype=torch.uint8, device=dev, generator=torch.Generator(device=dev).manual_seed(5))
pitch_max = CELL + 16
din = torch.zeros(16 + S * K * pitch_max, dtype=torch.uint8, device=dev)
dout = torch.zeros(16 + S * M * pitch_max, dtype=torch.uint8, device=dev)


def layout(off, pitch):
    """Copy src into din at (off, pitch); pointer/stride lists for both buffers."""
    view = din[off:off + S * K * pitch].view(S, K, pitch)[:, :, :CELL]
    view.copy_(src)
    ip = [din.data_ptr() + off + i * pitch for i in range(K)]
    op = [dout.data_ptr() + off + j * pitch for j in range(M)]
    return ip, [K * pitch] * K, op, [M * pitch] * M


def parity(off, pitch):
    return dout[off:off + S * M * pitch].view(S, M, pitch)[:, :, :CELL].clone()


ref = None
times = {v: [] for v in VARIANTS}
for _ in range(ROUNDS):
    for off, pitch, byte_only in VARIANTS:
        H.tune_set(18, byte_only)
        ip, ist, op, ost = layout(off, pitch)
        coder.encode_device(ip, ist, op, ost, CELL, S, sp)
        torch.cuda.synchronize()
        got = parity(off, pitch)
        if ref is None:
            ref = got
        assert torch.equal(got, ref), f"offset {off} pitch {pitch} key18 {byte_only}: parity differs"
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
        ev[0].record()
        for _ in range(REPS):
            coder.encode_device(ip, ist, op, ost, CELL, S, sp)
        ev[1].record()
        torch.cuda.synchronize()
        times[(off, pitch, byte_only)].append(ev[0].elapsed_time(ev[1]) / REPS)
H.tune_set(18, 0)
print(f"RS({K},{M}) encode, {S} stripes x {CELL} B cells", flush=True)
base = statistics.median(times[VARIANTS[0]])
for (off, pitch, byte_only), t in times.items():
    ms = statistics.median(t)
    kern = "byte kernel" if byte_only else ("vector" if (off, pitch) == (0, CELL) else "dword kernel")
    print(f"base offset {off:2d} pitch cell{pitch - CELL:+d} {kern:12s}: {ms:.3f} ms  {K * CELL * S / ms / 1e6 / 1.073741824:8.1f} GiB/s "
          f"of data  {(K + M) * CELL * S / ms / 1e9:7.2f} TB/s  ({base / ms:.3f} of aligned)", flush=True)
