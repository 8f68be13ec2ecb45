"""Measurement tool (GPU box): the GF matmul kernel at K inputs x R outputs
(hec_gf_matmul_device) across launch shapes, to separate the memory side
from the per-output GF math (VALU) -- e.g. RS(10,4) encode is K=10, R=4.
Interleaved rounds, median per variant; GB/s counts (K+R) * cell * S.

  PROBE_K=10 PROBE_S=512 python scripts/probe_rows.py
"""
import os
import statistics
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "hdfs-native_amd"))
import torch  # noqa: E402

import hdfs_native_ec as H  # noqa: E402

K = int(os.environ.get("PROBE_K", "10"))
S = int(os.environ.get("PROBE_S", "512"))
CELL = int(os.environ.get("PROBE_CELL", str(1 << 20)))
REPS = int(os.environ.get("PROBE_REPS", "10"))
ROUNDS = int(os.environ.get("PROBE_ROUNDS", "4"))
RS = [int(x) for x in os.environ.get("PROBE_R", "1,2,3,4").split(",")]
# "unroll:block:blocks_per_cu[:key=value...]" (extra hec_tune_set keys);
# 0:0:0 = engine default
SHAPES = os.environ.get("PROBE_SHAPES", "0:0:0,2:256:1,2:256:2,4:256:1,2:512:1,2:512:2,1:512:2,1:256:4").split(",")
EXTRA_KEYS = sorted({int(f.split("=")[0]) for s in SHAPES for f in s.split(":")[3:]})

dev = torch.device("cuda:0")
data = torch.empty((S, K, CELL), dtype=torch.uint8, device=dev)
data.random_(0, 256, generator=torch.Generator(device=dev).manual_seed(7))
out = torch.empty((S, 4, CELL), dtype=torch.uint8, device=dev)
coder = H.Coder(K, 4 if K <= 28 else 1, 0)
mat_all = H.gen_rs_matrix(K, 4)[K:]
ip, ist = H.stripe_layout_ptrs(data, K)
op, ost = H.stripe_layout_ptrs(out, 4)
stream = torch.cuda.current_stream(dev).cuda_stream


def run(r):
    coder.gf_matmul_device(mat_all[:r], ip, ist, op[:r], ost[:r], CELL, S, stream)


def set_shape(sh):
    f = sh.split(":")
    H.tune_set(1, int(f[0]))
    H.tune_set(4, int(f[1]))
    H.tune_set(3, int(f[2]))
    extra = dict(tuple(int(v) for v in e.split("=")) for e in f[3:])
    for key in EXTRA_KEYS:
        H.tune_set(key, extra.get(key, 0))


variants = [(r, sh) for r in RS for sh in SHAPES]
times = {v: [] for v in variants}
ref = {}
for r in RS:
    set_shape("0:0:0")
    run(r)
    torch.cuda.synchronize()
    ref[r] = out[:, :r].clone()
for _ in range(ROUNDS):
    for r, sh in variants:
        set_shape(sh)
        run(r)
        torch.cuda.synchronize()
        assert torch.equal(out[:, :r], ref[r]), f"R={r} shape {sh} mismatch"
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
        ev[0].record()
        for _ in range(REPS):
            run(r)
        ev[1].record()
        torch.cuda.synchronize()
        times[(r, sh)].append(ev[0].elapsed_time(ev[1]) / REPS)
set_shape("0:0:0")
print(f"K={K} S={S} cell={CELL}")
for (r, sh), t in times.items():
    ms = statistics.median(t)
    print(f"R={r} shape {sh}: {ms:.3f} ms  {(K + r) * CELL * S / ms / 1e6:.1f} GB/s  "
          f"data {K * CELL * S / ms / 1e6 / 1.073741824:.1f} GiB/s  (min {min(t):.3f} max {max(t):.3f})")
