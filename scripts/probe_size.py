"""Measurement tool (GPU box): does the engine kernel slow down with the
batch footprint, and does physically contiguous HBM (hec_device_alloc with
HEC_ALLOC_CONTIGUOUS: large page fragments, fewer translation entries)
recover it?  Encode launches (K inputs -> R outputs) at several stripe
counts, buffers from torch or from hec_device_alloc, interleaved rounds.

  PROBE_K=10 PROBE_R=4 PROBE_SIZES=256,1024,2048 python scripts/probe_size.py
"""
import os
import statistics
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "hdfs-native_amd"))
import torch  # noqa: E402

import hdfs_native_ec as H  # noqa: E402

K = int(os.environ.get("PROBE_K", "10"))
R = int(os.environ.get("PROBE_R", "4"))
CELL = int(os.environ.get("PROBE_CELL", str(1 << 20)))
SIZES = [int(s) for s in os.environ.get("PROBE_SIZES", "256,1024,2048").split(",")]
ALLOCS = os.environ.get("PROBE_ALLOCS", "torch,default,contig").split(",")
REPS = int(os.environ.get("PROBE_REPS", "6"))
ROUNDS = int(os.environ.get("PROBE_ROUNDS", "3"))
dev = torch.device("cuda:0")
coder = H.Coder(K, R, 0)
stream = torch.cuda.current_stream(dev).cuda_stream
gen = torch.Generator(device=dev).manual_seed(11)


def buffers(kind, S):
    shp_in, shp_out = (S, K, CELL), (S, R, CELL)
    if kind == "torch":
        return None, torch.empty(shp_in, dtype=torch.uint8, device=dev), torch.empty(shp_out, dtype=torch.uint8,
                                                                                     device=dev)
    flags = H.ALLOC_CONTIGUOUS if kind == "contig" else H.ALLOC_DEFAULT
    bi = H.DeviceBuffer(S * K * CELL, 0, flags)
    bo = H.DeviceBuffer(S * R * CELL, 0, flags)
    ti = torch.as_tensor(bi, device=dev).view(shp_in)
    to = torch.as_tensor(bo, device=dev).view(shp_out)
    return (bi, bo), ti, to


results = {}
for S in SIZES:
    sets = {}
    for kind in ALLOCS:
        try:
            keep, ti, to = buffers(kind, S)
        except Exception as e:  # e.g. no contiguous range that large
            print(f"S={S} {kind}: alloc failed: {e}", flush=True)
            continue
        ti.random_(0, 256, generator=gen)
        sets[kind] = (keep, ti, to)
    ref = None
    for kind, (_, ti, to) in sets.items():
        H.encode_batch(coder, ti, to)
        torch.cuda.synchronize()
        if ref is None:
            ref = (ti[:2].clone(), to[:2].clone())
    times = {kind: [] for kind in sets}
    for _ in range(ROUNDS):
        for kind, (_, ti, to) in sets.items():
            ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
            ev[0].record()
            for _ in range(REPS):
                H.encode_batch(coder, ti, to)
            ev[1].record()
            torch.cuda.synchronize()
            times[kind].append(ev[0].elapsed_time(ev[1]) / REPS)
    for kind, t in times.items():
        ms = statistics.median(t)
        gib = S * (K + R) * CELL / 2**30
        print(f"K={K} R={R} S={S} ({gib:.1f} GiB) {kind:8s}: {ms:.3f} ms  {(K + R) * CELL * S / ms / 1e6:.1f} GB/s "
              f"frac {(K + R) * CELL * S / ms / 1e6 / 8000:.4f} (min {min(t):.3f} max {max(t):.3f})", flush=True)
    for kind in list(sets):
        keep, ti, to = sets.pop(kind)
        del ti, to
        if keep:
            for b in keep:
                b.close()
    torch.cuda.empty_cache()
