"""Measurement tool (GPU box): CRC32C-per-chunk kernel variants (tune key 11
scheme x key 12 prefetch) on 9 x 1 MiB cells x S stripes, interleaved over
ROUNDS rounds so clock/thermal drift hits every variant alike; prints the
median per variant (PROBE_VARIANTS="scheme:prefetch,..." to pick).  Also the
target of scripts/pmc_crc.sh."""
import os
import statistics
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "hdfs-native_amd"))
import torch  # noqa: E402

import hdfs_native_ec as H  # noqa: E402

S = int(os.environ.get("PROBE_STRIPES", "256"))
REPS = int(os.environ.get("PROBE_REPS", "10"))
ROUNDS = int(os.environ.get("PROBE_ROUNDS", "5"))
n, cell = 9, 1 << 20
dev = torch.device("cuda:0")
cells = torch.empty((S, n, cell), dtype=torch.uint8, device=dev)
cells.random_(0, 256, generator=torch.Generator(device=dev).manual_seed(1))
coder = H.Coder(6, 3, 0)
# "scheme:prefetch,..." (tune keys 11:12); default: every scheme x prefetch
variants = ([tuple(int(x) for x in v.split(":")) for v in os.environ["PROBE_VARIANTS"].split(",")]
            if os.environ.get("PROBE_VARIANTS") else [(v, p) for v in (1, 2, 3, 4, 9) for p in (1, 2)])
for kv in filter(None, os.environ.get("PROBE_TUNE", "").split(",")):  # extra hec_tune_set keys, e.g. 7=2048
    H.tune_set(*(int(v) for v in kv.split("=")))
ref = H.crc32c_batch(coder, cells)
times = {v: [] for v in variants}
for _ in range(ROUNDS):
    for variant, pf in variants:
        H.tune_set(11, variant)
        H.tune_set(12, pf)
        out = H.crc32c_batch(coder, cells)
        torch.cuda.synchronize()
        assert variant == 9 or torch.equal(out, ref), f"variant {variant} mismatch"
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
        ev[0].record()
        for _ in range(REPS):
            H.crc32c_batch(coder, cells)
        ev[1].record()
        torch.cuda.synchronize()
        times[(variant, pf)].append(ev[0].elapsed_time(ev[1]) / REPS)
H.tune_set(11, 0)
H.tune_set(12, 0)
for (variant, pf), t in times.items():
    ms = statistics.median(t)
    print(f"variant {variant} prefetch {pf}: median {ms:.3f} ms  {n * cell * S / ms / 1e9:.2f} TB/s  "
          f"(min {min(t):.3f} max {max(t):.3f})")
