"""Measurement tool (GPU box): PCIe-inclusive pinned-host pipelines
(hec_encode_host_batch, hec_decode_host_batch with data shards 0..m-1 lost)
across chunk sizes and host copy threads (tune key 14), median of REPS.

  PROBE_K=6 PROBE_M=3 PROBE_S=256 python scripts/probe_hostpath.py
"""
import os
import statistics
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "hdfs-native_amd"))
import torch  # noqa: E402

import hdfs_native_ec as H  # noqa: E402

K = int(os.environ.get("PROBE_K", "6"))
M = int(os.environ.get("PROBE_M", "3"))
S = int(os.environ.get("PROBE_S", "256"))
CELL = int(os.environ.get("PROBE_CELL", str(1 << 20)))
REPS = int(os.environ.get("PROBE_REPS", "5"))
GIB = float(1 << 30)
coder = H.Coder(K, M, 0)
h_in = torch.randint(0, 256, (S, K, CELL), dtype=torch.uint8).pin_memory()
h_par = torch.empty((S, M, CELL), dtype=torch.uint8).pin_memory()
coder.encode_host_batch(h_in.data_ptr(), h_par.data_ptr(), CELL, S, 16)
vert = [None if i < M else h_in[:, i].contiguous().pin_memory() for i in range(K)] + \
       [h_par[:, j].contiguous().pin_memory() for j in range(M)]
vaddr = [None if v is None else v.data_ptr() for v in vert]
h_file = torch.empty((S, K, CELL), dtype=torch.uint8).pin_memory()


def timed(fn):
    fn()
    ts = []
    for _ in range(REPS):
        t0 = time.perf_counter()
        fn()
        ts.append(time.perf_counter() - t0)
    return statistics.median(ts)


for chunk in (8, 16, 32):
    t = timed(lambda: coder.encode_host_batch(h_in.data_ptr(), h_par.data_ptr(), CELL, S, chunk))
    print(f"encode chunk {chunk}: {K * CELL * S / t / GIB:.2f} GiB/s of data")
for threads in (1, 2, 4, 8, 12, 16):
    H.tune_set(14, threads)
    for chunk in (16,):
        h_file.zero_()
        t = timed(lambda: coder.decode_host_batch(vaddr, CELL, S, h_file.data_ptr(), chunk))
        assert torch.equal(h_file, h_in)
        print(f"decode threads {threads} chunk {chunk}: {K * CELL * S / t / GIB:.2f} GiB/s of data")
H.tune_set(14, 0)
