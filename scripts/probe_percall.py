"""Measurement tool (GPU box): the per-call drop-in (hec_encode / hec_decode,
one RS(6,3) row per call, pageable host buffers) across the values of one
tune key (PROBE_KEY, default 17 = pipeline piece KiB per shard; 0 = default),
interleaved rounds, median us per call.  Every variant's output is checked.

  PROBE_KEY=17 PROBE_VALUES=0,128,512 PROBE_CELL=1048576 python scripts/probe_percall.py
"""
import ctypes
import os
import statistics
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "hdfs-native_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402,F401  (HIP runtime first: see DESIGN.md §1)

import hdfs_native_ec as H  # noqa: E402
from hdfs_native_ec.synth import batch_data  # noqa: E402

K, M = 6, 3
CELL = int(os.environ.get("PROBE_CELL", str(1 << 20)))
KEY = int(os.environ.get("PROBE_KEY", "17"))
THREADS = [int(v) for v in os.environ.get("PROBE_VALUES", "0").split(",")]
CALLS = int(os.environ.get("PROBE_CALLS", "32"))
ROUNDS = int(os.environ.get("PROBE_ROUNDS", "5"))
coder = H.Coder(K, M, 0)
data = batch_data(1, K, CELL, first=99)[0]
par = np.empty((M, CELL), dtype=np.uint8)
rec = np.empty((K, CELL), dtype=np.uint8)
ins = (ctypes.c_void_p * K)(*[data[i].ctypes.data for i in range(K)])
outs = (ctypes.c_void_p * M)(*[par[j].ctypes.data for j in range(M)])
shards = (ctypes.c_void_p * (K + M))(*([0] * M + [data[i].ctypes.data for i in range(M, K)] +
                                        [par[j].ctypes.data for j in range(M)]))
recs = (ctypes.c_void_p * (K + M))(*([rec[i].ctypes.data for i in range(K)] + [0] * M))
lib = H.lib
enc = {t: [] for t in THREADS}
dec = {t: [] for t in THREADS}
ref = None
for _ in range(ROUNDS):
    for t in THREADS:
        H.tune_set(KEY, t)
        assert lib.hec_encode(coder.handle, ins, CELL, outs) == 0
        rec[:] = 0
        assert lib.hec_decode(coder.handle, shards, CELL, recs) == 0
        assert np.array_equal(rec[:M], data[:M]), f"threads {t}: decode mismatch"
        if ref is None:
            ref = par.copy()
        assert np.array_equal(par, ref), f"threads {t}: parity mismatch"
        te = td = 0.0
        for _ in range(CALLS):
            t0 = time.perf_counter()
            lib.hec_encode(coder.handle, ins, CELL, outs)
            t1 = time.perf_counter()
            lib.hec_decode(coder.handle, shards, CELL, recs)
            t2 = time.perf_counter()
            te += t1 - t0
            td += t2 - t1
        enc[t].append(te / CALLS * 1e6)
        dec[t].append(td / CALLS * 1e6)
H.tune_set(KEY, 0)
print(f"RS({K},{M}) one row of {CELL} B cells per call, pageable buffers; os.cpu_count() {os.cpu_count()}, "
      f"sched_getaffinity {len(os.sched_getaffinity(0))}", flush=True)
for t in THREADS:
    e, d = statistics.median(enc[t]), statistics.median(dec[t])
    print(f"key {KEY} = {t}: encode {e:7.1f} us ({K * CELL / e / 1e3 / 1.073741824:6.2f} GiB/s)  "
          f"decode {d:7.1f} us ({K * CELL / d / 1e3 / 1.073741824:6.2f} GiB/s)", flush=True)
