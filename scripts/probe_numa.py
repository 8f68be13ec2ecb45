"""Measurement tool (GPU box): PCIe-inclusive encode / striped-read decode
rates with the pinned host buffers placed on each NUMA node
(hec_host_alloc), against the device's own node (hec_device_numa_node).

  python scripts/probe_numa.py
"""
import glob
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "hdfs-native_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import hdfs_native_ec as H  # noqa: E402

k, m, cell, S, chunk = 6, 3, 1 << 20, 128, 16
nodes = sorted(int(p.rsplit("node", 1)[1]) for p in glob.glob("/sys/devices/system/node/node[0-9]*"))
local = H.device_numa_node(0)
print(f"NUMA nodes {nodes}; device 0 on node {local}", flush=True)
torch.cuda.init()
coder = H.Coder(k, m, 0)
rng = np.random.default_rng(5)
src = rng.integers(0, 256, size=(S, k, cell), dtype=np.uint8)
for node in ([local] if local >= 0 else []) + [n for n in nodes if n != local][:3] + ([local] if local >= 0 else []):
    hin, hout = H.HostBuffer(S * k * cell, 0, node), H.HostBuffer(S * m * cell, 0, node)
    a_in, a_out = hin.array().reshape(S, k, cell), hout.array()
    a_in[:] = src
    coder.encode_host_batch(hin.ptr, hout.ptr, cell, S, chunk)
    ts = []
    for _ in range(5):
        t0 = time.perf_counter()
        coder.encode_host_batch(hin.ptr, hout.ptr, cell, S, chunk)
        ts.append(time.perf_counter() - t0)
    t = sorted(ts)[len(ts) // 2]
    print(f"node {node}{' (local)' if node == local else ''}: encode_host_batch {k * cell * S / t / 2**30:.2f} GiB/s "
          f"of data (median of 5, {S} stripes)", flush=True)
    hin.close()
    hout.close()
