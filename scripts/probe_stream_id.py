"""Probe: the stream properties the work-queue counter sets depend on
(ec_kernels.hip queue_lease, DESIGN.md §3.1 "Counter sets").

  * hipStreamGetId: unique over stream create / destroy while stream
    handles are reused?  Different for hipStreamPerThread in every thread?
  * hipStreamDestroy: does it wait for the stream's queued work (so a
    reused handle never has a predecessor still running)?

Two runtimes: `python probe_stream_id.py torch` uses the HIP runtime a torch
wheel bundles (the tests' and bench's process), `python probe_stream_id.py
rocm` the system ROCm one (/opt/rocm, what a Rust or C consumer links); no
torch is imported in that mode.  Prints one JSON line.
"""
import ctypes
import json
import sys
import threading
import time


def hip_lib(mode):
    if mode == "rocm":
        return ctypes.CDLL("/opt/rocm/lib/libamdhip64.so")
    import torch  # loads torch's libamdhip64 first (one HIP runtime per process)
    torch.cuda.init()
    with open("/proc/self/maps") as f:
        for line in f:
            if "libamdhip64" in line:
                return ctypes.CDLL(line.split()[-1])
    raise RuntimeError("libamdhip64 not mapped")


def main():
    mode = sys.argv[1] if len(sys.argv) > 1 else "torch"
    hip = hip_lib(mode)
    hip.hipMemsetAsync.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_size_t, ctypes.c_void_p]
    hip.hipMalloc.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_size_t]
    assert hip.hipSetDevice(0) == 0
    has_id = hasattr(hip, "hipStreamGetId")
    sid = ctypes.c_ulonglong()
    handles, ids = [], []
    for _ in range(500):
        s = ctypes.c_void_p()
        assert hip.hipStreamCreate(ctypes.byref(s)) == 0
        if has_id:
            assert hip.hipStreamGetId(s, ctypes.byref(sid)) == 0
            ids.append(sid.value)
        handles.append(s.value)
        assert hip.hipStreamDestroy(s) == 0
    per_thread = {}

    def grab(i):
        hip.hipSetDevice(0)
        v = ctypes.c_ulonglong()
        rc = hip.hipStreamGetId(ctypes.c_void_p(2), ctypes.byref(v)) if has_id else None  # hipStreamPerThread
        per_thread[i] = (rc, v.value)

    ts = [threading.Thread(target=grab, args=(i,)) for i in range(4)]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    rc_null = hip.hipStreamGetId(ctypes.c_void_p(0), ctypes.byref(sid)) if has_id else None
    # does hipStreamDestroy wait for the stream's pending work?  Queue 40
    # memsets of 4 GiB on a fresh stream, time the destroy call, then a sync.
    buf = ctypes.c_void_p()
    assert hip.hipMalloc(ctypes.byref(buf), 4 << 30) == 0
    assert hip.hipDeviceSynchronize() == 0
    s = ctypes.c_void_p()
    assert hip.hipStreamCreate(ctypes.byref(s)) == 0
    t0 = time.perf_counter()
    for _ in range(40):
        assert hip.hipMemsetAsync(buf, 1, 4 << 30, s) == 0
    t1 = time.perf_counter()
    assert hip.hipStreamDestroy(s) == 0
    t2 = time.perf_counter()
    assert hip.hipDeviceSynchronize() == 0
    t3 = time.perf_counter()
    print(json.dumps({
        "mode": mode,
        "has_hipStreamGetId": has_id,
        "streams": len(handles),
        "distinct_handles": len(set(handles)),
        "distinct_ids": len(set(ids)),
        "ids_monotone": all(b > a for a, b in zip(ids, ids[1:])),
        "per_thread": per_thread,
        "null_stream": [rc_null, sid.value],
        "destroy": {"enqueue_ms": (t1 - t0) * 1e3, "destroy_ms": (t2 - t1) * 1e3,
                    "sync_after_ms": (t3 - t2) * 1e3},
    }))


if __name__ == "__main__":
    main()
