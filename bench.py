#!/usr/bin/env python3
"""Benchmark: device-resident RS(6,3) encode + worst-case decode, 1 MiB cells.

One "step" = one pass of the hot path over one batch: Coder::encode of every
stripe (6 data cells -> 3 parity cells) followed by Coder::decode of every
stripe with data shards {0,1,2} missing (survivors 3,4,5,6,7,8 -> 3
reconstructed cells).  Both are the same gfx950 kernel (6 inputs, 3
outputs), launched through the C ABI on torch's current stream.

value = data bytes coded per second over all ranks, GiB/s, counting k*cell
per stripe for the encode and again for the decode -- the reference
Criterion convention Throughput::Bytes(6 x slice) (rust/benches/ec.rs:30,42).

Multi-GPU: stripes are independent, so every rank codes its own batch of
`--stripes` stripes (weak scaling) -- or its contiguous share of
`--global-stripes` (strong scaling) -- with no data-path collective; the
process group is used only for the barrier and the max-over-ranks time.
`--gpus N` without a launcher's WORLD_SIZE starts N ranks itself
(torch.distributed.run, before anything touches the GPU).

`--ref-cases` instead mirrors rust/benches/ec.rs (matrix inversion, rs-encode
of 6 x 16 MiB, decode with 1/2/3 data slices missing) with the CPU port timed
in the same run.

Prints ONE JSON line on rank 0.
"""
from __future__ import annotations

import argparse
import json
import os
import socket
import subprocess
import sys
import threading
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "hdfs-native_amd"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))

METRIC = "GiB/s device-resident RS(6,3) encode+decode, 1 MiB cells, at 1/2/4/8 MI355X"
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: 8.0 TB/s spec
HBM_COPY_GBS = 6290.0  # measured float4 copy, same guide
GIB = float(1 << 30)
TRAFFIC_FILE = os.path.join(ROOT, "profiles", "pmc_traffic_configs.json")


def log(msg):
    """Progress on stderr (the JSON line stays the only stdout line)."""
    print(f"bench[{os.environ.get('RANK', '0')}] {time.strftime('%H:%M:%S')} {msg}", file=sys.stderr, flush=True)


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--k", "--data-units", dest="k", type=int, default=6)
    ap.add_argument("--m", "--parity-units", dest="m", type=int, default=3)
    ap.add_argument("--cell", type=int, default=1 << 20)
    ap.add_argument("--stripes", type=int, default=1024, help="stripes per GPU (weak scaling)")
    ap.add_argument("--global-stripes", type=int, default=0,
                    help="split this many stripes across the ranks instead (strong scaling)")
    ap.add_argument("--cpu-seconds", type=float, default=10.0, help="CPU baseline budget (0 = skip)")
    ap.add_argument("--cpu-threads", type=int, default=int(os.environ.get("OMP_NUM_THREADS", "0") or 0),
                    help="also time the oracle stripe-parallel on T threads (default $OMP_NUM_THREADS: the "
                         "box's CPU share; 0/1 = single-threaded only)")
    ap.add_argument("--host-path", type=int, default=-1,
                    help="also measure the PCIe-inclusive paths (pinned pipelines and the per-call drop-in): "
                         "1 = yes, 0 = no, -1 = default (yes at N=1)")
    ap.add_argument("--traffic", default=TRAFFIC_FILE)
    ap.add_argument("--tune", default="", help="key=value,... passed to hec_tune_set (measurement)")
    ap.add_argument("--encode-only", action="store_true")
    ap.add_argument("--codec", default="rs", choices=["rs", "xor", "rs-legacy"],
                    help="coding matrix (same kernels): the reference's rs, xor (m = 1) or Hadoop rs-legacy")
    ap.add_argument("--decode-mode", default="uniform", choices=["uniform", "mixed"],
                    help="uniform: data shards 0..m-1 missing in every stripe; mixed: a random pattern of "
                         "1..m missing data shards per stripe (hec_decode_device_mixed)")
    ap.add_argument("--crc", action="store_true",
                    help="also time encode + CRC32C per 512-B chunk of all k+m cells (hec_encode_crc_device)")
    ap.add_argument("--corrupt", default="0.01,0.1",
                    help="with --crc: fractions of stripes with one corrupt survivor for the verified read (none = skip)")
    ap.add_argument("--ref-cases", action="store_true",
                    help="mirror rust/benches/ec.rs instead of the headline step (one JSON line)")
    ap.add_argument("--backend", default="nccl", help="process-group backend (nccl = RCCL; gloo for rehearsals)")
    ap.add_argument("--dry-run", action="store_true",
                    help="launcher / rank / reduction plumbing only: no GPU, no engine, value null (CPU tests)")
    ap.add_argument("--spinup", type=float, default=0.5, help="untimed seconds of steps before warmup")
    ap.add_argument("--extra-configs", type=int, default=-1,
                    help="also time the other multi-GPU BASELINE configs (RS(10,4) 1 MiB x 2048 and RS(6,3) "
                         "64 KiB x 65536, both split over the ranks): 1 = yes, 0 = no, -1 = default (yes for the "
                         "default RS(6,3) run)")
    ap.add_argument("--rows-call-host", action="store_true",
                    help="internal: the host-routine side of host_path.rows_call (child process, no GPU)")
    ap.add_argument("--verify", default="full", choices=["full", "sample"],
                    help="post-timing correctness gate: every stripe against the C oracle (full) or stripe 0")
    return ap.parse_args(argv)


def spawn_ranks(args) -> int:
    """`--gpus N` run directly: start N ranks with torch.distributed.run
    (loopback rendezvous) and return their exit status.  Runs before this
    process touches the GPU."""
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    # torch.distributed.run's own parser prefix-matches "--m" (ambiguous with
    # its --master-* / --max-* options) even after the script: pass the long name
    fwd = ["--parity-units" + a[3:] if a == "--m" or a.startswith("--m=") else a for a in sys.argv[1:]]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           "--master-addr", "127.0.0.1", f"--master-port={port}", os.path.abspath(__file__)] + fwd
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY=os.environ.get("HSA_ENABLE_IPC_MODE_LEGACY", "0"))
    return subprocess.call(cmd, env=env)


def host_info():
    """CPU model and core counts of the host the baseline ran on (§8d)."""
    model = None
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    try:
        usable = len(os.sched_getaffinity(0))
    except AttributeError:
        usable = os.cpu_count()
    return {"cpu_model": model, "nproc": os.cpu_count(), "usable_cpus": usable,
            "omp_num_threads": os.environ.get("OMP_NUM_THREADS")}


def cpu_baseline(k, m, cell, seconds, threads=1):
    """Times the C restatement of the reference loop (oracle, matrix.rs:204-231
    order) on the host: encode + decode({0..m-1} missing) of 1-stripe calls,
    the same work as one Coder::encode + Coder::decode per stripe.  With
    threads > 1 every thread codes its own stripe buffers (stripe-parallel,
    ctypes releases the GIL around each call)."""
    import ctypes

    import numpy as np

    import ec_oracle
    from hdfs_native_ec.synth import batch_data
    lib = ec_oracle.load_c_oracle()
    bufs = []
    for t in range(threads):
        data = batch_data(1, k, cell, first=t)[0]
        par = np.empty((m, cell), dtype=np.uint8)
        rec = np.empty((k, cell), dtype=np.uint8)
        ins = (ctypes.c_void_p * k)(*[data[i].ctypes.data for i in range(k)])
        outs = (ctypes.c_void_p * m)(*[par[j].ctypes.data for j in range(m)])
        shards = (ctypes.c_void_p * (k + m))(*([0] * m + [data[i].ctypes.data for i in range(m, k)] +
                                                [par[j].ctypes.data for j in range(m)]))
        recs = (ctypes.c_void_p * (k + m))(*([rec[i].ctypes.data for i in range(k)] + [0] * m))
        bufs.append((data, par, rec, ins, outs, shards, recs))
    counts = [0] * threads
    stop = time.perf_counter() + seconds

    def work(t):
        _, _, _, ins, outs, shards, recs = bufs[t]
        while time.perf_counter() < stop:
            lib.orc_encode(k, m, ins, cell, outs)
            lib.orc_decode(k, m, shards, cell, recs)
            counts[t] += 1

    t0 = time.perf_counter()
    ths = [threading.Thread(target=work, args=(t,)) for t in range(threads)]
    for th in ths:
        th.start()
    for th in ths:
        th.join()
    el = time.perf_counter() - t0
    for data, _, rec, *_ in bufs:
        assert np.array_equal(rec[:m], data[:m]), "cpu baseline decode mismatch"
    n = sum(counts)
    hi = host_info()
    res = {"value": round(2 * n * k * cell / GIB / el, 4), "unit": "GiB/s", "cores": threads, "kind": "port",
           "sample": f"{n} x (encode + decode 0..{m - 1} missing) of one RS({k},{m}) stripe per thread, "
                     f"{cell} B cells, {el:.1f} s on {threads} thread(s), C restatement oracle/ec_oracle.c "
                     f"(reference Rust path unbuildable here)",
           "host": hi}
    if threads > 1 and hi["usable_cpus"] and threads < hi["usable_cpus"]:
        res["cores_reason"] = (f"the GPU box allots this run a {threads}-CPU share per GPU (OMP_NUM_THREADS="
                               f"{hi['omp_num_threads']}; worker pools are sized to it) although "
                               f"{hi['usable_cpus']} CPUs are visible")
    return res


def cpu_config_batch(H, k, m, cell, stripes, threads, config_stripes=None, source="BASELINE.json configs[0]"):
    """A BASELINE.json config on the CPU (the reference's rust/benches/ec.rs:
    16-63 shape, no GPU): `stripes` stripes encoded, then decoded with data
    shards 0..m-1 missing (the worst case each config names), by the C
    restatement of the reference loop (kind "port", orc_encode_batch /
    orc_decode_batch over contiguous stripe slices) and by the engine's own
    host routine (hec_encode / hec_decode per stripe on host-only coders, as
    the per-row drop-in calls it without a GPU), each on 1 thread and on the
    box's CPU share.  configs[0] (RS(3,2) 1 MiB x 1024) runs whole; for the
    GPU configs `stripes` is a bounded sample of the config's
    `config_stripes` (stated in the record).  The engine's parity is checked
    against the port's for every stripe."""
    import ctypes

    import numpy as np

    import ec_oracle
    lib = ec_oracle.load_c_oracle()
    rng = np.random.default_rng(0x3232)
    data = np.frombuffer(rng.bytes(stripes * k * cell), dtype=np.uint8).reshape(stripes, k, cell)
    present = ((1 << (k + m)) - 1) & ~((1 << m) - 1)
    out = {}
    ref_par = None
    for kind in ("port", "engine_host"):
        for th in sorted({1, max(1, threads)}):
            par = np.empty((stripes, m, cell), dtype=np.uint8)
            rec = np.empty((stripes, m, cell), dtype=np.uint8)
            rcs = []
            # host-only coders (HEC_DEVICE_HOST): the engine's host routine for
            # every row, no device involved
            coders = [H.Coder(k, m, H.HEC_DEVICE_HOST) for _ in range(th)] if kind == "engine_host" else []

            def work(t):
                a, b = stripes * t // th, stripes * (t + 1) // th
                if kind == "port":
                    rcs.append(lib.orc_encode_batch(k, m, data[a:b].ctypes.data, cell, b - a, par[a:b].ctypes.data))
                    rcs.append(lib.orc_decode_batch(k, m, data[a:b].ctypes.data, par[a:b].ctypes.data, cell, b - a,
                                                    ctypes.c_uint64(present), rec[a:b].ctypes.data))
                    return
                h = coders[t].handle
                for s in range(a, b):
                    ins = (ctypes.c_void_p * k)(*[data[s, i].ctypes.data for i in range(k)])
                    outs = (ctypes.c_void_p * m)(*[par[s, j].ctypes.data for j in range(m)])
                    rcs.append(H.lib.hec_encode(h, ins, cell, outs))
                for s in range(a, b):
                    shards = (ctypes.c_void_p * (k + m))(*([0] * m + [data[s, i].ctypes.data for i in range(m, k)] +
                                                            [par[s, j].ctypes.data for j in range(m)]))
                    recs = (ctypes.c_void_p * (k + m))(*([rec[s, i].ctypes.data for i in range(m)] + [0] * (k)))
                    rcs.append(H.lib.hec_decode(h, shards, cell, recs))

            t0 = time.perf_counter()
            ths = [threading.Thread(target=work, args=(t,)) for t in range(th)]
            for x in ths:
                x.start()
            for x in ths:
                x.join()
            el = time.perf_counter() - t0
            for c in coders:
                c.close()
            assert all(rc == 0 for rc in rcs), f"cpu config {kind} rc {set(rcs)}"
            assert np.array_equal(rec, data[:, :m]), f"cpu config {kind} decode mismatch"
            if ref_par is None:
                ref_par = par
            else:
                assert np.array_equal(par, ref_par), f"cpu config {kind} parity != port parity"
            out[f"{kind}_{th}t"] = {"value": round(2 * stripes * k * cell / GIB / el, 4), "unit": "GiB/s",
                                    "cores": th, "seconds": round(el, 3),
                                    "kind": "port" if kind == "port" else "engine"}
    whole = config_stripes is None or config_stripes == stripes
    return {"config": f"RS({k},{m}) {cell} B cells, {stripes}-stripe batch, encode + decode data 0..{m - 1} missing "
                      f"({source}, rust/benches/ec.rs:16-63)",
            "stripes_timed": stripes, "config_stripes": config_stripes or stripes,
            "sample": "the whole batch" if whole else
                      f"a bounded sample: {stripes} of the config's {config_stripes} stripes (same per-stripe work; "
                      f"stripes are independent, so GiB/s is the config's rate on this host)",
            "legs": out, "host_isa": H.host_isa(), "host": host_info(),
            "note": "port = oracle/ec_oracle.c (restates matrix.rs:204-231; the Rust path is unbuildable here), "
                    "engine = hec_encode / hec_decode per stripe on the host routine; every timed stripe's "
                    "engine parity == port parity, rebuilt cells == data"}


def traffic_for(path, k, m, cell, stripes, mode):
    """PMC HBM bytes per launch for this exact config, from the committed
    per-config profile (scripts/profile_configs.py: FETCH_SIZE / WRITE_SIZE
    passes of this same command on this tree), else None."""
    if not os.path.exists(path):
        return None, None
    with open(path) as f:
        tr = json.load(f)
    for c in tr.get("configs", []):
        if (c["k"], c["m"], c["cell"], c["stripes"], c.get("decode_mode", "uniform")) == (k, m, cell, stripes, mode):
            return c["hbm_bytes_per_launch"], f"{os.path.relpath(path, ROOT)}:{c['config']} ({tr.get('tag')})"
    return None, None


def rank_identity(rank, local, device, shared=False):
    """(rank, device ordinal, PCI location, UUID) of this rank's GPU, so an
    N-rank line shows that the ranks ran on N distinct cards;
    device None = no GPU (dry run)."""
    ident = {"rank": rank, "local_rank": int(os.environ.get("LOCAL_RANK", "0")), "device": device,
             "host": socket.gethostname(), "pci_domain_id": None, "pci_bus_id": None, "pci_device_id": None,
             "uuid": None, "shared_gpu": bool(shared)}
    if device is not None:
        import torch
        p = torch.cuda.get_device_properties(device)
        ident.update({"pci_domain_id": getattr(p, "pci_domain_id", None), "pci_bus_id": getattr(p, "pci_bus_id", None),
                      "pci_device_id": getattr(p, "pci_device_id", None), "uuid": str(getattr(p, "uuid", "")) or None,
                      "name": p.name})
    return ident


def gather_ranks(ident, world, dist):
    """Every rank's identity, in rank order (all_gather_object over the
    process group; the barrier / max-reduction group, no data)."""
    if world == 1 or not dist.is_initialized():
        return [ident]
    out = [None] * world
    dist.all_gather_object(out, ident)
    return sorted(out, key=lambda r: r["rank"])


def gather_list(value, world, dist):
    """Every rank's `value`, in rank order (all_gather_object over the
    process group; timing and shard metadata only, no data)."""
    if world == 1 or not dist.is_initialized():
        return [value]
    out = [None] * world
    dist.all_gather_object(out, value)
    return out


def process_group_info(args, world, dist):
    init = dist.is_available() and dist.is_initialized()
    return {"backend": dist.get_backend() if init else None, "requested_backend": args.backend,
            "world_size": dist.get_world_size() if init else 1, "env_world_size": world}


def dry_run(args, world, rank):
    """Plumbing only: ranks, rendezvous, the barrier and the max/sum
    reductions bench.py uses, the JSON line -- no GPU and no engine."""
    import torch.distributed as dist

    from hdfs_native_ec.dist import max_over_ranks, shard_range, sum_over_ranks
    if world > 1:
        dist.init_process_group("gloo")
    if args.global_stripes:
        first, S = shard_range(args.global_stripes, world, rank)
    else:
        first, S = rank * args.stripes, args.stripes
    t0 = time.perf_counter()
    if world > 1:
        dist.barrier()
    el = max_over_ranks(time.perf_counter() - t0)
    total = sum_over_ranks(float(S))
    ranks = gather_ranks(rank_identity(rank, int(os.environ.get("LOCAL_RANK", "0")), None), world, dist)
    extra = {}
    for cfg in EXTRA_CONFIGS:  # the same per-rank split extra_configs() runs
        c_first, share = shard_range(cfg["global_stripes"], world, rank)
        extra[cfg["name"]] = {"scaling": "strong", "stripes_per_gpu_rank0": share,
                              "stripes_summed_over_ranks": int(sum_over_ranks(float(share))), "value_GiBps": None,
                              "shards": gather_list([c_first, share], world, dist)}
    shards = gather_list([first, S], world, dist)
    if rank == 0:
        print(json.dumps({"metric": METRIC, "value": None, "unit": "GiB/s", "n_gpus": world, "dry_run": True,
                          "scaling": "strong" if args.global_stripes else "weak",
                          "config": {"k": args.k, "m": args.m, "cell_bytes": args.cell, "stripes_per_gpu": S,
                                     "global_stripes": args.global_stripes or S * world,
                                     "stripes_summed_over_ranks": int(total), "shards": shards},
                          "extra_configs": extra, "ranks": ranks,
                          "process_group": process_group_info(args, world, dist),
                          "max_elapsed_s": el}), flush=True)
    if world > 1:
        dist.destroy_process_group()


def per_call_leg(H, k, m, cell, calls, oracle_lib):
    """The drop-in exactly as the reference calls it: one Coder::encode per
    row (CellBuffer::encode, block_writer.rs:838) and one Coder::decode per
    row (ec/mod.rs:71-72), pageable host buffers, synchronous; the CPU port
    per call beside it."""
    import ctypes

    import numpy as np

    from hdfs_native_ec.synth import batch_data
    coder = H.Coder(k, m, 0)
    data = batch_data(1, k, cell, first=99)[0]
    par = np.empty((m, cell), dtype=np.uint8)
    rec = np.empty((k, cell), dtype=np.uint8)
    ins = (ctypes.c_void_p * k)(*[data[i].ctypes.data for i in range(k)])
    outs = (ctypes.c_void_p * m)(*[par[j].ctypes.data for j in range(m)])
    shards = (ctypes.c_void_p * (k + m))(*([0] * m + [data[i].ctypes.data for i in range(m, k)] +
                                            [par[j].ctypes.data for j in range(m)]))
    recs = (ctypes.c_void_p * (k + m))(*([rec[i].ctypes.data for i in range(k)] + [0] * m))
    lib = H.lib
    res = {}
    for name, fn in (("engine", lambda: (lib.hec_encode(coder.handle, ins, cell, outs),
                                         lib.hec_decode(coder.handle, shards, cell, recs))),
                     ("cpu_port", lambda: (oracle_lib.orc_encode(k, m, ins, cell, outs),
                                           oracle_lib.orc_decode(k, m, shards, cell, recs)))):
        n = calls if name == "engine" else max(2, calls // 16)
        for _ in range(2):
            rc = fn()
            assert rc == (0, 0), f"{name} per-call rc {rc}"
        te = td = 0.0
        for _ in range(n):
            t0 = time.perf_counter()
            a = (lib.hec_encode(coder.handle, ins, cell, outs) if name == "engine"
                 else oracle_lib.orc_encode(k, m, ins, cell, outs))
            t1 = time.perf_counter()
            b = (lib.hec_decode(coder.handle, shards, cell, recs) if name == "engine"
                 else oracle_lib.orc_decode(k, m, shards, cell, recs))
            t2 = time.perf_counter()
            assert a == 0 and b == 0
            te += t1 - t0
            td += t2 - t1
        assert np.array_equal(rec[:m], data[:m]), f"{name} per-call decode mismatch"
        res[name] = {"encode_GiBps": round(n * k * cell / te / GIB, 3), "decode_GiBps": round(n * k * cell / td / GIB, 3),
                     "encode_us_per_call": round(te / n * 1e6, 1), "decode_us_per_call": round(td / n * 1e6, 1),
                     "calls": n}
    coder.close()
    res["note"] = (f"one RS({k},{m}) row of {cell} B cells per call, pageable host buffers: hec_encode then "
                   f"hec_decode with data shards 0..{m - 1} missing (the Rust shim's per-row calls); cpu_port = "
                   "oracle/ec_oracle.c on one core, same calls")
    return res


def per_call_sizes(H, k, m, oracle_lib):
    """The per-call drop-in (hec_encode + hec_decode of one row, pageable
    buffers) by row size, three ways -- the coder's default routing (rows up
    to its host limit on the host routine), the device forced (host limit 0)
    and the host routine forced -- beside the CPU port of the reference loop
    on one core; the crossover is the smallest size where the device wins."""
    import ctypes

    import numpy as np

    from hdfs_native_ec.synth import batch_data
    sizes = [16, 512, 4096, 16384, 65536, 262144, 1 << 20]
    coder = H.Coder(k, m, 0)
    default_limit = coder.host_limit
    lib = H.lib
    rows = []
    for n in sizes:
        data = batch_data(1, k, n, first=n)[0]
        par = np.empty((m, n), dtype=np.uint8)
        rec = np.empty((k, n), dtype=np.uint8)
        ins = (ctypes.c_void_p * k)(*[data[i].ctypes.data for i in range(k)])
        outs = (ctypes.c_void_p * m)(*[par[j].ctypes.data for j in range(m)])
        shards = (ctypes.c_void_p * (k + m))(*([0] * m + [data[i].ctypes.data for i in range(m, k)] +
                                                [par[j].ctypes.data for j in range(m)]))
        recs = (ctypes.c_void_p * (k + m))(*([rec[i].ctypes.data for i in range(k)] + [0] * m))
        row = {"shard_bytes": n}
        for name, limit in (("engine", default_limit), ("engine_device", 0), ("engine_host", 1 << 40),
                            ("cpu_port", None)):
            if limit is not None:
                coder.host_limit = limit
                enc = lambda: lib.hec_encode(coder.handle, ins, n, outs)  # noqa: E731
                dec = lambda: lib.hec_decode(coder.handle, shards, n, recs)  # noqa: E731
            else:
                enc = lambda: oracle_lib.orc_encode(k, m, ins, n, outs)  # noqa: E731
                dec = lambda: oracle_lib.orc_decode(k, m, shards, n, recs)  # noqa: E731
            assert enc() == 0 and dec() == 0
            budget = 0.15 if limit is not None else 0.3
            per = {}
            for op, fn in (("encode", enc), ("decode", dec)):
                reps, t = 0, 0.0
                t0 = time.perf_counter()
                while t < budget or reps < 3:
                    fn()
                    reps += 1
                    t = time.perf_counter() - t0
                per[op] = t / reps
            assert np.array_equal(rec[:m], data[:m]), f"per-call {name} {n}"
            row[name] = {"encode_us": round(per["encode"] * 1e6, 3), "decode_us": round(per["decode"] * 1e6, 3),
                         "encode_GiBps": round(k * n / per["encode"] / GIB, 3)}
        rows.append(row)
    # cold: every call codes a different row of a 1 GiB pool (4x the host's
    # L3), so neither route finds its input in the CPU caches -- the case a
    # writer or reader streaming a file meets (the hot figures
    # above flatter the host routine at 1 MiB)
    cold_sizes = [4096, 65536, 262144, 1 << 20, 4 << 20]
    pool = np.frombuffer(np.random.default_rng(0xC01D).bytes(1 << 30), dtype=np.uint8)
    par_pool = np.empty((1 << 30) * m // k, dtype=np.uint8)
    rec_pool = np.empty((1 << 30) * m // k, dtype=np.uint8)
    par_pool[::4096] = 0  # touch: first-touch page faults outside the timed calls
    rec_pool[::4096] = 0
    for n in cold_sizes:
        R = (1 << 30) // (k * n)
        dv = pool[:R * k * n].reshape(R, k, n)
        pv = par_pool[:R * m * n].reshape(R, m, n)
        rv = rec_pool[:R * m * n].reshape(R, m, n)
        ins = [(ctypes.c_void_p * k)(*[dv[r, i].ctypes.data for i in range(k)]) for r in range(R)]
        outs = [(ctypes.c_void_p * m)(*[pv[r, j].ctypes.data for j in range(m)]) for r in range(R)]
        shards = [(ctypes.c_void_p * (k + m))(*([0] * m + [dv[r, i].ctypes.data for i in range(m, k)] +
                                                [pv[r, j].ctypes.data for j in range(m)])) for r in range(R)]
        recs = [(ctypes.c_void_p * (k + m))(*([rv[r, i].ctypes.data for i in range(m)] + [0] * k)) for r in range(R)]
        row = next((x for x in rows if x["shard_bytes"] == n), None)
        if row is None:
            row = {"shard_bytes": n}
            rows.append(row)
        for name, limit in (("engine_device", 0), ("engine_host", 1 << 40)):
            coder.host_limit = limit
            per = {}
            for op in ("encode", "decode"):
                reps, t, r = 0, 0.0, 0
                t0 = time.perf_counter()
                while t < 0.25 or reps < 3:
                    rc = (lib.hec_encode(coder.handle, ins[r], n, outs[r]) if op == "encode"
                          else lib.hec_decode(coder.handle, shards[r], n, recs[r]))
                    assert rc == 0
                    r = (r + 1) % R
                    reps += 1
                    t = time.perf_counter() - t0
                per[op] = t / reps
            row.setdefault("cold", {})[name] = {"encode_us": round(per["encode"] * 1e6, 2),
                                                "decode_us": round(per["decode"] * 1e6, 2),
                                                "encode_GiBps": round(k * n / per["encode"] / GIB, 3),
                                                "rows_in_pool": R}
        assert np.array_equal(rv[0], dv[0, :m]), f"cold per-call decode {n}"
    del pool, par_pool, rec_pool
    rows.sort(key=lambda x: x["shard_bytes"])
    coder.host_limit = default_limit
    coder.close()
    cross = next((r["shard_bytes"] for r in rows if "engine_device" in r and
                  r["engine_device"]["encode_us"] < r["engine_host"]["encode_us"]), None)
    cross_cold = next((r["shard_bytes"] for r in rows if "cold" in r and
                       r["cold"]["engine_device"]["encode_us"] < r["cold"]["engine_host"]["encode_us"]), None)
    return {"rows": rows, "default_host_limit": default_limit, "host_isa": H.host_isa(),
            "device_beats_host_from_cold": cross_cold,
            "device_beats_host_from": cross,
            "note": f"RS({k},{m}), one row per hec_encode / hec_decode (data shards 0..{m - 1} missing), pageable "
                    "buffers; engine = default routing, engine_device = host limit 0, engine_host = the engine's "
                    "host routine forced; cpu_port = oracle/ec_oracle.c on one core; cold = each call on a "
                    "different row of a 1 GiB pool (4x the L3), device forced vs host routine forced"}


ROWS_CALL_SHAPES = (1, 4)  # rows per call: the reference's per-row calls, the row-batched writer / reader's 4


def _rows_pools(k, cell, rows, pool_bytes):
    """Calls' worth of slots (one call's buffers each) so that the data of a
    pass over them spans >= pool_bytes: every call's buffers are cold."""
    return max(3, pool_bytes // (rows * k * cell))


def rows_call_host(k, m, cell, seconds=0.4):
    """Child process (no GPU): the engine's host routine on pageable buffers
    at the writer's / reader's call shapes, cold, on however many threads
    HEC_HOST_THREADS gives it.  Prints one JSON object."""
    import ctypes

    import numpy as np

    import hdfs_native_ec as H
    out = {}
    coder = H.Coder(k, m, H.HEC_DEVICE_HOST)
    for rows in ROWS_CALL_SHAPES:
        n = rows * cell  # a vertical stripe: each shard's `rows` cells back to back
        slots = _rows_pools(k, cell, rows, 1 << 30)
        vert = np.frombuffer(np.random.default_rng(rows).bytes(slots * (k + m) * n), dtype=np.uint8).reshape(
            slots, k + m, n)
        rec = np.empty((slots, m, n), dtype=np.uint8)
        rec[:, :, ::4096] = 0
        res = {}
        for op in ("encode", "decode"):
            calls, t, r = 0, 0.0, 0
            c0, t0 = time.process_time(), time.perf_counter()
            while t < seconds or calls < 3:
                v = vert[r]
                if op == "encode":
                    rc = H.lib.hec_encode(coder.handle, (ctypes.c_void_p * k)(*[v[i].ctypes.data for i in range(k)]),
                                          n, (ctypes.c_void_p * m)(*[v[k + j].ctypes.data for j in range(m)]))
                else:  # data shards 0..m-1 lost, rebuilt from the rest
                    sh = (ctypes.c_void_p * (k + m))(*([0] * m + [v[i].ctypes.data for i in range(m, k + m)]))
                    outs = (ctypes.c_void_p * (k + m))(*([rec[r, i].ctypes.data for i in range(m)] + [0] * k))
                    rc = H.lib.hec_decode(coder.handle, sh, n, outs)
                assert rc == 0, rc
                r = (r + 1) % slots
                calls += 1
                t = time.perf_counter() - t0
            cpu = time.process_time() - c0
            gib = calls * k * n / GIB
            res[op] = {"us_per_call": round(t / calls * 1e6, 1), "GiBps": round(gib / t, 2),
                       "cpu_core_s_per_GiB": round(cpu / gib, 4), "calls": calls}
        # slot 0 was encoded first: its rebuilt shards == the originals
        assert np.array_equal(rec[0], vert[0, :m]), f"rows={rows}: host decode != data"
        out[f"rows={rows}"] = res
        del vert, rec
    coder.close()
    out["threads"] = int(os.environ.get("HEC_HOST_THREADS", "4"))
    out["isa"] = H.host_isa()
    print(json.dumps(out), flush=True)


def rows_call_leg(H, k, m, cell, coder, torch):
    """The striped writer's and reader's call shapes, cold (each call on a
    different slice of a >= 1 GiB pool): `rows` rows per call, 1 (the
    reference: block_writer.rs:838, ec/mod.rs:71-72) or 4 (the row-batched
    writer / reader, rust/src/hdfs/ec_rows.rs).  device = the engine's pinned
    pipeline on page-locked buffers (hec_encode_host_batch: file-order rows
    in, parity out, one stripe per pipeline chunk; hec_decode_host_batch:
    vertical shards in, file-order rows out, data shards 0..m-1 lost);
    host_<T>t = the engine's host routine on pageable buffers (hec_encode /
    hec_decode of the vertical stripes) on T threads, each in a child process
    that never touches the GPU (HEC_HOST_THREADS=T).  Wall time per call and
    CPU core-seconds per GiB of data (process CPU time over the calls: every
    thread of the process, the HIP runtime's included)."""
    import numpy as np
    res = {}
    dev_res = {}
    for rows in ROWS_CALL_SHAPES:
        slots = _rows_pools(k, cell, rows, 1 << 30)
        d_bytes, p_bytes = rows * k * cell, rows * m * cell
        hb_data = H.HostBuffer(slots * d_bytes)
        hb_par = H.HostBuffer(slots * p_bytes)
        hb_file = H.HostBuffer(slots * d_bytes)
        data = hb_data.array().reshape(slots, rows, k, cell)
        par = hb_par.array().reshape(slots, rows, m, cell)
        filev = hb_file.array().reshape(slots, rows, k, cell)
        data[:] = np.frombuffer(np.random.default_rng(7 + rows).bytes(slots * d_bytes), dtype=np.uint8).reshape(
            data.shape)
        filev[:, :, :, ::4096] = 0
        par[:, :, :, ::4096] = 0
        # the reader's vertical shards: [k+m][rows*cell] per slot, pinned
        hb_vert = H.HostBuffer(slots * (k + m) * rows * cell)
        vert = hb_vert.array().reshape(slots, k + m, rows * cell)
        r_res = {}
        for op in ("encode", "decode"):
            calls, t, r = 0, 0.0, 0
            fn = (lambda s: coder.encode_host_batch(data[s].ctypes.data, par[s].ctypes.data, cell, rows, 1)) \
                if op == "encode" else \
                (lambda s: coder.decode_host_batch([None] * m + [vert[s, i].ctypes.data for i in range(m, k + m)],
                                                   cell, rows, filev[s].ctypes.data, 1))
            if op == "decode":  # vertical shards of the encoded rows (untimed)
                for s in range(slots):
                    vert[s, :k] = data[s].transpose(1, 0, 2).reshape(k, rows * cell)
                    vert[s, k:] = par[s].transpose(1, 0, 2).reshape(m, rows * cell)
            fn(0)
            c0, t0 = time.process_time(), time.perf_counter()
            while t < 0.4 or calls < 3:
                fn(r)
                r = (r + 1) % slots
                calls += 1
                t = time.perf_counter() - t0
            cpu = time.process_time() - c0
            gib = calls * d_bytes / GIB
            r_res[op] = {"us_per_call": round(t / calls * 1e6, 1), "GiBps": round(gib / t, 2),
                         "cpu_core_s_per_GiB": round(cpu / gib, 4), "calls": calls}
        # every slot's rows came back whole (data 0..m-1 rebuilt), and slot
        # 0's parity matches the host routine's
        assert np.array_equal(filev, data), f"rows={rows}: decode_host_batch file rows != data"
        hc = H.Coder(k, m, H.HEC_DEVICE_HOST)
        want = np.empty((rows, m, cell), dtype=np.uint8)
        hc.encode_host_batch(data[0].ctypes.data, want.ctypes.data, cell, rows, 1)
        hc.close()
        assert np.array_equal(want, par[0]), f"rows={rows}: device parity != host routine parity"
        dev_res[f"rows={rows}"] = r_res
        for b in (hb_data, hb_par, hb_file, hb_vert):
            b.close()
    res["device_pinned"] = dev_res
    for threads in (1, int(os.environ.get("HEC_HOST_THREADS", "4") or 4)):
        env = dict(os.environ, HEC_HOST_THREADS=str(threads), HIP_VISIBLE_DEVICES="", ROCR_VISIBLE_DEVICES="")
        out = subprocess.run([sys.executable, os.path.abspath(__file__), "--rows-call-host", "--k", str(k),
                              "--m", str(m), "--cell", str(cell)], capture_output=True, text=True, env=env,
                             timeout=300)
        assert out.returncode == 0, out.stderr[-2000:]
        res[f"host_{threads}t"] = json.loads(out.stdout.strip().splitlines()[-1])
    res["note"] = (f"RS({k},{m}) {cell} B cells, rows per call 1 (reference) and 4 (row-batched writer / reader), "
                   "cold pools; device_pinned = hec_encode_host_batch / hec_decode_host_batch on page-locked "
                   "buffers (data shards 0..m-1 lost), host_<T>t = the host routine on pageable vertical stripes "
                   "(hec_encode / hec_decode) on T threads; cpu_core_s_per_GiB = process CPU time / data GiB")
    return res


def ref_cases(args):
    """rust/benches/ec.rs:5-64 mirrored: matrix-inversion/invert (RS(6,3)
    rows 3..8), rs-encode/encode (one stripe of 6 x 16 MiB), and
    rs-decode/decode-{1,2,3}-slice (data shards 0 / 0,1 / 0,1,2 missing).
    Throughput is the reference's Throughput::Bytes(6 x slice).  Each case:
    the engine device-resident (one stripe, hec_*_device + stream sync), the
    engine's host drop-in (hec_encode / hec_decode on pageable buffers), and
    the CPU port (oracle/ec_oracle.c, 1 core) in the same run."""
    import ctypes

    import numpy as np
    import torch

    import ec_oracle
    import hdfs_native_ec as H
    from hdfs_native_ec.synth import bench_counter_shards
    olib = ec_oracle.load_c_oracle()
    k, m, slice_ = 6, 3, 16 << 20
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    coder = H.Coder(k, m, 0)
    stream = torch.cuda.current_stream(dev)
    out = {"metric": "rust/benches/ec.rs cases (Criterion throughput = 6 x slice bytes)", "unit": "GiB/s",
           "n_gpus": 1, "slice_bytes": slice_, "cases": {}}

    def timeit(fn, reps, sync=None):
        fn()
        if sync:
            sync()
        t0 = time.perf_counter()
        for _ in range(reps):
            fn()
        if sync:
            sync()
        return (time.perf_counter() - t0) / reps

    # matrix-inversion/invert
    enc = H.gen_rs_matrix(k, m)
    sub = [enc[r] for r in range(3, 9)]
    flat = (ctypes.c_uint8 * 36)()
    flat_o = (ctypes.c_uint8 * 36)()

    def inv_engine():
        ctypes.memmove(flat, bytes(v for row in sub for v in row), 36)
        assert H.lib.hec_matrix_invert(flat, 6) == 0

    def inv_port():
        ctypes.memmove(flat_o, bytes(v for row in sub for v in row), 36)
        assert olib.orc_invert(flat_o, 6) == 0

    t_e, t_p = timeit(inv_engine, 20000), timeit(inv_port, 20000)
    assert bytes(flat) == bytes(flat_o)
    out["cases"]["matrix-inversion/invert"] = {"engine_host_us": round(t_e * 1e6, 3), "cpu_port_us": round(t_p * 1e6, 3),
                                               "note": "6x6 Gauss-Jordan over GF(2^8), host code (incl. a 36-B copy)"}

    # rs-encode/encode: one stripe, the bench's big-endian counter fill
    data = list(bench_counter_shards(k, slice_))
    d = torch.from_numpy(np.stack(data)).unsqueeze(0).to(dev)
    p = torch.empty((1, m, slice_), dtype=torch.uint8, device=dev)
    t_dev = timeit(lambda: H.encode_batch(coder, d, p), 50, torch.cuda.synchronize)
    ins = (ctypes.c_void_p * k)(*[x.ctypes.data for x in data])
    par = [np.empty(slice_, dtype=np.uint8) for _ in range(m)]
    outs = (ctypes.c_void_p * m)(*[x.ctypes.data for x in par])
    t_host = timeit(lambda: H.lib.hec_encode(coder.handle, ins, slice_, outs), 10)
    par_o = [np.empty(slice_, dtype=np.uint8) for _ in range(m)]
    outs_o = (ctypes.c_void_p * m)(*[x.ctypes.data for x in par_o])
    t_port = timeit(lambda: olib.orc_encode(k, m, ins, slice_, outs_o), 2)
    assert all(np.array_equal(a, b) for a, b in zip(par, par_o))
    assert all(np.array_equal(p[0, j].cpu().numpy(), par_o[j]) for j in range(m))
    gib = k * slice_ / GIB
    out["cases"]["rs-encode/encode"] = {"device_GiBps": round(gib / t_dev, 2), "host_call_GiBps": round(gib / t_host, 3),
                                        "cpu_port_GiBps": round(gib / t_port, 4),
                                        "device_ms": round(t_dev * 1e3, 4)}

    # rs-decode/decode-{1,2,3}-slice
    full = data + par_o
    dp_all = torch.cat([d[0], p[0]]).unsqueeze(0)  # [1, k+m, slice]
    for e in (1, 2, 3):
        miss = list(range(e))
        shard_ptrs = [None if i in miss else dp_all.data_ptr() + i * slice_ for i in range(k + m)]
        rec = torch.empty((1, k, slice_), dtype=torch.uint8, device=dev)
        rp = [rec.data_ptr() + i * slice_ for i in range(k)]
        strides = [(k + m) * slice_] * (k + m)

        def dec_dev():
            coder.decode_device(shard_ptrs, strides, rp, [k * slice_] * k, slice_, 1, stream.cuda_stream)

        t_dev = timeit(dec_dev, 50, torch.cuda.synchronize)
        assert all(torch.equal(rec[0, i], d[0, i]) for i in miss)
        hs = (ctypes.c_void_p * (k + m))(*[0 if i in miss else full[i].ctypes.data for i in range(k + m)])
        hrec = [np.empty(slice_, dtype=np.uint8) for _ in range(k)]
        hout = (ctypes.c_void_p * (k + m))(*([x.ctypes.data for x in hrec] + [0] * m))
        t_host = timeit(lambda: H.lib.hec_decode(coder.handle, hs, slice_, hout), 10)
        orec = [np.empty(slice_, dtype=np.uint8) for _ in range(k)]
        oout = (ctypes.c_void_p * (k + m))(*([x.ctypes.data for x in orec] + [0] * m))
        t_port = timeit(lambda: olib.orc_decode(k, m, hs, slice_, oout), 2)
        assert all(np.array_equal(hrec[i], data[i]) and np.array_equal(orec[i], data[i]) for i in miss)
        out["cases"][f"rs-decode/decode-{e}-slice"] = {
            "device_GiBps": round(gib / t_dev, 2), "host_call_GiBps": round(gib / t_host, 3),
            "cpu_port_GiBps": round(gib / t_port, 4), "device_ms": round(t_dev * 1e3, 4)}
    out["note"] = ("device = one stripe already in HBM (hec_encode_device / hec_decode_device + sync); host_call = "
                   "the drop-in on pageable host buffers (what the Rust shim calls); cpu_port = the C restatement "
                   "of the reference loop on 1 core (the reference Rust bench cannot be built here: no cargo)")
    out["host"] = host_info()
    coder.close()
    print(json.dumps(out), flush=True)


def main():
    args = parse()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(spawn_ranks(args))  # before anything touches the GPU
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    if args.dry_run:
        return dry_run(args, world, rank)
    if args.rows_call_host:
        return rows_call_host(args.k, args.m, args.cell)
    if args.ref_cases:
        return ref_cases(args)

    import numpy as np
    import torch
    import torch.distributed as dist

    import hdfs_native_ec as H
    from hdfs_native_ec.dist import max_over_ranks, shard_range, sum_over_ranks

    local = int(os.environ.get("LOCAL_RANK", "0"))
    ndev = torch.cuda.device_count()
    shared = local >= ndev
    if shared:
        if args.backend == "nccl" or ndev == 0:
            # one rank per GPU is the contract: a world larger than the node's
            # GPU count would fold ranks onto shared cards and over-report
            log(f"refusing: LOCAL_RANK {local} but {ndev} GPU(s) visible (backend {args.backend}); "
                "one rank per GPU")
            sys.exit(3)
        local %= ndev  # gloo rehearsal only: ranks share cards, flagged in the line
    if world > 1:
        torch.cuda.set_device(local)
        if args.backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(args.backend)
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)
    # --tune: measurement knobs exist only in the HEC_EXPERIMENTAL build
    # (include/hdfs_ec_amd_exp.h); the coder then runs on that library
    xlib = H.experimental_lib() if args.tune else None
    for kv in filter(None, args.tune.split(",")):
        key, val = kv.split("=")
        H.tune_set(int(key), int(val), xlib)

    k, m, cell = args.k, args.m, args.cell
    if args.global_stripes:
        first, S = shard_range(args.global_stripes, world, rank)
        scaling = "strong"
    else:
        first, S = rank * args.stripes, args.stripes
        scaling = "weak"
    coder = H.Coder(k, m, local, codec=args.codec, lib=xlib)
    g = torch.Generator(device=dev)
    g.manual_seed(0x5EED_EC00 + first)
    data = torch.randint(0, 256, (S, k, cell), dtype=torch.uint8, device=dev, generator=g)
    parity = torch.empty((S, m, cell), dtype=torch.uint8, device=dev)
    mixed = args.decode_mode == "mixed"
    # reconstructed data: [S, m, cell] for the uniform worst case (shards
    # 0..m-1), [S, k, cell] when every stripe has its own pattern
    rec = torch.empty((S, k if mixed else m, cell), dtype=torch.uint8, device=dev)
    stream = torch.cuda.current_stream(dev)
    sp = stream.cuda_stream

    dp, ds = H.stripe_layout_ptrs(data, k)
    pp, ps = H.stripe_layout_ptrs(parity, m)
    rp, rs = H.stripe_layout_ptrs(rec, k if mixed else m)
    miss = list(range(m))  # worst case: m data shards missing
    shard_ptrs = [None if i in miss else dp[i] for i in range(k)] + pp
    out_ptrs = [rp[i] if i in miss else 0 for i in range(k)]
    out_strides = [rs[0]] * k
    if mixed:
        rng = np.random.default_rng(0x5EED_EC00 + first)
        full = (1 << (k + m)) - 1
        masks, erased = [], 0
        for _ in range(S):
            e = int(rng.integers(1, m + 1))
            lost = rng.choice(k, size=e, replace=False)
            masks.append(full & ~sum(1 << int(i) for i in lost))
            erased += e
        ws = torch.empty(coder.decode_mixed_workspace_size(S), dtype=torch.uint8, device=dev)
        mixed_ptrs, mixed_strides = dp + pp, ds + ps

    def encode():
        coder.encode_device(dp, ds, pp, ps, cell, S, sp)

    def decode():
        if mixed:
            coder.decode_device_mixed(mixed_ptrs, mixed_strides, rp, rs, masks, cell, S, ws.data_ptr(), ws.numel(),
                                      sp)
        else:
            coder.decode_device(shard_ptrs, ds + ps, out_ptrs, out_strides, cell, S, sp)

    def step(events=None):
        if events is not None:
            events[0].record(stream)
        encode()
        if events is not None:
            events[1].record(stream)
        if not args.encode_only:
            decode()
        if events is not None:
            events[2].record(stream)

    # Clock spin-up (untimed): a few ms of work leaves the memory/GPU clocks
    # ramping and under-reports the first ~10 ms; spin for `--spinup` s first.
    t_spin = time.perf_counter()
    while time.perf_counter() - t_spin < args.spinup:
        step()
        torch.cuda.synchronize(dev)
    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize(dev)

    evs = [[torch.cuda.Event(enable_timing=True) for _ in range(3)] for _ in range(args.steps)]
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for i in range(args.steps):
        step(evs[i])
    torch.cuda.synchronize(dev)
    t1 = time.perf_counter()
    if world > 1:
        dist.barrier()
    elapsed = max_over_ranks(t1 - t0, dev)
    log(f"timed {args.steps} steps: {elapsed / args.steps * 1e3:.3f} ms/step")

    # correctness gate (after the timed region): decode reconstructs the
    # erased shards of every stripe (on the device), and every stripe's parity
    # and rebuilt cells match the C oracle bit for bit (stripe-parallel on the
    # host's CPU share; --verify sample: stripe 0 only)
    if not args.encode_only and not mixed:
        assert torch.equal(rec, data[:, :m]), "decode != original"
    if not args.encode_only and mixed:
        lost = torch.tensor([[not (mk >> i) & 1 for i in range(k)] for mk in masks], device=dev)
        assert bool(((rec == data) | ~lost[:, :, None]).all()), "mixed decode != original"
    import ec_oracle
    clib = ec_oracle.load_c_oracle()
    verified = verify_batch(args, ec_oracle, clib, data, parity, None if (args.encode_only or mixed) else rec, k, m)
    log(f"verified: {verified}")


    enc_ms = [evs[i][0].elapsed_time(evs[i][1]) for i in range(args.steps)]
    dec_ms = [evs[i][1].elapsed_time(evs[i][2]) for i in range(args.steps)] if not args.encode_only else []
    launch_ms = enc_ms + dec_ms
    avg_launch_ms = sum(launch_ms) / len(launch_ms)
    ops = 1 if args.encode_only else 2
    bytes_per_step = sum_over_ranks(float(ops * k * cell * S), dev)
    value = bytes_per_step * args.steps / elapsed / GIB
    algo_bytes = (k + m) * cell * S  # per launch: k inputs read + m outputs written
    achieved = algo_bytes / (avg_launch_ms * 1e-3) / 1e9
    if mixed:  # decode launches move (k + e_s) cells per stripe
        dec_bytes = (k * S + erased) * cell
        enc_avg = sum(enc_ms) / len(enc_ms) * 1e-3
        dec_avg = sum(dec_ms) / len(dec_ms) * 1e-3 if dec_ms else enc_avg
        achieved = (algo_bytes + dec_bytes) / (enc_avg + dec_avg) / 1e9

    traffic, traffic_src = traffic_for(args.traffic, k, m, cell, S, args.decode_mode) if not args.tune else (None, None)
    # every rank's own launch average and stripe range (rank order): an N-rank
    # line shows each GPU's kernel time, not only rank 0's and the max
    launch_per_rank = [round(x, 4) for x in gather_list(avg_launch_ms, world, dist)]
    shards = gather_list([first, S], world, dist)

    result = {
        "metric": METRIC,
        "value": round(value, 2),
        "unit": "GiB/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(elapsed / args.steps * 1e3, 4),
        "higher_is_better": True,
        "scaling": scaling,
        "vs_baseline": None,
        "dtype": "u8",
        "data": "synthetic: seeded uniform random bytes (torch.randint on device, seed 0x5EED_EC00 + first stripe)",
        "config": {
            "workload": f"RS({k},{m}) {cell >> 10} KiB cells: encode + decode with "
                        + ("data shards " if not mixed else "")
                        + (f"{{{','.join(map(str, miss))}}} missing, " if not mixed else
                           f"a random 1..{m} data shards missing per stripe, ")
                        + (f"{args.global_stripes} stripes split over {world} GPU(s)" if args.global_stripes
                           else f"{S} stripes per GPU")
                        + (" (encode only)" if args.encode_only else ""),
            "k": k, "m": m, "cell_bytes": cell, "stripes_per_gpu": S,
            "global_stripes": args.global_stripes or S * world,
            "shards": shards,
            "parallelism": f"stripe-sharded x{world}, no collectives",
            "decode_mode": args.decode_mode,
            "codec": args.codec,
        },
        "roofline": {
            "bound": "hbm",
            "achieved": round(achieved, 1),
            "peak": HBM_PEAK_GBS,
            "unit": "GB/s",
            "frac": round(achieved / HBM_PEAK_GBS, 4),
            "traffic": traffic,
            "traffic_source": traffic_src,
            "kernel": (f"gf_matmul_v16<{k},{m}> (encode and decode launches; work queue of wave-tiles)"
                       if k in (2, 3, 6, 10) else f"gf_matmul_v16<{k},{m}> (encode and decode launches)"),
            "algorithmic_bytes_per_launch": algo_bytes,
            "avg_launch_ms": round(avg_launch_ms, 4),
            "avg_launch_ms_per_rank": launch_per_rank,
            "frac_of_measured_copy": round(achieved / HBM_COPY_GBS, 4),
        },
        "encode_GiBps": round(k * cell * S / (sum(enc_ms) / len(enc_ms) * 1e-3) / GIB, 2),
        "decode_GiBps": round(k * cell * S / (sum(dec_ms) / len(dec_ms) * 1e-3) / GIB, 2) if dec_ms else None,
        "parity_check": verified,
    }
    if mixed and dec_ms:
        # the mixed-pattern decode kernel alone: k survivors read + e_s rebuilt
        # cells written per stripe, over its own launch average
        result["roofline"]["kernel"] = (f"gf_matmul_v16<{k},{m}> encode + gf_decode_mixed<{k},{min(m, 4)}> "
                                        f"(achieved / frac over both launch kinds)")
        dec_avg_ms = sum(dec_ms) / len(dec_ms)
        result["roofline"]["decode_mixed"] = {
            "algorithmic_bytes_per_launch": dec_bytes, "avg_launch_ms": round(dec_avg_ms, 4),
            "achieved": round(dec_bytes / (dec_avg_ms * 1e-3) / 1e9, 1),
            "frac": round(dec_bytes / (dec_avg_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
            "erased_cells": int(erased)}

    if args.crc:
        result["crc32c"] = crc_leg(args, H, coder, data, parity, rec, dp, ds, pp, ps, rp, rs, shard_ptrs, miss,
                                   decode, dev, stream, mixed)

    host_path = args.host_path if args.host_path >= 0 else int(world == 1)
    if host_path and rank == 0 and not mixed:
        result["host_path"] = pinned_leg(coder, data, parity, k, m, cell, S, torch)
        result["host_path"]["per_call"] = per_call_leg(H, k, m, cell, 64, clib)
        log("host path legs")
        result["host_path"]["per_call_by_size"] = per_call_sizes(H, k, m, clib)
        log("per-call table")
        result["host_path"]["rows_call"] = rows_call_leg(H, k, m, cell, coder, torch)
        log("writer / reader call shapes")

    if rank == 0 and world == 1 and args.cpu_seconds > 0:
        log("cpu baseline")
        result["cpu_baseline"] = cpu_baseline(k, m, cell, args.cpu_seconds, 1)
        if args.cpu_threads > 1:
            result["cpu_baseline_parallel"] = cpu_baseline(k, m, cell, args.cpu_seconds, args.cpu_threads)
        if (k, m, cell) == (6, 3, 1 << 20) and args.codec == "rs" and not args.tune:
            log("cpu config RS(3,2) x 1024")
            result["cpu_baseline_configs"] = [cpu_config_batch(H, 3, 2, 1 << 20, 1024, args.cpu_threads)]
            # the two other BASELINE configs with a device line in extra_configs
            # (BASELINE.md:47-48): bounded stripe samples, ~2-5 s per 1-thread leg
            log("cpu config RS(10,4) 1 MiB sample")
            result["cpu_baseline_configs"].append(cpu_config_batch(
                H, 10, 4, 1 << 20, 128, args.cpu_threads, config_stripes=2048, source="BASELINE.json configs[3]"))
            log("cpu config RS(6,3) 64 KiB sample")
            result["cpu_baseline_configs"].append(cpu_config_batch(
                H, 6, 3, 1 << 16, 4096, args.cpu_threads, config_stripes=65536, source="BASELINE.json configs[4]"))
    elif rank == 0:
        result["cpu_baseline"] = None

    extra = args.extra_configs if args.extra_configs >= 0 else int(
        (k, m, cell, args.codec, args.decode_mode) == (6, 3, 1 << 20, "rs", "uniform") and not args.global_stripes
        and not args.encode_only and not args.tune)
    if extra:
        del data, parity, rec
        torch.cuda.empty_cache()
        result["extra_configs"] = extra_configs(args, H, dist, world, rank, dev, max_over_ranks, shard_range)

    result["process_group"] = process_group_info(args, world, dist)
    result["ranks"] = gather_ranks(rank_identity(rank, local, dev.index, shared), world, dist)
    result["distinct_gpus"] = len({(r["pci_domain_id"], r["pci_bus_id"], r["pci_device_id"], r["uuid"])
                                   for r in result["ranks"]})
    if rank == 0:
        print(json.dumps(result), flush=True)
    coder.close()
    if world > 1:
        dist.destroy_process_group()


def verify_batch(args, ec_oracle, clib, data, parity, rec, k, m):
    """Every stripe against the oracle (test infrastructure, the checker):
    parity, and with rec ([S, m, cell] = data shards 0..m-1 rebuilt) the
    oracle's decode of the same survivors; <= 2 GiB of data per host slice.
    xor / rs-legacy (and --verify sample): stripe 0 against the Python oracle."""
    import numpy as np
    S, _, cell = data.shape
    if args.codec != "rs" or args.verify == "sample":
        s0 = data[0].cpu().numpy()
        want = (ec_oracle.c_encode(clib, k, m, list(s0)) if args.codec == "rs" else
                ec_oracle.legacy_encode(k, m, list(s0)) if args.codec == "rs-legacy" else
                ec_oracle.matmul_shards(ec_oracle.select_rows(ec_oracle.codec_matrix(args.codec, k, m),
                                                              range(k, k + m)), list(s0)))
        assert all(np.array_equal(parity[0, j].cpu().numpy(), want[j]) for j in range(m)), "parity != oracle"
        return "ok: stripe 0 vs oracle"
    threads = max(1, min(16, int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or (os.cpu_count() or 8)))
    present = ((1 << (k + m)) - 1) & ~((1 << m) - 1)
    step = max(1, (1 << 31) // (k * cell))
    t0 = time.perf_counter()
    for a in range(0, S, step):
        b = min(S, a + step)
        ec_oracle.c_check_batch(clib, k, m, data[a:b].cpu().numpy(), parity[a:b].cpu().numpy(),
                                present if rec is not None else None,
                                rec[a:b].cpu().numpy() if rec is not None else None, threads=threads)
    return (f"ok: all {S} stripes' parity" + (f" and rebuilt shards 0..{m - 1}" if rec is not None else "") +
            f" == C oracle ({threads} threads, {time.perf_counter() - t0:.1f} s)")


EXTRA_CONFIGS = [  # split over the ranks: the headline's strong-scaling twin (1024 stripes in all, not per
    # GPU) and the other multi-GPU BASELINE configs (BASELINE.json configs[3], [4])
    {"name": "rs63_1MiB_x1024_strong", "k": 6, "m": 3, "cell": 1 << 20, "global_stripes": 1024},
    {"name": "rs104_1MiB_x2048", "k": 10, "m": 4, "cell": 1 << 20, "global_stripes": 2048},
    {"name": "rs63_64KiB_x65536", "k": 6, "m": 3, "cell": 1 << 16, "global_stripes": 65536},
]


def extra_configs(args, H, dist, world, rank, dev, max_over_ranks, shard_range):
    """The headline's strong-scaling twin (RS(6,3) 1 MiB x 1024 stripes IN
    ALL), RS(10,4) 1 MiB x 2048 and RS(6,3) 64 KiB x 65536, each split into
    contiguous per-rank shares (strong scaling, no collective): encode +
    worst-case decode per step, allocation and warmup outside the timed
    loop, barrier + max-over-ranks time, every rank's batch checked against
    its own device copy after timing."""
    import torch
    out = {}
    steps = max(3, min(args.steps, 10))
    stream = torch.cuda.current_stream(dev)
    sp = stream.cuda_stream
    for cfg in EXTRA_CONFIGS:
        k, m, cell = cfg["k"], cfg["m"], cfg["cell"]
        first, S = shard_range(cfg["global_stripes"], world, rank)
        coder = H.Coder(k, m, dev.index)
        g = torch.Generator(device=dev)
        g.manual_seed(0x5EED_EC00 + first)
        data = torch.randint(0, 256, (S, k, cell), dtype=torch.uint8, device=dev, generator=g)
        parity = torch.empty((S, m, cell), dtype=torch.uint8, device=dev)
        rec = torch.empty((S, m, cell), dtype=torch.uint8, device=dev)
        dp, ds = H.stripe_layout_ptrs(data, k)
        pp, ps = H.stripe_layout_ptrs(parity, m)
        rp, rs = H.stripe_layout_ptrs(rec, m)
        shard_ptrs = [None] * m + dp[m:] + pp
        out_ptrs = rp + [0] * (k - m)

        def step(ev=None):
            if ev:
                ev[0].record(stream)
            coder.encode_device(dp, ds, pp, ps, cell, S, sp)
            if ev:
                ev[1].record(stream)
            coder.decode_device(shard_ptrs, ds + ps, out_ptrs, [rs[0]] * k, cell, S, sp)
            if ev:
                ev[2].record(stream)

        for _ in range(3):
            step()
        torch.cuda.synchronize(dev)
        evs = [[torch.cuda.Event(enable_timing=True) for _ in range(3)] for _ in range(steps)]
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        for i in range(steps):
            step(evs[i])
        torch.cuda.synchronize(dev)
        t1 = time.perf_counter()
        if world > 1:
            dist.barrier()
        elapsed = max_over_ranks(t1 - t0, dev)
        log(f"extra config {cfg['name']}: {elapsed / steps * 1e3:.3f} ms/step")
        assert torch.equal(rec, data[:, :m]), f"{cfg['name']}: decode != original"
        launch = [evs[i][0].elapsed_time(evs[i][1]) for i in range(steps)] + \
                 [evs[i][1].elapsed_time(evs[i][2]) for i in range(steps)]
        avg_ms = sum(launch) / len(launch)
        avg_max = max_over_ranks(avg_ms, dev)
        per_rank = [round(x, 4) for x in gather_list(avg_ms, world, dist)]
        shards = gather_list([first, S], world, dist)
        algo = (k + m) * cell * S
        total = cfg["global_stripes"]
        out[cfg["name"]] = {
            "workload": f"RS({k},{m}) {cell >> 10} KiB cells, {total} stripes split over {world} GPU(s): encode + "
                        f"decode with data shards {{0..{m - 1}}} missing",
            "scaling": "strong", "stripes_per_gpu_rank0": S, "steps": steps,
            "value_GiBps": round(2 * k * cell * total * steps / elapsed / GIB, 2),
            "ms_per_step": round(elapsed / steps * 1e3, 4),
            "avg_launch_ms_rank0": round(avg_ms, 4), "avg_launch_ms_max_over_ranks": round(avg_max, 4),
            "avg_launch_ms_per_rank": per_rank, "shards": shards,
            "frac_rank0": round(algo / (avg_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
            "algorithmic_bytes_per_launch_rank0": algo,
            "check": "rebuilt == original on every rank (device)",
        }
        coder.close()
        del data, parity, rec
        torch.cuda.empty_cache()
    return out


def pinned_leg(coder, data, parity, k, m, cell, S, torch):
    """The path starts and ends in host memory (DataNode sockets in, write
    pipeline out): pinned host buffers through the coder's 3-slot
    H2D / kernel / D2H pipelines.  Never `value`."""
    hs = min(S, 256)
    h_in = data[:hs].cpu().pin_memory()
    h_out = torch.empty((hs, m, cell), dtype=torch.uint8).pin_memory()
    coder.encode_host_batch(h_in.data_ptr(), h_out.data_ptr(), cell, hs, 16)
    reps = 3
    th0 = time.perf_counter()
    for _ in range(reps):
        coder.encode_host_batch(h_in.data_ptr(), h_out.data_ptr(), cell, hs, 16)
    th = (time.perf_counter() - th0) / reps
    assert torch.equal(h_out, parity[:hs].cpu())
    # read side: the reader's per-shard vertical buffers (data shards
    # 0..m-1 lost) -> file-order rows with the lost cells rebuilt
    vert = [None if i < m else h_in[:, i].contiguous().pin_memory() for i in range(k)] + \
           [h_out[:, j].contiguous().pin_memory() for j in range(m)]
    h_file = torch.empty((hs, k, cell), dtype=torch.uint8).pin_memory()
    vaddr = [None if v is None else v.data_ptr() for v in vert]
    coder.decode_host_batch(vaddr, cell, hs, h_file.data_ptr(), 16)
    td0 = time.perf_counter()
    for _ in range(reps):
        coder.decode_host_batch(vaddr, cell, hs, h_file.data_ptr(), 16)
    td = (time.perf_counter() - td0) / reps
    assert torch.equal(h_file, h_in)
    return {"encode_GiBps_pcie_inclusive": round(k * cell * hs / th / GIB, 2),
            "decode_GiBps_pcie_inclusive": round(k * cell * hs / td / GIB, 2),
            "stripes": hs, "chunk_stripes": 16,
            "note": "pinned host -> H2D -> kernel -> D2H -> pinned host, 3-slot pipelines "
                    "(hec_encode_host_batch; hec_decode_host_batch with data shards "
                    f"0..{m - 1} lost, file-order rows out); data GiB/s, never `value`"}


def crc_leg(args, H, coder, data, parity, rec, dp, ds, pp, ps, rp, rs, shard_ptrs, miss, decode, dev, stream, mixed):
    import torch

    import ec_oracle
    k, m, cell = args.k, args.m, args.cell
    S = data.shape[0]
    sp = stream.cuda_stream
    bpc = 512
    nch = (cell + bpc - 1) // bpc
    sums = torch.empty((S, k + m, nch, 4), dtype=torch.uint8, device=dev)
    cells_ptrs, cells_strides = dp + pp, ds + ps

    def enc_crc():
        coder.encode_crc_device(dp, ds, pp, ps, cell, S, bpc, sums.data_ptr(), sp)

    def crc_only():
        coder.crc32c_device(cells_ptrs, cells_strides, cell, S, bpc, sums.data_ptr(), sp)

    def enc_crc_unfused():  # the two passes a non-fused engine runs
        coder.encode_device(dp, ds, pp, ps, cell, S, sp)
        crc_only()

    for fn in (enc_crc, crc_only, enc_crc_unfused):
        fn()
    torch.cuda.synchronize(dev)
    reps = max(3, args.steps // 2)
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(4)]
    ev[0].record(stream)
    for _ in range(reps):
        crc_only()
    ev[1].record(stream)
    for _ in range(reps):
        enc_crc_unfused()
    ev[2].record(stream)
    for _ in range(reps):
        enc_crc()  # last: the spot-check below reads the fused kernel's sums
    ev[3].record(stream)
    torch.cuda.synchronize(dev)
    t_c = ev[0].elapsed_time(ev[1]) / reps * 1e-3
    t_u = ev[1].elapsed_time(ev[2]) / reps * 1e-3
    t_ec = ev[2].elapsed_time(ev[3]) / reps * 1e-3
    # spot-check one stripe's sums against the oracle
    s0_cells = torch.cat([data[0], parity[0]]).cpu().numpy()
    want = b"".join(ec_oracle.chunk_crc32c(s0_cells[i].tobytes(), bpc) for i in range(k + m))
    assert sums[0].cpu().numpy().tobytes() == want, "crc32c != oracle"
    # algorithmic bytes per launch, the 4-B chunk sums included
    # (scripts/profile_configs.py crc_leg_bytes): k+m cells + their sums
    enc_crc_bytes = ((k + m) * cell + 4 * nch * (k + m)) * S
    res = {
        "bytes_per_checksum": bpc,
        "encode_crc_GiBps": round(k * cell * S / t_ec / GIB, 2),
        "encode_crc_ms": round(t_ec * 1e3, 3),
        "encode_crc_hbm_TBps": round(enc_crc_bytes / t_ec / 1e12, 3),
        "encode_crc_frac": round(enc_crc_bytes / t_ec / 1e9 / HBM_PEAK_GBS, 4),
        "encode_crc_algorithmic_bytes": enc_crc_bytes,
        "encode_then_crc_GiBps": round(k * cell * S / t_u / GIB, 2),
        "encode_then_crc_ms": round(t_u * 1e3, 3),
        "crc_only_GBps": round(enc_crc_bytes / t_c / 1e9, 1),
        "crc_only_ms": round(t_c * 1e3, 3),
        "crc_only_frac": round(enc_crc_bytes / t_c / 1e9 / HBM_PEAK_GBS, 4),
        "note": "CRC32C of all k+m cells per 512-B chunk (WritePacket::calculate_checksum), big-endian",
    }
    if args.encode_only or mixed:
        return res
    # read side: survivors' chunk sums verified while the missing data cells
    # are rebuilt (hec_decode_verify_device: fused kernel, then a host look at
    # the flags); vs. verify pass + decode pass; then with corrupt survivors
    bad = torch.empty((S, k + m), dtype=torch.uint8, device=dev)
    surv = [i for i in range(k + m) if shard_ptrs[i] is not None][:k]
    sv_ptrs = [(dp + pp)[i] for i in surv]
    sv_strides = [(ds + ps)[i] for i in surv]
    sv_sums = sums[:, surv].contiguous()
    # present data shards are repaired in place if they fail
    vo_ptrs = [rp[i] if i in miss else dp[i] for i in range(k)]
    vo_strides = [rs[0] if i in miss else ds[i] for i in range(k)]

    def dec_verify():
        coder.decode_verify_device(H.CHECKSUM_CRC32C, shard_ptrs, ds + ps, vo_ptrs, vo_strides, cell, S, bpc,
                                   sums.data_ptr(), bad.data_ptr(), sp)

    def verify_then_decode():
        bad.zero_()
        coder.checksum_verify_device(H.CHECKSUM_CRC32C, sv_ptrs, sv_strides, cell, S, bpc, sv_sums.data_ptr(),
                                     bad.data_ptr(), sp)
        decode()
        torch.cuda.synchronize(dev)

    # the plan-specialised fused kernel (jit.hpp: the decode plan's bit-sliced
    # XOR network compiled with hiprtc), prepared before anything is timed --
    # as a DataNode's reconstruct worker prepares its plans; HEC_JIT=0 runs the
    # ahead-of-time v_perm kernel instead (A/B)
    t_0 = time.perf_counter()
    lost = [i for i in range(k + m) if shard_ptrs[i] is None]
    jit_ready = coder.prepare_decode(lost, H.CHECKSUM_CRC32C)
    jit_ready_c = coder.prepare_decode([0], H.CHECKSUM_CRC32C)  # the corrupt-survivor leg's plan
    t_prep = time.perf_counter() - t_0
    for fn in (dec_verify, verify_then_decode):
        fn()
    torch.cuda.synchronize(dev)
    reps = max(3, args.steps // 2)
    tv = {}
    for name, fn in (("unfused", verify_then_decode), ("fused", dec_verify)):
        t_0 = time.perf_counter()
        for _ in range(reps):
            fn()
        torch.cuda.synchronize(dev)
        tv[name] = (time.perf_counter() - t_0) / reps
    assert not bad.any() and torch.equal(rec, data[:, :m]), "decode+verify mismatch"
    e_ = len(miss)
    res.update({
        "decode_verify_GiBps": round(k * cell * S / tv["fused"] / GIB, 2),
        "decode_verify_ms": round(tv["fused"] * 1e3, 3),
        "decode_verify_hbm_TBps": round(((k + e_) * cell + 4 * nch * k) * S / tv["fused"] / 1e12, 3),
        "decode_verify_frac": round(((k + e_) * cell + 4 * nch * k) * S / tv["fused"] / 1e9 / HBM_PEAK_GBS, 4),
        "verify_then_decode_GiBps": round(k * cell * S / tv["unfused"] / GIB, 2),
        "verify_then_decode_ms": round(tv["unfused"] * 1e3, 3),
        "read_note": "CRC32C of the k survivors verified against their packet sums while data shards "
                     f"{{{','.join(map(str, miss))}}} are rebuilt (ReadPacket::get_data + ec_decode); "
                     "wall time of the synchronous call incl. the flag read-back",
        "decode_verify_kernel": ("plan-specialised (bit-sliced network of the decode plan, hiprtc)" if jit_ready
                                 else "ahead-of-time (v_perm product tables)"),
        "jit": dict(H.jit_stats(), prepare_s=round(t_prep, 2), ready=bool(jit_ready),
                    ready_corrupt_leg=bool(jit_ready_c)),
    })
    # corrupt survivors: data shard 0 unavailable (one spare shard beyond k),
    # and a fraction of the stripes gets one flipped byte in its first
    # survivor (data shard 1).  The call re-plans those stripes (phase 2):
    # shard 1 is dropped, the next parity shard read and verified, shards 0
    # and 1 rebuilt -- shard 1 in place over its corrupt cell.
    corrupt = {}
    c_ptrs = [None] + [dp[i] for i in range(1, k)] + pp
    c_out = [rp[0]] + [dp[i] for i in range(1, k)]
    c_ost = [rs[0]] + [ds[i] for i in range(1, k)]

    def dec_verify_c():
        coder.decode_verify_device(H.CHECKSUM_CRC32C, c_ptrs, ds + ps, c_out, c_ost, cell, S, bpc, sums.data_ptr(),
                                   bad.data_ptr(), sp)

    dec_verify_c()
    torch.cuda.synchronize(dev)
    t_0 = time.perf_counter()
    for _ in range(reps):
        dec_verify_c()
    torch.cuda.synchronize(dev)
    corrupt["0"] = {"stripes_corrupt": 0, "ms": round((time.perf_counter() - t_0) / reps * 1e3, 3)}
    corrupt["0"]["GiBps"] = round(k * cell * S / (corrupt["0"]["ms"] * 1e-3) / GIB, 2)
    for frac in [float(x) for x in args.corrupt.split(",") if x and x.lower() != "none"]:
        n_bad = max(1, int(round(frac * S)))
        idx = torch.linspace(0, S - 1, n_bad, device=dev).long().unique()
        orig = data[idx, 1, 7].clone()
        ts = []
        for _ in range(3):
            data[idx, 1, 7] ^= 0x5A
            torch.cuda.synchronize(dev)
            t_0 = time.perf_counter()
            dec_verify_c()
            torch.cuda.synchronize(dev)
            ts.append(time.perf_counter() - t_0)
            assert torch.equal(data[idx, 1, 7], orig), "in-place repair failed"
            assert torch.equal(bad[:, 1].nonzero().flatten(), idx), "wrong cells flagged"
        assert torch.equal(rec[:, 0], data[:, 0]), "decode+verify with corrupt survivors mismatch"
        t = min(ts)
        corrupt[f"{frac:g}"] = {"stripes_corrupt": int(idx.numel()), "ms": round(t * 1e3, 3),
                                "GiBps": round(k * cell * S / t / GIB, 2)}
    res["decode_verify_corrupt"] = corrupt
    res["corrupt_note"] = ("data shard 0 unavailable, a fraction of stripes with a corrupt data shard 1 "
                           "(re-planned, repaired in place); key = fraction of stripes")
    dec_verify()  # leave clean flags behind
    torch.cuda.synchronize(dev)
    return res


if __name__ == "__main__":
    main()
