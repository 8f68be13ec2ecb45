"""Multi-rank path: world_size-2 gloo process groups exercising the stripe
sharding and max-over-ranks timing used by bench.py (the data path itself
has no collective; each rank codes its own stripe range).  On the CPU every
rank codes its share with the ENGINE's host routine (hec_gf_matmul_host);
the GPU variant runs the device engine on both ranks (one card, two
processes); both are checked against the oracle."""
import hashlib
import json
import os
import socket
import sys

import numpy as np
import pytest

from hdfs_native_ec.dist import shard_range

torch = pytest.importorskip("torch")
import torch.distributed as dist  # noqa: E402
import torch.multiprocessing as mp  # noqa: E402


@pytest.mark.parametrize("total", [0, 1, 7, 8, 1024, 2049])
@pytest.mark.parametrize("world", [1, 2, 3, 8])
def test_shard_range_tiles_batch(total, world):
    ranges = [shard_range(total, world, r) for r in range(world)]
    pos = 0
    for start, count in ranges:
        assert start == pos
        pos += count
    assert pos == total
    counts = [c for _, c in ranges]
    assert max(counts) - min(counts) <= 1


def test_shard_range_rejects_bad_rank():
    with pytest.raises(ValueError):
        shard_range(10, 2, 2)


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, total, k, m, cell, out_path, root, device=False):
    sys.path[:0] = [os.path.join(root, "hdfs-native_amd"), os.path.join(root, "oracle")]
    import hdfs_native_ec as H
    from hdfs_native_ec.dist import max_over_ranks, shard_range, sum_over_ranks
    from hdfs_native_ec.synth import batch_data
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    try:
        first, count = shard_range(total, world, rank)
        data = batch_data(count, k, cell, first=first)
        digests = []
        if device:  # the device engine on this rank's share (ranks share card 0)
            coder = H.Coder(k, m, 0)
            d = torch.from_numpy(data).to("cuda:0")
            p = torch.empty((count, m, cell), dtype=torch.uint8, device="cuda:0")
            if count:
                H.encode_batch(coder, d, p)
            torch.cuda.synchronize()
            pars = [list(p[s].cpu().numpy()) for s in range(count)]
            coder.close()
        else:  # the engine's host routine, no device
            enc = H.gen_rs_matrix(k, m)[k:]
            pars = [[np.frombuffer(x, dtype=np.uint8) for x in H.gf_matmul_host(enc, list(data[s]))]
                    for s in range(count)]
        for par in pars:
            digests.append(hashlib.sha256(b"".join(p.tobytes() for p in par)).hexdigest())
        gathered = [None] * world
        dist.all_gather_object(gathered, (first, digests))
        tmax = max_over_ranks(float(rank + 1))
        nbytes = sum_over_ranks(float(count * k * cell))
        dist.barrier()
        if rank == 0:
            with open(out_path, "w") as f:
                json.dump({"gathered": gathered, "tmax": tmax, "bytes": nbytes}, f)
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2])
@pytest.mark.parametrize("device", [False, pytest.param(True, marks=pytest.mark.gpu)])
def test_gloo_sharded_encode_matches_single_process(tmp_path, world, device):
    import ec_oracle as O
    from hdfs_native_ec.synth import batch_data
    from conftest import ROOT
    total, k, m, cell = 7, 6, 3, 4096
    out = tmp_path / "res.json"
    mp.spawn(_worker, args=(world, _free_port(), total, k, m, cell, str(out), ROOT, device), nprocs=world, join=True)
    res = json.loads(out.read_text())
    assert res["tmax"] == float(world)
    assert res["bytes"] == float(total * k * cell)
    lib = O.load_c_oracle()
    data = batch_data(total, k, cell)
    want = [hashlib.sha256(b"".join(p.tobytes() for p in O.c_encode(lib, k, m, list(data[s])))).hexdigest()
            for s in range(total)]
    got = []
    for first, digests in sorted(res["gathered"], key=lambda t: t[0]):
        assert first == len(got)
        got.extend(digests)
    assert got == want


@pytest.mark.parametrize("args,want_S,want_global,scaling", [
    (["--k", "10", "--m", "4", "--global-stripes", "2048"], 1024, 2048, "strong"),
    (["--stripes", "1024"], 1024, 2048, "weak"),
    (["--global-stripes", "7"], 4, 7, "strong"),
])
def test_bench_gpus_flag_spawns_ranks(args, want_S, want_global, scaling):
    """`bench.py --gpus 2` run directly (no launcher WORLD_SIZE) starts two
    ranks itself through torch.distributed.run, which rendezvous over
    loopback, reduce, and print ONE JSON line with n_gpus = 2 (dry run: gloo,
    no GPU, no engine -- the launcher/rank/reduction plumbing only)."""
    import subprocess
    from conftest import ROOT
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--backend", "gloo",
                          "--dry-run"] + args, capture_output=True, text=True, timeout=240, env=env, cwd=ROOT)
    assert out.returncode == 0, out.stderr[-3000:]
    lines = [ln for ln in out.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, out.stdout
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["dry_run"] and d["scaling"] == scaling
    assert d["config"]["global_stripes"] == want_global
    assert d["config"]["stripes_summed_over_ranks"] == want_global
    assert d["config"]["stripes_per_gpu"] == want_S  # rank 0's share
    # the other multi-GPU BASELINE configs are timed by the same invocation,
    # each split over the ranks (bench.py --extra-configs)
    ex = d["extra_configs"]
    assert set(ex) == {"rs63_1MiB_x1024_strong", "rs104_1MiB_x2048", "rs63_64KiB_x65536"}
    assert ex["rs63_1MiB_x1024_strong"]["stripes_per_gpu_rank0"] == 512
    assert ex["rs104_1MiB_x2048"]["stripes_per_gpu_rank0"] == 1024
    assert ex["rs104_1MiB_x2048"]["stripes_summed_over_ranks"] == 2048
    assert ex["rs63_64KiB_x65536"]["stripes_per_gpu_rank0"] == 32768
    assert ex["rs63_64KiB_x65536"]["stripes_summed_over_ranks"] == 65536
    assert all(v["scaling"] == "strong" and v["value_GiBps"] is None for v in ex.values())
    # every rank reports its identity (device ordinal / PCI location / UUID on
    # a GPU run; None here), gathered over the process group in rank order
    assert d["process_group"]["world_size"] == 2 and d["process_group"]["backend"] == "gloo"
    assert [r["rank"] for r in d["ranks"]] == [0, 1]
    assert [r["local_rank"] for r in d["ranks"]] == [0, 1]
    assert all(set(r) >= {"device", "pci_bus_id", "pci_domain_id", "uuid", "host", "shared_gpu"} for r in d["ranks"])


def test_bench_refuses_more_nccl_ranks_than_gpus():
    """One rank per GPU: an nccl world whose LOCAL_RANK has no GPU of its own
    (here: no GPU at all) exits non-zero before anything is timed, instead of
    folding ranks onto shared cards."""
    import subprocess
    from conftest import ROOT
    if torch.cuda.device_count() >= 2:
        pytest.skip("needs fewer GPUs than ranks")
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--backend", "nccl",
                          "--steps", "1", "--warmup", "0", "--cpu-seconds", "0", "--host-path", "0"],
                         capture_output=True, text=True, timeout=240, env=env, cwd=ROOT)
    assert out.returncode != 0
    assert "refusing" in out.stderr and "one rank per GPU" in out.stderr
    assert not [ln for ln in out.stdout.splitlines() if ln.startswith("{")]


def test_bench_dry_run_world_8():
    """The 8-GPU line's plumbing at world 8 (gloo, no GPU): `bench.py --gpus 8
    --dry-run` starts 8 ranks that rendezvous over loopback and print ONE
    line whose shard tables tile every batch in rank order -- the weak
    headline (1024 stripes per rank), its strong twin (1024 in all, 128 per
    rank) and the two other BASELINE configs -- and whose `ranks` list holds
    all 8 ranks."""
    import subprocess
    from conftest import ROOT
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env["OMP_NUM_THREADS"] = "1"
    out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "8", "--backend", "gloo",
                          "--dry-run"], capture_output=True, text=True, timeout=400, env=env, cwd=ROOT)
    assert out.returncode == 0, out.stderr[-3000:]
    lines = [ln for ln in out.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, out.stdout
    d = json.loads(lines[0])
    assert d["n_gpus"] == 8 and d["scaling"] == "weak"
    assert d["config"]["shards"] == [[1024 * r, 1024] for r in range(8)]
    assert d["config"]["global_stripes"] == 8192
    want = {"rs63_1MiB_x1024_strong": 1024, "rs104_1MiB_x2048": 2048, "rs63_64KiB_x65536": 65536}
    assert set(d["extra_configs"]) == set(want)
    for name, total in want.items():
        assert d["extra_configs"][name]["shards"] == [[r * total // 8, total // 8] for r in range(8)], name
        assert d["extra_configs"][name]["stripes_summed_over_ranks"] == total
    assert [r["rank"] for r in d["ranks"]] == list(range(8))
    assert [r["local_rank"] for r in d["ranks"]] == list(range(8))
    assert d["process_group"]["world_size"] == 8
