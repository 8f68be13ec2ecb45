"""The C++ host mirror (hdfs-native_amd/csrc/hdfs_ec.hpp) of the reference's
EcSchema / resolve_ec_policy / CellBuffer / Coder callers, driven by
tests/cpp/test_host_mirror.cpp."""
import json
import os
import subprocess

import pytest

import ec_oracle as O
from conftest import PKG_DIR

BIN = os.path.join(PKG_DIR, "build", "test_host_mirror")


SRCS = [os.path.join(PKG_DIR, "..", "tests", "cpp", "test_host_mirror.cpp"),
        os.path.join(PKG_DIR, "csrc", "hdfs_ec.hpp"), os.path.join(PKG_DIR, "..", "include", "hdfs_ec_amd.h")]


@pytest.fixture(scope="module")
def binary():
    # Rebuilt only when missing or older than its own sources.  It links the
    # engine dynamically, so a rebuilt .so needs no relink; and the compile is
    # a direct g++ line, not `make`, whose rule would also walk the engine's
    # object files -- they do not travel to the GPU box, so make would
    # rebuild the whole engine there.
    if not os.path.exists(BIN) or os.path.getmtime(BIN) < max(os.path.getmtime(p) for p in SRCS):
        os.makedirs(os.path.dirname(BIN), exist_ok=True)
        subprocess.check_call(["g++", "-O2", "-std=c++17", "-Wall", "-Wextra", "-pthread", "-o", BIN, SRCS[0],
                               "-L" + os.path.join(PKG_DIR, "lib"), "-lhdfs_ec_amd", "-Wl,-rpath,$ORIGIN/../lib"])
    return BIN


def test_cpu_side_matches_oracle(binary):
    out = subprocess.run([binary, "cpu"], capture_output=True, text=True, check=True, timeout=60).stdout
    rows = [json.loads(l) for l in out.splitlines() if l.startswith("{")]
    pol = {r["policy"]: r for r in rows if "policy" in r}
    for pid, (codec, k, m, cell) in O.POLICIES.items():  # mod.rs:93-144
        assert (pol[pid]["codec"], pol[pid]["k"], pol[pid]["m"], pol[pid]["cell"]) == (codec, k, m, cell)
    assert "error" in pol[6]
    assert (pol[99]["codec"], pol[99]["k"], pol[99]["m"], pol[99]["cell"]) == ("rs", 4, 2, 65536)
    grid = [r["max_offset"] for r in rows if "max_offset" in r]
    assert len(grid) > 100
    for index, bs, got in grid:
        assert got == O.max_offset(3, 16, index, bs), (index, bs)
    row6 = next(r["rs63_row6"] for r in rows if "rs63_row6" in r)
    assert row6 == O.gen_rs_matrix(6, 3)[6]
    # ec_decode's split (mod.rs:82-86): 2 rows of 3 cells; a short shard is
    # split_to's panic (out_of_range), never a clamped cell
    split = next(r["split_cells"] for r in rows if "split_cells" in r)
    assert split == [6, 2, 1]
    assert next(r["split_short"] for r in rows if "split_short" in r) == "out_of_range"
    with pytest.raises(ValueError):
        O.ec_decode(3, 2, 16, "rs", [b"\1" * 32, b"\2" * 32, b"\3" * 20, None, None])


def _counter_file(size):
    import numpy as np
    v = np.arange(size // 4, dtype=np.uint32).astype(">u4").view(np.uint8)
    return v.tobytes() + b"\0" * (size % 4)


def _oracle_striped_write(k, m, cell, data):
    """StripedBlockWriter (block_writer.rs:904-1035) over one block group with
    the oracle's CellBuffer::encode (block_writer.rs:817-851) per row."""
    shards = [b""] * (k + m)
    row = k * cell
    for r0 in range(0, len(data), row):
        chunk = data[r0:r0 + row]
        cells = [chunk[i * cell:(i + 1) * cell] for i in range(k)]
        out = O.cell_buffer_encode(k, m, cells)
        shards = [s + o for s, o in zip(shards, out)]
    return shards


@pytest.mark.gpu
def test_striped_write_faulty_read_roundtrip(binary, tmp_path):
    env = dict(os.environ, HEC_MIRROR_DUMP=str(tmp_path))
    r = subprocess.run([binary, "gpu"], capture_output=True, text=True, timeout=900, env=env)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "ALL OK" in r.stdout
    # the striped write's shard bytes, pinned against the oracle
    cell = 65536
    for k, m in [(3, 2), (6, 3), (10, 4)]:
        for size in (cell * k * 5 + 4, cell - 4):
            want = _oracle_striped_write(k, m, cell, _counter_file(size))
            for i in range(k + m):
                got = (tmp_path / f"{k}_{m}_{size}_{i}.bin").read_bytes()
                assert got == want[i], (k, m, size, i)
