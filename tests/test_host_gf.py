"""The engine's host-side GF(2^8) multiply (hdfs-native_amd/csrc/host_gf.cpp:
AVX-512BW+GFNI, AVX2, scalar), the per-call drop-in's small-row path, against
the oracle on the CPU: tests/cpp/host_gf_check.cpp runs every ISA this CPU
supports over RS encode/decode matrices and random matrices at every tail
length, and checks the affine bit matrix of every coefficient."""
import os
import subprocess

from conftest import PKG_DIR

BIN = os.path.join(PKG_DIR, "build", "host_gf_check")


def test_host_gf_every_isa_vs_oracle():
    if not os.path.exists(BIN):
        subprocess.check_call(["make", "-s", "-C", PKG_DIR, "build/host_gf_check"])
    out = subprocess.run([BIN], capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stderr[-4000:]
    assert "host gf ok" in out.stdout


BSL_BIN = os.path.join(PKG_DIR, "build", "bitslice_check")


def test_bitslice_networks_vs_oracle():
    """The fused encode kernel's bit-sliced parity (8x8 bit transpose +
    generated XOR networks) equals the oracle's RS parity, per byte."""
    subprocess.check_call(["make", "-s", "-C", PKG_DIR, "build/bitslice_check"])
    out = subprocess.run([BSL_BIN], capture_output=True, text=True, timeout=120)
    assert out.returncode == 0, out.stderr[-4000:]
    assert "ok" in out.stdout


NET_BIN = os.path.join(PKG_DIR, "build", "xor_net_check")


def test_plan_time_xor_networks_every_decode_plan():
    """The networks the JIT-specialised decode + verify kernel runs
    (csrc/xor_net.hpp): every decode plan of RS(3,2), RS(6,3) and RS(10,4)
    and random 1..4-row matrices, evaluated on bit-sliced cells on the host,
    equal the oracle's decode / multiply."""
    subprocess.check_call(["make", "-s", "-C", PKG_DIR, "build/xor_net_check"])
    out = subprocess.run([NET_BIN], capture_output=True, text=True, timeout=120)
    assert out.returncode == 0, out.stdout[-4000:] + out.stderr[-4000:]
    assert "xor net ok" in out.stdout


def _oracle_matmul(mat, ins):
    import ec_oracle as O
    return [bytes(x) for x in O.matmul_shards(mat, ins)]


def test_host_split_more_rows_than_piece_arrays():
    """Rows past the split pieces' 64-entry pointer arrays: a
    >= 256 KiB row of an 80 x 3 matrix is coded unsplit, bit-exact."""
    import numpy as np
    import hdfs_native_ec as H
    rng = np.random.default_rng(80)
    rows, cols, n = 80, 3, (256 << 10) + 4096
    mat = [[int(v) for v in rng.integers(0, 256, cols)] for _ in range(rows)]
    ins = [rng.integers(0, 256, n, dtype=np.uint8) for _ in range(cols)]
    got = H.gf_matmul_host(mat, ins)
    # the oracle on a slice of each row keeps this quick; the split would
    # have cut the row at 4 KiB multiples, so check both ends of every row
    for lo, hi in ((0, 8192), (n - 8192, n)):
        want = _oracle_matmul(mat, [x[lo:hi] for x in ins])
        assert [g[lo:hi] for g in got] == want


def _fork_child(q):
    import numpy as np
    import hdfs_native_ec as H
    rng = np.random.default_rng(7)
    ins = [rng.integers(0, 256, 1 << 20, dtype=np.uint8) for _ in range(6)]
    mat = H.gen_rs_matrix(6, 3)[6:]
    q.put(b"".join(H.gf_matmul_host(mat, ins)))


def test_host_split_pool_survives_fork():
    """The worker pool that splits long rows is process-wide; a fork()ed
    child (multiprocessing's default start method) must code a long row on
    a pool of its own instead of waiting for the parent's workers, which do
    not exist in the child."""
    import multiprocessing as mp
    import numpy as np
    import hdfs_native_ec as H
    rng = np.random.default_rng(7)
    ins = [rng.integers(0, 256, 1 << 20, dtype=np.uint8) for _ in range(6)]
    mat = H.gen_rs_matrix(6, 3)[6:]
    want = b"".join(H.gf_matmul_host(mat, ins))  # the parent's pool exists now
    ctx = mp.get_context("fork")
    q = ctx.Queue()
    p = ctx.Process(target=_fork_child, args=(q,))
    p.start()
    got = q.get(timeout=60)
    p.join(timeout=60)
    assert p.exitcode == 0
    assert got == want
