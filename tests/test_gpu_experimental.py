"""Parity of the measured-and-rejected kernel variants, which exist only in
the HEC_EXPERIMENTAL build (hdfs-native_amd/lib/libhdfs_ec_amd_exp.so, `make
exp`; ec_experimental.hip and the #ifdef'd CRC schemes).  Same oracle and
same bit-exact bar as the default library; every coder here is bound to the
experimental library and its knobs are that library's own."""
import numpy as np
import pytest

import ec_oracle as O
import hdfs_native_ec as H
from hdfs_native_ec.synth import batch_data

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")


@pytest.fixture(scope="module")
def dev():
    assert torch.cuda.is_available(), "GPU test run without a GPU"
    return torch.device("cuda:0")


@pytest.fixture(scope="module")
def xlib():
    return H.experimental_lib()


_coders = {}


def xcoder(xlib, k, m):
    if (k, m) not in _coders:
        _coders[(k, m)] = H.Coder(k, m, 0, lib=xlib)
    return _coders[(k, m)]


def oracle_batch_encode(c_oracle, k, m, data):
    S, _, n = data.shape
    par = np.empty((S, m, n), dtype=np.uint8)
    d = np.ascontiguousarray(data)
    assert c_oracle.orc_encode_batch(k, m, d.ctypes.data, n, S, par.ctypes.data) == 0
    return par


def run_variant(xlib, c_oracle, dev, k, m, S, cell, knobs, first):
    data = batch_data(S, k, cell, first=first)
    want = oracle_batch_encode(c_oracle, k, m, data)
    d = torch.from_numpy(data).to(dev)
    p = torch.zeros((S, m, cell), dtype=torch.uint8, device=dev)
    out = torch.zeros_like(d)
    try:
        for key, val in knobs:
            H.tune_set(key, val, xlib)
        H.encode_batch(xcoder(xlib, k, m), d, p)
        H.decode_batch(xcoder(xlib, k, m), d, p, list(range(m)), out)
        torch.cuda.synchronize()
    finally:
        for key, _ in knobs:
            H.tune_set(key, -1 if key == 2 else 0, xlib)
    assert np.array_equal(p.cpu().numpy(), want)
    assert torch.equal(out[:, :m], d[:, :m])


@pytest.mark.parametrize("unroll", [1, 2, 3])
@pytest.mark.parametrize("grid", [0, 1, 5, 6])
@pytest.mark.parametrize("k,m", [(2, 1), (3, 2), (6, 3), (10, 4)])
def test_register_pipe_vs_oracle(xlib, dev, c_oracle, unroll, grid, k, m):
    # tune key 5 = 3: register pipe kernel.  Small grids walk many tiles per
    # block (both register sets, odd and even tile counts, the clamped
    # past-the-end prefetch); the cell leaves a partial last tile.
    cell = 3 * 65536 + 48
    run_variant(xlib, c_oracle, dev, k, m, 3, cell, [(5, 3), (1, unroll), (7, grid)], cell + 7 * k + unroll)


@pytest.mark.parametrize("unroll,block", [(4, 256), (2, 256), (1, 512)])
@pytest.mark.parametrize("grid", [0, 1, 5, 6])
@pytest.mark.parametrize("k,m", [(2, 1), (3, 2), (6, 3), (10, 4)])
def test_double_buffered_vs_oracle(xlib, dev, c_oracle, unroll, block, grid, k, m):
    # tune key 5 = 5: drain-free register double buffering (two register and
    # two accumulator sets); grids of 1/5/6 blocks cover odd and even tile
    # counts per block and the past-the-end re-read
    cell = 3 * 65536 + 48
    run_variant(xlib, c_oracle, dev, k, m, 3, cell, [(5, 5), (1, unroll), (4, block), (7, grid)],
                cell + 13 * k + unroll)


@pytest.mark.parametrize("tiles", [2, 3])
@pytest.mark.parametrize("grid", [0, 1, 5])
@pytest.mark.parametrize("k,m", [(2, 1), (3, 2), (6, 3)])
def test_output_burst_vs_oracle(xlib, dev, c_oracle, tiles, grid, k, m):
    # tune key 5 = 4: outputs parked in LDS, stored in bursts of `tiles`
    # column tiles; partial super-tiles at the cell end, many per block
    cell = 3 * 65536 + 48
    run_variant(xlib, c_oracle, dev, k, m, 3, cell, [(5, 4), (15, tiles), (7, grid)], cell + 11 * k + tiles)


@pytest.mark.parametrize("pol", [1, 2, 3, 4])
@pytest.mark.parametrize("unroll", [1, 2])
@pytest.mark.parametrize("k,m", [(6, 3), (10, 4)])
def test_store_policies_vs_oracle(xlib, dev, c_oracle, pol, unroll, k, m):
    # tune key 13: cache policy of the pipe kernel's stores (sc1 / sc0 sc1 /
    # nt sc1 / plain, inline-asm stores) at the bench shapes
    run_variant(xlib, c_oracle, dev, k, m, 5, 65536 + 32, [(5, 3), (1, unroll), (13, pol), (7, 7)], pol * 31 + unroll)


def _oracle_sums(cells, bpc, ctype=H.CHECKSUM_CRC32C):
    S, n, cell = cells.shape
    nch = (cell + bpc - 1) // bpc
    out = np.empty((S, n, nch, 4), dtype=np.uint8)
    for s in range(S):
        for i in range(n):
            out[s, i] = np.frombuffer(O.chunk_checksums(cells[s, i].tobytes(), bpc, ctype),
                                      dtype=np.uint8).reshape(nch, 4)
    return out


@pytest.mark.parametrize("ctype", [H.CHECKSUM_CRC32C, H.CHECKSUM_CRC32])
@pytest.mark.parametrize("cell,bpc,n", [(512 * 64, 512, 3), (512 * 70 + 256, 512, 2), (1000, 512, 3)])
@pytest.mark.parametrize("variant,pf", [(2, 2), (3, 1), (3, 2), (4, 0), (6, 1), (6, 2)])
def test_crc_schemes_vs_oracle(xlib, dev, ctype, cell, bpc, n, variant, pf):
    """Bank-replicated slicing-by-1 (4 / 8 chains), slicing-by-8 at 4 waves
    per SIMD and bank-replicated slicing-by-2 (tune key 11 = 2, 3, 4, 6)."""
    cells = batch_data(3, n, cell, first=cell + bpc + ctype + variant)
    H.tune_set(11, variant, xlib)
    H.tune_set(12, pf, xlib)
    try:
        got = H.checksum_batch(xcoder(xlib, 6, 3), torch.from_numpy(cells).to(dev), ctype, bpc)
        torch.cuda.synchronize()
    finally:
        H.tune_set(11, 0, xlib)
        H.tune_set(12, 0, xlib)
    assert np.array_equal(got.cpu().numpy(), _oracle_sums(cells, bpc, ctype))


FUSED_TUNES = [[(11, 2)], [(11, 6)], [(16, 3)], [(16, 3), (11, 1)]]


@pytest.mark.parametrize("k,m,cell,S", [(6, 3, 1 << 16, 3), (10, 4, 1 << 15, 2), (3, 2, 8192 + 512, 4)])
@pytest.mark.parametrize("tunes", FUSED_TUNES)
def test_fused_variants_encode_vs_oracle(xlib, dev, c_oracle, k, m, cell, S, tunes):
    """Fused encode + CRC32C with the rejected variants: bank-replicated
    slicing-by-1 / -by-2 tables (tune key 11 = 2 / 6) and one 768-thread
    block per CU (key 16 = 3, 11-bit slicing or slicing-by-8)."""
    bpc = 512
    data = batch_data(S, k, cell, first=77 + cell)
    par = oracle_batch_encode(c_oracle, k, m, data)
    d = torch.from_numpy(data).to(dev)
    p = torch.zeros((S, m, cell), dtype=torch.uint8, device=dev)
    nch = (cell + bpc - 1) // bpc
    sums = torch.zeros((S, k + m, nch, 4), dtype=torch.uint8, device=dev)
    dp, ds = H.stripe_layout_ptrs(d, k)
    pp, ps = H.stripe_layout_ptrs(p, m)
    for key, value in tunes:
        H.tune_set(key, value, xlib)
    try:
        xcoder(xlib, k, m).encode_crc_device(dp, ds, pp, ps, cell, S, bpc, sums.data_ptr(),
                                              torch.cuda.current_stream().cuda_stream)
        torch.cuda.synchronize()
    finally:
        for key, _ in tunes:
            H.tune_set(key, 0, xlib)
    assert np.array_equal(p.cpu().numpy(), par)
    assert np.array_equal(sums.cpu().numpy(), _oracle_sums(np.concatenate([data, par], axis=1), bpc))


@pytest.mark.parametrize("ctype", [H.CHECKSUM_CRC32C, H.CHECKSUM_CRC32])
@pytest.mark.parametrize("k,m,cell,S", [(6, 3, 1 << 15, 3), (10, 4, 1 << 14, 2)])
@pytest.mark.parametrize("tunes", [t for t in FUSED_TUNES if t != [(11, 2)]])
def test_fused_variants_verify_vs_oracle(xlib, dev, c_oracle, ctype, k, m, cell, S, tunes):
    """Fused decode + verify with the rejected variants: data shard 0 missing,
    one survivor byte of stripe 1 corrupted -> flagged, re-planned, rebuilt."""
    bpc = 512
    data = batch_data(S, k, cell, first=91 + cell + ctype)
    par = oracle_batch_encode(c_oracle, k, m, data)
    sums = torch.from_numpy(_oracle_sums(np.concatenate([data, par], axis=1), bpc, ctype)).to(dev)
    bent = data.copy()
    bent[1, 2, cell // 3] ^= 0x21
    d, p = torch.from_numpy(bent).to(dev), torch.from_numpy(par).to(dev)
    out = torch.zeros_like(d)
    bad = torch.zeros((S, k + m), dtype=torch.uint8, device=dev)
    dp, ds = H.stripe_layout_ptrs(d, k)
    pp, ps = H.stripe_layout_ptrs(p, m)
    op, os_ = H.stripe_layout_ptrs(out, k)
    for key, value in tunes:
        H.tune_set(key, value, xlib)
    try:
        xcoder(xlib, k, m).decode_verify_device(ctype, [None] + dp[1:] + pp, ds + ps, op, os_, cell, S, bpc,
                                                sums.data_ptr(), bad.data_ptr(),
                                                torch.cuda.current_stream().cuda_stream)
        torch.cuda.synchronize()
    finally:
        for key, _ in tunes:
            H.tune_set(key, 0, xlib)
    o, b = out.cpu().numpy(), bad.cpu().numpy()
    want_bad = np.zeros((S, k + m), dtype=np.uint8)
    want_bad[1, 2] = 1
    assert np.array_equal(b, want_bad)
    assert np.array_equal(o[:, 0], data[:, 0])
    assert np.array_equal(o[1, 2], data[1, 2])
