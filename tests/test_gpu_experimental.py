"""Parity of every knob-selected shape and of the measured-and-rejected
kernel variants, which exist only in the HEC_EXPERIMENTAL measurement build
(hdfs-native_amd/lib/libhdfs_ec_amd_exp.so, `make -C hdfs-native_amd exp`;
the #ifdef'd shapes and CRC schemes; knobs in
include/hdfs_ec_amd_exp.h).  Same oracle and same bit-exact bar as the
product library; every coder here is bound to the measurement build and its
knobs are that library's own.  The product library has no knobs: its
default paths are covered by tests/test_gpu_parity.py, whose test bodies are
reused here with knobs set.  Skipped when the measurement build is absent
(it is not built or shipped by default)."""
import threading

import numpy as np
import pytest

import ec_oracle as O
import hdfs_native_ec as H
import test_gpu_parity as P
from hdfs_native_ec.synth import batch_data

pytestmark = [pytest.mark.gpu,
              pytest.mark.skipif(not H.experimental_available(),
                                 reason="measurement build not built (make -C hdfs-native_amd exp)")]

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


@pytest.mark.parametrize("k,m", [(10, 4), (10, 1), (10, 3)])
@pytest.mark.parametrize("cell", [8192 + 16, 3 * 65536 + 48, 1 << 20])
@pytest.mark.parametrize("bpc", [0, 2, 3])
@pytest.mark.parametrize("S", [1, 3, 9])
def test_pair_kernel_vs_oracle(xlib, dev, c_oracle, k, m, cell, bpc, S):
    # tune key 32 = 1: RS(10,*) on the wave-pair kernel (two waves per
    # wave-tile, partials through LDS), 1-4 rows (decode of 1..m data shards:
    # wave 1 stores nothing at one row), partial last tiles, 2 / 3 / 4 blocks
    # of 128 threads per CU, small batches (fewer tiles than counters)
    knobs = [(32, 1)] + ([(3, bpc)] if bpc else [])
    run_variant(xlib, c_oracle, dev, k, m, S, cell, knobs, cell + 7 * S + bpc)


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


@pytest.mark.parametrize("cell,bpc,n", [c for c in P.CRC32C_CASES if c[1] == 512])
@pytest.mark.parametrize("wq", [1, 2, 4, 8, 16])
def test_crc_wq_vs_oracle(xlib, dev, cell, bpc, n, wq):
    """Tune key 29: the CRC32C fold kernel on the work queue, 1 / 2 / 4 tasks
    per unit (partial last tasks, short last chunks, units that run past the
    last task), against the oracle."""
    P.crc32c_body(dev, cell, bpc, n, P.coder(6, 3, xlib), [(29, wq)], xlib)


@pytest.mark.parametrize("cell,bpc,n", [c for c in P.CRC32C_CASES if c[1] == 512])
@pytest.mark.parametrize("runs", [2, 4, 8, 16])
def test_crc_runs_vs_oracle(xlib, dev, cell, bpc, n, runs):
    """Tune key 31: the CRC32C fold kernel in runs of 2 / 4 consecutive tasks
    per wave, against the oracle, and at full size against the default."""
    P.crc32c_body(dev, cell, bpc, n, P.coder(6, 3, xlib), [(31, runs)], xlib)
    S, nn, c1 = 16, 9, 1 << 20
    x = torch.empty((S, nn, c1), dtype=torch.uint8, device=dev)
    x.random_(0, 256, generator=torch.Generator(device=dev).manual_seed(31 + runs))
    c = xcoder(xlib, 6, 3)
    want = H.crc32c_batch(c, x, 512)
    with P.knobs([(31, runs)], xlib):
        got = H.crc32c_batch(c, x, 512)
        torch.cuda.synchronize()
    assert torch.equal(got, want)


@pytest.mark.parametrize("cell,bpc,n", [c for c in P.CRC32C_CASES if c[1] == 512])
def test_crc_768_vs_oracle(xlib, dev, cell, bpc, n):
    """Tune key 33 = 768: the CRC32C fold kernel in one 768-thread block per
    CU (3 waves per SIMD), against the oracle."""
    P.crc32c_body(dev, cell, bpc, n, P.coder(6, 3, xlib), [(33, 768)], xlib)


@pytest.mark.parametrize("knob", [(29, 1), (29, 4), (29, 16), (33, 768)])
def test_crc_wq_full_size_compute_and_verify(xlib, dev, knob):
    """Keys 29 / 33 at full size (9 x 1 MiB x 64 cells), three launches in a
    row on one stream: sums equal the default kernel's, and verify mode flags
    exactly the corrupted cells."""
    S, n, cell = 64, 9, 1 << 20
    c = xcoder(xlib, 6, 3)
    g = torch.Generator(device=dev).manual_seed(29 + knob[1])
    x = torch.empty((S, n, cell), dtype=torch.uint8, device=dev)
    x.random_(0, 256, generator=g)
    want = H.crc32c_batch(c, x, 512)
    hits = {(0, 0): 0, (5, 8): cell - 1, (31, 4): cell // 2 + 3, (63, 2): 8191, (63, 6): 8192}
    with P.knobs([knob], xlib):
        for _ in range(3):
            got = H.crc32c_batch(c, x, 512)
            torch.cuda.synchronize()
            assert torch.equal(got, want)
        y = x.clone()
        for (s_, i), b in hits.items():
            y[s_, i, b] ^= 0x41
        bad = H.checksum_verify_batch(c, y, want, H.CHECKSUM_CRC32C, 512)
        torch.cuda.synchronize()
    flags = torch.zeros((S, n), dtype=torch.uint8)
    for s_, i in hits:
        flags[s_, i] = 1
    assert torch.equal(bad.cpu(), flags)


FUSED_TUNES = [[(11, 2)], [(11, 6)], [(16, 3)], [(16, 3), (11, 1)]]


@pytest.mark.parametrize("k,m,cell,S", [(6, 3, 1 << 16, 3), (10, 4, 1 << 15, 2), (3, 2, 8192 + 512, 4)])
@pytest.mark.parametrize("tunes", FUSED_TUNES + [[(22, 1)], [(22, 1), (5, 0)], [(24, 3)], [(10, 4)], [(10, 4), (24, 2)],
                                   [(25, 1)], [(25, 7), (10, 4)]])
def test_fused_variants_encode_vs_oracle(xlib, dev, c_oracle, k, m, cell, S, tunes):
    """Fused encode + CRC32C with the rejected variants: bank-replicated
    slicing-by-1 / -by-2 tables (tune key 11 = 2 / 6), one 768-thread block
    per CU (key 16 = 3, 11-bit slicing or slicing-by-8), the v_perm table
    parity instead of the default bit-sliced networks (key 22 = 1), the
    load schedules: early issue at 8 slabs (key 24 = 3), inputs in pairs at 4
    slabs with one or two pairs ahead (key 10 = 4, key 24 = 2), and the
    per-stripe column rotation (key 25)."""
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


@pytest.mark.parametrize("k,m,cell,S", [(6, 3, 1 << 16, 3), (6, 3, (1 << 15) + 512 + 100, 2), (10, 4, 1 << 15, 2)])
def test_fused_encode_slice32_tail_vs_oracle(xlib, dev, c_oracle, k, m, cell, S):
    """Fused encode + CRC32C with the slicing-by-32 CRC tail (tune key 11 =
    12): parity and every chunk sum, short last chunks included."""
    test_fused_variants_encode_vs_oracle(xlib, dev, c_oracle, k, m, cell, S, [(11, 12)])


def _xjit_launches(xlib):
    import ctypes
    v = [ctypes.c_uint64(0) for _ in range(4)]
    xlib.hec_jit_stats(*[ctypes.byref(x) for x in v])
    return v[3].value


JIT_SHAPE_CASES = [
    # (k, m, cell, missing, tunes, checksum type): every case a fresh hiprtc compile
    (6, 3, 1 << 15, (0, 1, 2), [(24, 3)], H.CHECKSUM_CRC32C),
    (6, 3, (1 << 15) + 512, (0,), [(24, 3)], H.CHECKSUM_CRC32),
    (3, 2, 8192 + 512, (0, 1), [(24, 3)], H.CHECKSUM_CRC32C),
    (6, 3, 1 << 15, (0, 1, 2), [(10, 4)], H.CHECKSUM_CRC32C),
    (6, 3, (1 << 15) + 512, (0, 2), [(10, 4), (24, 2)], H.CHECKSUM_CRC32C),
    (10, 4, 1 << 14, (0, 1, 2, 3), [(10, 4), (24, 2)], H.CHECKSUM_CRC32),
    (6, 3, 1 << 15, (1,), [(10, 4), (16, 3)], H.CHECKSUM_CRC32C),
    (10, 4, (1 << 14) + 512, (0, 5), [(10, 4), (16, 3)], H.CHECKSUM_CRC32C),
    (6, 3, 1 << 15, (0, 1, 2), [(10, 8)], H.CHECKSUM_CRC32),
    (6, 3, 1 << 15, (0, 1, 2), [(24, 4)], H.CHECKSUM_CRC32C),
    (6, 3, (1 << 15) + 512, (1,), [(24, 4)], H.CHECKSUM_CRC32),
    (6, 3, (1 << 15) + 512, (0, 2), [(10, 4), (24, 4)], H.CHECKSUM_CRC32C),
    (10, 4, (1 << 14) + 512, (0, 1, 2, 3), [(24, 4)], H.CHECKSUM_CRC32C),
    (3, 2, 8192 + 512, (0, 1), [(24, 4)], H.CHECKSUM_CRC32),
    (6, 3, 1 << 15, (0, 1, 2), [(24, 5)], H.CHECKSUM_CRC32C),
    (6, 3, (1 << 15) + 512, (1,), [(24, 5)], H.CHECKSUM_CRC32),
    (6, 3, (1 << 15) + 512, (0, 2), [(10, 8), (24, 5)], H.CHECKSUM_CRC32C),
    (10, 4, (1 << 14) + 512, (0, 1, 2, 3), [(24, 5)], H.CHECKSUM_CRC32C),
    (3, 2, 8192 + 512, (0, 1), [(24, 5)], H.CHECKSUM_CRC32),
    (2, 1, 8192, (0,), [(24, 5)], H.CHECKSUM_CRC32C),
    (6, 3, 1 << 15, (0, 1, 2), [(11, 12)], H.CHECKSUM_CRC32C),
    (6, 3, (1 << 15) + 512, (1,), [(11, 12)], H.CHECKSUM_CRC32C),
    (10, 4, (1 << 14) + 512, (0, 1, 2, 3), [(11, 12)], H.CHECKSUM_CRC32C),
    (3, 2, 8192 + 512, (0, 1), [(11, 12), (10, 8)], H.CHECKSUM_CRC32C),
    (6, 3, (1 << 15) + 512, (0, 1, 2), [(25, 1)], H.CHECKSUM_CRC32C),
    (10, 4, (1 << 16) + 512, (0, 3), [(25, 7)], H.CHECKSUM_CRC32),
    (6, 3, (1 << 16) + 512, (2,), [(25, 5), (24, 3), (10, 8)], H.CHECKSUM_CRC32C),
    # tune key 28 = 1: the specialised kernel on the work queue of wave-tiles
    (6, 3, (1 << 15) + 512, (0, 1, 2), [(28, 1)], H.CHECKSUM_CRC32C),
    (6, 3, 1 << 15, (1,), [(28, 1)], H.CHECKSUM_CRC32),
    (10, 4, (1 << 14) + 512, (0, 1, 2, 3), [(28, 1)], H.CHECKSUM_CRC32C),
    (10, 4, (1 << 16) + 512, (0, 5), [(28, 1)], H.CHECKSUM_CRC32),
    (3, 2, 8192 + 512, (0, 1), [(28, 1)], H.CHECKSUM_CRC32C),
    (2, 1, 8192, (0,), [(28, 1)], H.CHECKSUM_CRC32C),
    (6, 3, (1 << 15) + 512, (0, 2), [(28, 1), (16, 3), (10, 4)], H.CHECKSUM_CRC32C),
    (6, 3, (1 << 15) + 512, (0, 1, 2), [(28, 1), (24, 5)], H.CHECKSUM_CRC32C),
]


@pytest.mark.parametrize("k,m,cell,missing,tunes,ctype", JIT_SHAPE_CASES)
def test_jit_verify_shapes_vs_oracle(xlib, dev, c_oracle, k, m, cell, missing, tunes, ctype):
    """The plan-specialised decode + verify kernel at every shape the
    measurement build can ask for (slabs, waves per SIMD, load schedule),
    prepared synchronously on a measurement-build coder: rebuilt data, bad
    flags and errors as the oracle's read_slice restatement (the parity suite's
    body); the library's launch counter proves the specialised kernel ran."""
    for key, value in tunes:
        H.tune_set(key, value, xlib)
    try:
        cod = H.Coder(k, m, 0, lib=xlib)
        assert cod.prepare_decode(list(missing), ctype), "hiprtc unavailable on the GPU box"
        before = _xjit_launches(xlib)
        P.decode_verify_body(dev, c_oracle, ctype, k, m, cell, 512, list(missing), [], cod)
        assert _xjit_launches(xlib) > before
        cod.close()
    finally:
        for key, _ in tunes:
            H.tune_set(key, 0, xlib)


# ---- knob-selected shapes of the product kernels -------------------------

@pytest.mark.parametrize("knob", [((1, 1),), ((1, 2),), ((1, 4),), ((2, 0),), ((3, 2),), ((4, 512), (1, 1)),
                                  ((4, 512), (1, 2)), ((1, 4), (2, 0), (3, 3)), ((5, 2),), ((5, 2), (1, 2)),
                                  ((5, 2), (4, 512)), ((5, 2), (3, 2)), ((5, 1),), ((6, 1),), ((6, 2),),
                                  ((6, 2), (4, 512)), ((7, 100),), ((7, 3),), ((8, 2),), ((8, 3),), ((8, 4), (5, 2)),
                                  ((8, 64),), ((7, 16),), ((7, 12),)])
def test_tuning_variants_bit_identical(xlib, dev, c_oracle, knob):
    run_variant(xlib, c_oracle, dev, 6, 3, 5, 8192 + 16, list(knob), 21)


@pytest.mark.parametrize("knob", [((1, 8),), ((1, 8), (3, 2)), ((1, 8), (7, 5))])
@pytest.mark.parametrize("k,m", [(2, 1), (3, 2)])
@pytest.mark.parametrize("cell", [8192 + 16, 3 * 65536 + 48, (1 << 20) + 16])
def test_eight_chunks_per_lane_small_k(xlib, dev, c_oracle, knob, k, m, cell):
    # 8 x 16-B chunks per lane (k <= 3): full and partial tiles, small grids
    run_variant(xlib, c_oracle, dev, k, m, 3, cell, list(knob) + [(5, 1)], cell + k)


@pytest.mark.parametrize("pipeline", [1, 2])
@pytest.mark.parametrize("grid", [0, 1, 5])
@pytest.mark.parametrize("k,m", [(2, 1), (3, 2), (6, 3), (10, 4)])
@pytest.mark.parametrize("cell", [8192 + 16, 3 * 65536 + 48])
def test_bitsliced_encode_kernels(xlib, dev, c_oracle, pipeline, grid, k, m, cell):
    # tune key 23 = 1: the RS parity rows as bit-sliced XOR networks in the
    # register kernel (gf_encode_bsl, pipeline 1) and the LDS-DMA kernel
    # (pipeline 2); RS(2,1) keeps the tables; partial last tiles, small grids
    run_variant(xlib, c_oracle, dev, k, m, 3, cell, [(23, 1), (5, pipeline), (7, grid)], cell + 3 * k + grid)


@pytest.mark.parametrize("pipeline", [1, 2])
@pytest.mark.parametrize("k,m", [(2, 1), (3, 2), (6, 3), (10, 4)])
@pytest.mark.parametrize("cell", [4096, 4096 + 16, 3 * 65536 + 48])
@pytest.mark.parametrize("S", [3, 6])
def test_pipelines_forced_vs_oracle(xlib, dev, c_oracle, pipeline, k, m, cell, S):
    # tune key 5: the register (1) or LDS-DMA (2) kernel whatever the cell size
    with P.knobs([(5, pipeline)], xlib):
        P.pipelines_body(dev, c_oracle, k, m, cell, S, P.coder(k, m, xlib))


def test_tune_set_concurrent_with_launches(xlib, dev, c_oracle):
    # hec_tune_set while other threads launch: the knobs are atomics read once
    # per launch, and every value toggled here is result-neutral
    k, m, S, cell = 6, 3, 4, 65536 + 16
    data = batch_data(S, k, cell, first=5)
    want = oracle_batch_encode(c_oracle, k, m, data)
    stop = threading.Event()
    errors = []

    def toggler():
        i = 0
        while not stop.is_set():
            H.tune_set(3, 1 + i % 2, xlib)
            H.tune_set(8, 1 + 3 * (i % 2), xlib)
            H.tune_set(7, (i % 3) * 64, xlib)
            i += 1

    def launcher(seed):
        try:
            cod = H.Coder(k, m, 0, lib=xlib)
            st = torch.cuda.Stream(dev)
            d = torch.from_numpy(data).to(dev)
            for _ in range(40):
                p = torch.zeros((S, m, cell), dtype=torch.uint8, device=dev)
                with torch.cuda.stream(st):
                    H.encode_batch(cod, d, p, st)
                st.synchronize()
                if not np.array_equal(p.cpu().numpy(), want):
                    errors.append(seed)
            cod.close()
        except Exception as e:  # pragma: no cover - reported below
            errors.append(repr(e))

    t = threading.Thread(target=toggler)
    ls = [threading.Thread(target=launcher, args=(i,)) for i in range(4)]
    t.start()
    for th in ls:
        th.start()
    for th in ls:
        th.join()
    stop.set()
    t.join()
    for key in (3, 7, 8):
        H.tune_set(key, 0, xlib)
    assert not errors, errors


def test_tune_set_rejects_unknown_values(xlib):
    for key, value in [(3, 99), (1, 5), (5, 6), (11, 8), (11, 13), (16, 1), (17, 6), (19, 3), (20, 3), (21, 2), (5, 3), (13, 1), (15, 2), (22, 2), (23, 2), (24, 6), (25, 4097), (26, 5), (27, 4), (28, 3), (29, 3), (30, 2), (31, 3), (32, 2), (33, 512), (34, 0), (0, 0)]:
        with pytest.raises(ValueError):
            H.tune_set(key, value, xlib)


@pytest.mark.parametrize("case", P.UNALIGNED_CASES)
def test_unaligned_byte_kernel_alone(xlib, dev, c_oracle, case):
    # tune key 18 = 1: unaligned layouts through the byte kernel alone
    with P.knobs([(18, 1)], xlib):
        P.unaligned_layouts_body(dev, c_oracle, *case, P.coder(case[0], case[1], xlib))


@pytest.mark.parametrize("k,m,cell", [(6, 3, 4096), (10, 4, 8192), (3, 2, 4096 + 16), (4, 2, 4096)])
@pytest.mark.parametrize("skip", [1, 2])
def test_mixed_row_policies(xlib, dev, c_oracle, k, m, cell, skip):
    # tune key 20: rows past a stripe's erasure count computed (1) or skipped (2)
    P.mixed_patterns_body(dev, c_oracle, k, m, cell, P.coder(k, m, xlib), [(20, skip)], xlib)


def test_mixed_many_plans_skipped_rows(xlib, dev):
    P.mixed_many_plans_body(dev, P.coder(10, 4, xlib), [(20, 2)], xlib)


@pytest.mark.parametrize("k,m,cell", [(6, 3, 4096), (6, 3, 65536 + 64), (10, 4, 8192), (3, 2, 4096 + 16),
                                      (2, 1, 1024), (6, 3, 1 << 20)])
@pytest.mark.parametrize("wq", [2, 3])
def test_mixed_work_queue(xlib, dev, c_oracle, k, m, cell, wq):
    """Tune key 26: the mixed decode's work queue at 2 rounds of wave-tiles
    per atomic (the product runs 1 and 4) and the fixed tile order it
    replaced (3), against the oracle."""
    for _ in range(2):
        P.mixed_patterns_body(dev, c_oracle, k, m, cell, P.coder(k, m, xlib), [(26, wq)], xlib)


@pytest.mark.parametrize("k,m,cell,S", [(6, 3, 1 << 20, 24), (10, 4, 1 << 20, 12), (3, 2, 1 << 20, 24),
                                        (2, 1, 65536 * 8, 9), (10, 4, 65536, 40), (6, 3, 1 << 20, 1)])
@pytest.mark.parametrize("wq", [1, 2, 3])
def test_matmul_work_queue(xlib, dev, c_oracle, k, m, cell, S, wq):
    """Tune key 27: the register kernel's work queue at 1 and 2 rounds of
    wave-tiles per atomic (the product runs 2 for k <= 3, 1 for k = 6, 10)
    and the fixed tile order it replaced (3): encode and decode of data
    0..m-1 against the oracle, three launches in a row (the counters must
    come back to zero)."""
    d = P._device_random((S, k, cell), dev, seed=k * 100 + S + wq)
    c = P.coder(k, m, xlib)
    with P.knobs([(27, wq)], xlib):
        for _ in range(3):
            p = torch.empty((S, m, cell), dtype=torch.uint8, device=dev)
            H.encode_batch(c, d, p)
            out = torch.zeros_like(d)
            H.decode_batch(c, d, p, list(range(m)), out)
            torch.cuda.synchronize()
            assert torch.equal(out[:, :m], d[:, :m])
    O.c_check_batch(c_oracle, k, m, d.cpu().numpy(), p.cpu().numpy(), threads=4)


@pytest.mark.parametrize("codec,k,m,cell,S", [c for c in P.ENCODE_CRC_CASES if c[1] in (3, 6, 10) and c[0] == "rs"])
@pytest.mark.parametrize("wq", [1, 2])
def test_encode_crc_work_queue(xlib, dev, c_oracle, codec, k, m, cell, S, wq):
    """Tune key 28: fused encode + CRC with the work queue at k = 3, 6, 10 (1)
    and with the block tiles it replaced at k = 3, 10 (2), against the
    oracle's parity and sums."""
    P.encode_crc_body(dev, c_oracle, codec, k, m, cell, S, xlib, [(28, wq)])


@pytest.mark.parametrize("S", [24, 256])
@pytest.mark.parametrize("wq", [2, 3])
def test_mixed_work_queue_resident_plans(xlib, dev, S, wq):
    """RS(10,4) random losses of any shards, key 26 = 2 / 3: plans under and
    past 64 KiB of LDS (S = 512 restages per stripe: no queue there)."""
    P.mixed_many_plans_body(dev, P.coder(10, 4, xlib), [(26, wq)], xlib, S=S)
    P.mixed_many_plans_body(dev, P.coder(10, 4, xlib), [(26, wq)], xlib, S=512)


@pytest.mark.parametrize("cell,bpc,n", P.CRC32C_CASES)
@pytest.mark.parametrize("variant,pf", [(0, 2), (1, 1), (1, 2), (5, 0), (5, 1), (5, 2), (7, 1), (10, 1), (11, 1)])
def test_crc32c_lookup_schemes(xlib, dev, cell, bpc, n, variant, pf):
    # tune key 11: slicing-by-8 (1), 11-bit slicing (5), the fold (0 / 7), fold depth 16 / 20
    # (10 / 11); key 12: prefetch
    P.crc32c_body(dev, cell, bpc, n, P.coder(6, 3, xlib), [(11, variant), (12, pf)], xlib)


@pytest.mark.parametrize("ctype", P.CKSUM_TYPES)
@pytest.mark.parametrize("cell,bpc,n", P.CHECKSUM_CASES)
@pytest.mark.parametrize("variant", [1, 5])
def test_checksum_lookup_schemes(xlib, dev, ctype, cell, bpc, n, variant):
    P.checksum_body(dev, ctype, cell, bpc, n, P.coder(6, 3, xlib), [(11, variant)], xlib)


@pytest.mark.parametrize("case", P.ENCODE_CRC_CASES)
@pytest.mark.parametrize("fused,scheme", [(4, 0), (8, 0), (None, 0), (0, 1), (0, 5), (4, 5), (8, 1), (0, 10), (0, 11)])
def test_encode_crc_knobs(xlib, dev, c_oracle, case, fused, scheme):
    # key 9 = 1: two passes; key 10: slabs per wave; key 11: lookup scheme
    pairs = [(9, 1 if fused is None else 0), (10, fused or 0), (11, scheme)]
    P.encode_crc_body(dev, c_oracle, *case, xlib, pairs)


@pytest.mark.parametrize("k,m,cell,S,slabs", [(10, 4, 1 << 15, 3, 0), (3, 2, 8192 + 512, 4, 4), (6, 3, 1 << 14, 2, 4)])
@pytest.mark.parametrize("pair", [1, 2])
def test_fused_input_pairing(xlib, dev, c_oracle, k, m, cell, S, slabs, pair):
    """Fused encode + CRC32C and decode + verify at 4 slabs per wave with the
    inputs two at a time (tune key 19 = 2, the default) and one at a time (1),
    an odd k included, against the oracle."""
    bpc = 512
    data = batch_data(S, k, cell, first=57 + cell + pair)
    par = oracle_batch_encode(c_oracle, k, m, data)
    d = torch.from_numpy(data).to(dev)
    p = torch.zeros((S, m, cell), dtype=torch.uint8, device=dev)
    nch = cell // bpc
    sums = torch.zeros((S, k + m, nch, 4), dtype=torch.uint8, device=dev)
    dp, ds = H.stripe_layout_ptrs(d, k)
    pp, ps = H.stripe_layout_ptrs(p, m)
    sp = torch.cuda.current_stream().cuda_stream
    cod = P.coder(k, m, xlib)
    with P.knobs([(19, pair), (10, slabs)], xlib):
        cod.encode_crc_device(dp, ds, pp, ps, cell, S, bpc, sums.data_ptr(), sp)
        torch.cuda.synchronize()
        assert np.array_equal(p.cpu().numpy(), par)
        want = _oracle_sums(np.concatenate([data, par], axis=1), bpc)
        assert np.array_equal(sums.cpu().numpy(), want)
        out = torch.zeros_like(d)
        bad = torch.zeros((S, k + m), dtype=torch.uint8, device=dev)
        op, os_ = H.stripe_layout_ptrs(out, k)
        miss = list(range(min(m, k)))
        cod.decode_verify_device(H.CHECKSUM_CRC32C, [None if i in miss else dp[i] for i in range(k)] + pp, ds + ps,
                                 op, os_, cell, S, bpc, sums.data_ptr(), bad.data_ptr(), sp)
        torch.cuda.synchronize()
    assert not bad.cpu().numpy().any()
    o = out.cpu().numpy()
    for i in miss:
        assert np.array_equal(o[:, i], data[:, i])


@pytest.mark.parametrize("ctype", P.CKSUM_TYPES)
@pytest.mark.parametrize("case", P.VERIFY_CASES)
@pytest.mark.parametrize("scheme", [1, 5, 10, 11])
def test_decode_verify_lookup_schemes(xlib, dev, c_oracle, ctype, case, scheme):
    P.decode_verify_body(dev, c_oracle, ctype, *case, P.coder(case[0], case[1], xlib), [(11, scheme)], xlib)
