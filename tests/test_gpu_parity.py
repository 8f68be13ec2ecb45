"""GPU parity tests: the HIP path (through the C ABI) against the CPU oracle
and the committed golden vectors, bit-exact.  Full-size configs
(BASELINE.json) are checked through size-independent properties:
encode -> erase -> decode round trips, linearity, sampled-stripe oracle
checks.  Edge cases follow the reference tests (rust/tests/test_ec.rs:77-87
sizes 16 B .. +-4 B around cell boundaries; 0..m failures; m+1 fails)."""
import contextlib
import itertools

import numpy as np
import pytest

import ec_oracle as O
import hdfs_native_ec as H
from hdfs_native_ec.synth import batch_data, bench_counter_shards, splitmix64_bytes

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")


@pytest.fixture(scope="module")
def dev():
    assert torch.cuda.is_available(), "GPU test run without a GPU"
    return torch.device("cuda:0")


_coders = {}


def coder(k, m, lib=None):
    """A cached coder on the product library (lib=None) or on another build
    (tests/test_gpu_experimental.py passes the measurement build)."""
    key = (k, m, id(lib))
    if key not in _coders:
        _coders[key] = H.Coder(k, m, 0, lib=lib)
    return _coders[key]


@contextlib.contextmanager
def knobs(pairs, xlib=None):
    """hec_tune_set pairs on the measurement build for the duration of a
    block (the product library has no knobs: pairs must be empty there)."""
    assert not pairs or xlib is not None, "knobs exist only in the measurement build"
    try:
        for key, val in pairs:
            H.tune_set(key, val, xlib)
        yield
    finally:
        for key, _ in pairs:
            H.tune_set(key, -1 if key == 2 else 0, xlib)


def oracle_batch_encode(c_oracle, k, m, data: np.ndarray) -> np.ndarray:
    S, _, n = data.shape
    par = np.empty((S, m, n), dtype=np.uint8)
    d = np.ascontiguousarray(data)
    assert c_oracle.orc_encode_batch(k, m, d.ctypes.data, n, S, par.ctypes.data) == 0
    return par


# ---- host-buffer API (Coder::encode / Coder::decode drop-ins) ------------

def test_host_encode_matches_golden(golden):
    manifest, arrays = golden
    for case in manifest["cases"]:
        k, m, key = case["k"], case["m"], case["key"]
        data = arrays[key + "_data"]
        want = arrays[key + "_parity"]
        got = coder(k, m).encode([bytes(d) for d in data])
        for j in range(m):
            assert got[j] == want[j].tobytes(), (key, j)


def test_host_decode_golden_all_patterns(golden):
    manifest, arrays = golden
    for k, m in [(3, 2), (6, 3), (10, 4)]:
        for n in (17, 4096):
            key = f"rs{k}_{m}_n{n}"
            data, par = arrays[key + "_data"], arrays[key + "_parity"]
            full = [bytes(x) for x in data] + [bytes(x) for x in par]
            for e in range(1, m + 1):
                for miss in itertools.combinations(range(k + m), e):
                    shards = [None if i in miss else full[i] for i in range(k + m)]
                    coder(k, m).decode(shards)
                    for i in range(k):
                        assert shards[i] == full[i], (key, miss, i)
                    for i in range(k, k + m):  # parity never regenerated
                        assert (shards[i] is None) == (i in miss)


@pytest.fixture(scope="module")
def dev_coder():
    """Coders with host_limit = 0: every hec_encode / hec_decode call runs the
    HIP kernels, whatever the row length (the default routes rows of at most
    256 KiB per shard to the host routine, which would bypass the device)."""
    made = {}

    def get(k, m):
        if (k, m) not in made:
            c = H.Coder(k, m, 0)
            c.host_limit = 0
            assert c.host_limit == 0
            made[(k, m)] = c
        return made[(k, m)]

    yield get
    for c in made.values():
        c.close()


def test_device_encode_matches_golden(golden, dev_coder):
    """Every committed fixture (lengths 1 .. 4096 and the reference bench's
    counter fill, rust/benches/ec.rs:19-27) through the device kernels, per
    row (hec_encode with host_limit 0), byte for byte against `_parity`."""
    manifest, arrays = golden
    for case in manifest["cases"]:
        k, m, key = case["k"], case["m"], case["key"]
        data = arrays[key + "_data"]
        want = arrays[key + "_parity"]
        got = dev_coder(k, m).encode([bytes(d) for d in data])
        for j in range(m):
            assert got[j] == want[j].tobytes(), (key, j)


def test_device_decode_golden_all_patterns(golden, dev_coder):
    """gf256.rs:84-137 on the device: every erasure pattern of 1..m shards
    over the committed fixtures, rebuilt data == the fixture's data."""
    manifest, arrays = golden
    for case in manifest["cases"]:
        k, m, key = case["k"], case["m"], case["key"]
        data, par = arrays[key + "_data"], arrays[key + "_parity"]
        full = [bytes(x) for x in data] + [bytes(x) for x in par]
        for e in range(1, m + 1):
            for miss in itertools.combinations(range(k + m), e):
                shards = [None if i in miss else full[i] for i in range(k + m)]
                dev_coder(k, m).decode(shards)
                for i in range(k):
                    assert shards[i] == full[i], (key, miss, i)


def test_device_batch_golden(golden, dev, c_oracle):
    """The batched device-resident calls over the fixtures: each case's row
    replicated into a 3-stripe batch (stripe s XORed with s so the stripes
    differ; parity of stripe s = golden parity XOR encode(s-fill), linear),
    encode_batch parity == fixture parity for stripe 0, and decode_batch of
    every data-loss pattern rebuilds the fixture's data."""
    manifest, arrays = golden
    for case in manifest["cases"]:
        k, m, key = case["k"], case["m"], case["key"]
        data, par = arrays[key + "_data"], arrays[key + "_parity"]
        n = data.shape[1]
        batch = np.stack([data ^ np.uint8(s) for s in range(3)])
        d = torch.from_numpy(np.ascontiguousarray(batch)).to(dev)
        p = torch.empty((3, m, n), dtype=torch.uint8, device=dev)
        H.encode_batch(coder(k, m), d, p)
        torch.cuda.synchronize()
        got = p.cpu().numpy()
        assert np.array_equal(got[0], par), key
        want = oracle_batch_encode(c_oracle, k, m, batch)
        assert np.array_equal(got, want), key
        for e in range(1, m + 1):
            for miss in itertools.combinations(range(k), e):
                out = torch.zeros_like(d)
                H.decode_batch(coder(k, m), d, p, list(miss), out)
                torch.cuda.synchronize()
                o = out.cpu().numpy()
                for i in miss:
                    assert np.array_equal(o[0, i], data[i]), (key, miss, i)
                    assert np.array_equal(o[:, i], batch[:, i]), (key, miss, i)


def test_host_decode_too_many_failures():
    # test_ec.rs:116-121: m+1 failures must error
    k, m, n = 6, 3, 64
    data = [splitmix64_bytes(9 + i, n).tobytes() for i in range(k)]
    par = coder(k, m).encode(data)
    shards = [None] * (m + 1) + (data + par)[m + 1:]
    with pytest.raises(H.ErasureCodingError):
        coder(k, m).decode(shards)


def test_host_decode_nothing_missing_is_noop():
    k, m = 3, 2
    data = [b"abc", b"def", b"ghi"]
    shards = data + [None, None]
    coder(k, m).decode(shards)
    assert shards == data + [None, None]


def test_host_encode_reference_bench_fill(c_oracle):
    # rust/benches/ec.rs:16-33 at 1 MiB slices (the bench uses 16 MiB)
    k, m, n = 6, 3, 1 << 20
    data = bench_counter_shards(k, n)
    got = coder(k, m).encode([d.tobytes() for d in data])
    want = O.c_encode(c_oracle, k, m, list(data))
    assert all(g == w.tobytes() for g, w in zip(got, want))


@pytest.mark.parametrize("n", [1, 4, 15, 16, 17, 1000, 4093, (1 << 20) - 4, (1 << 20) + 4])
def test_host_encode_odd_lengths(c_oracle, n):
    k, m = 3, 2
    data = [splitmix64_bytes(100 + i + n, n) for i in range(k)]
    got = coder(k, m).encode([d.tobytes() for d in data])
    want = O.c_encode(c_oracle, k, m, data)
    assert all(g == w.tobytes() for g, w in zip(got, want))


def test_host_encode_edge_fills(c_oracle):
    for fill in (0x00, 0xFF, 0x01, 0x80):
        for k, m in [(3, 2), (6, 3), (10, 4)]:
            data = [np.full(4096, fill, dtype=np.uint8) for _ in range(k)]
            got = coder(k, m).encode([d.tobytes() for d in data])
            want = O.c_encode(c_oracle, k, m, data)
            assert all(g == w.tobytes() for g, w in zip(got, want))


# ---- device-resident batched API --------------------------------------

@pytest.mark.parametrize("k,m", [(3, 2), (6, 3), (10, 4), (2, 1), (5, 3), (12, 4), (4, 8), (32, 16), (1, 1)])
@pytest.mark.parametrize("cell", [4096, 4093, 48, 7])
def test_device_encode_batch_vs_oracle(dev, c_oracle, k, m, cell):
    S = 6
    data = batch_data(S, k, cell, first=k * 100 + cell)
    want = oracle_batch_encode(c_oracle, k, m, data)
    d = torch.from_numpy(data).to(dev)
    p = torch.full((S, m, cell), 0xA5, dtype=torch.uint8, device=dev)
    H.encode_batch(coder(k, m), d, p)
    torch.cuda.synchronize()
    assert np.array_equal(p.cpu().numpy(), want)


@pytest.mark.parametrize("k,m", [(3, 2), (6, 3), (10, 4)])
def test_device_decode_batch_all_data_patterns(dev, c_oracle, k, m):
    S, cell = 4, 4096 + 16
    data = batch_data(S, k, cell, first=7)
    par = oracle_batch_encode(c_oracle, k, m, data)
    d = torch.from_numpy(data).to(dev)
    p = torch.from_numpy(par).to(dev)
    # every data-loss pattern (385 for RS(10,4))
    pats = [c for e in range(1, m + 1) for c in itertools.combinations(range(k), e)]
    for miss in pats:
        out = torch.zeros_like(d)
        H.decode_batch(coder(k, m), d, p, miss, out)
        torch.cuda.synchronize()
        o = out.cpu().numpy()
        for i in range(k):
            if i in miss:
                assert np.array_equal(o[:, i], data[:, i]), (miss, i)
            else:
                assert not o[:, i].any()  # untouched


def test_device_decode_parity_survivor_mix(dev, c_oracle):
    # survivors are the first k present: missing {1, 7} in RS(6,3) uses
    # data 0,2,3,4,5 + parity 6
    k, m, S, cell = 6, 3, 3, 1024
    data = batch_data(S, k, cell, first=3)
    par = oracle_batch_encode(c_oracle, k, m, data)
    d = torch.from_numpy(data).to(dev)
    p = torch.from_numpy(par).to(dev)
    p[:, 1] = 0  # parity index 7 "missing" -- must not be read
    dp, ds = H.stripe_layout_ptrs(d, k)
    pp, ps = H.stripe_layout_ptrs(p, m)
    out = torch.zeros_like(d)
    op, os_ = H.stripe_layout_ptrs(out, k)
    ptrs = [dp[0], None, dp[2], dp[3], dp[4], dp[5], pp[0], None, pp[2]]
    coder(k, m).decode_device(ptrs, ds + ps, op, os_, cell, S, torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    assert np.array_equal(out[:, 1].cpu().numpy(), data[:, 1])


def test_device_not_enough_shards(dev):
    k, m = 6, 3
    d = torch.zeros((1, k, 64), dtype=torch.uint8, device=dev)
    p = torch.zeros((1, m, 64), dtype=torch.uint8, device=dev)
    out = torch.zeros_like(d)
    with pytest.raises(H.ErasureCodingError):
        H.decode_batch(coder(k, m), d, p, [0, 1, 2, 3], out)


def test_device_unaligned_layout(dev, c_oracle):
    # shard bases off 16-B alignment -> byte kernel; results identical
    k, m, S, cell = 6, 3, 3, 1000
    data = batch_data(S, k, cell, first=11)
    want = oracle_batch_encode(c_oracle, k, m, data)
    buf = torch.zeros(S * k * cell + 1, dtype=torch.uint8, device=dev)
    buf[1:] = torch.from_numpy(data.ravel()).to(dev)
    pbuf = torch.zeros(S * m * cell + 3, dtype=torch.uint8, device=dev)
    base, pbase = buf.data_ptr() + 1, pbuf.data_ptr() + 3
    coder(k, m).encode_device([base + i * cell for i in range(k)], [k * cell] * k,
                              [pbase + j * cell for j in range(m)], [m * cell] * m, cell, S,
                              torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    got = pbuf[3:].cpu().numpy().reshape(S, m, cell)
    assert np.array_equal(got, want)


@pytest.mark.parametrize("k,m,S,cell,in_off,out_off,pitch_extra,per_shard", [
    (6, 3, 3, 1000, 1, 3, 0, False), (6, 3, 2, 4096 + 7, 5, 0, 12, False), (6, 3, 2, 65536 + 5, 0, 2, 4, False),
    (10, 4, 2, 8192 + 5, 3, 1, 0, True), (3, 2, 4, 4096, 2, 6, 2, True), (3, 2, 3, 7, 1, 1, 0, False),
    (2, 1, 3, 24, 7, 5, 1, True)])
def test_device_unaligned_layouts(dev, c_oracle, k, m, S, cell, in_off, out_off, pitch_extra, per_shard):
    """Bases and strides off the 16-B grid: the dword-realigning kernel (8 B
    per lane, aligned dword loads + v_alignbyte, dword / short / byte stores
    by output alignment) plus the byte tail; encode and a decode with m data
    shards missing vs the oracle (the measurement build also runs the byte
    kernel alone, tests/test_gpu_experimental.py)."""
    unaligned_layouts_body(dev, c_oracle, k, m, S, cell, in_off, out_off, pitch_extra, per_shard, coder(k, m))


UNALIGNED_CASES = [
    (6, 3, 3, 1000, 1, 3, 0, False), (6, 3, 2, 4096 + 7, 5, 0, 12, False), (6, 3, 2, 65536 + 5, 0, 2, 4, False),
    (10, 4, 2, 8192 + 5, 3, 1, 0, True), (3, 2, 4, 4096, 2, 6, 2, True), (3, 2, 3, 7, 1, 1, 0, False),
    (2, 1, 3, 24, 7, 5, 1, True)]


def unaligned_layouts_body(dev, c_oracle, k, m, S, cell, in_off, out_off, pitch_extra, per_shard, cod):
    data = batch_data(S, k, cell, first=13 + cell + in_off)
    want = oracle_batch_encode(c_oracle, k, m, data)
    pitch = cell + pitch_extra
    shard_off = [in_off + (3 * i + 1 if per_shard else 0) for i in range(k)]
    in_stride = k * pitch + (3 * k + 16 if per_shard else 0)  # per-shard offsets need room between stripes
    span = S * in_stride + max(shard_off) + 16
    buf = torch.zeros(span, dtype=torch.uint8, device=dev)
    hbuf = np.zeros(span, dtype=np.uint8)
    for s_ in range(S):
        for i in range(k):
            at = shard_off[i] + i * pitch + s_ * in_stride
            hbuf[at:at + cell] = data[s_, i]
    buf.copy_(torch.from_numpy(hbuf))
    ip = [buf.data_ptr() + shard_off[i] + i * pitch for i in range(k)]
    pbuf = torch.zeros(S * m * pitch + out_off + 16, dtype=torch.uint8, device=dev)
    op = [pbuf.data_ptr() + out_off + j * pitch for j in range(m)]
    sp = torch.cuda.current_stream().cuda_stream
    if True:
        cod.encode_device(ip, [in_stride] * k, op, [m * pitch] * m, cell, S, sp)
        torch.cuda.synchronize()
        hp = pbuf.cpu().numpy()
        got = np.stack([np.stack([hp[out_off + (s_ * m + j) * pitch:][:cell] for j in range(m)]) for s_ in range(S)])
        assert np.array_equal(got, want)
        # decode: data shards 0..m-1 missing, rebuilt into an unaligned buffer
        miss = list(range(min(m, k)))
        rbuf = torch.zeros(S * k * pitch + out_off + 16, dtype=torch.uint8, device=dev)
        shards = [None if i in miss else ip[i] for i in range(k)] + op
        outs = [rbuf.data_ptr() + out_off + i * pitch if i in miss else 0 for i in range(k)]
        cod.decode_device(shards, [in_stride] * k + [m * pitch] * m, outs, [k * pitch] * k, cell, S, sp)
        torch.cuda.synchronize()
        hr = rbuf.cpu().numpy()
        for s_ in range(S):
            for i in miss:
                assert np.array_equal(hr[out_off + (s_ * k + i) * pitch:][:cell], data[s_, i]), (s_, i)


def test_gf_matmul_device_arbitrary_matrix(dev):
    # the raw Mul<&[&[u8]]> (matrix.rs:204-231) with a random 7x5 matrix
    rng = np.random.default_rng(3)
    mat = rng.integers(0, 256, size=(7, 5)).tolist()
    S, cell = 2, 4096 + 48
    data = batch_data(S, 5, cell, first=1)
    d = torch.from_numpy(data).to(dev)
    out = torch.zeros((S, 7, cell), dtype=torch.uint8, device=dev)
    ip, is_ = H.stripe_layout_ptrs(d, 5)
    op, os_ = H.stripe_layout_ptrs(out, 7)
    coder(3, 2).gf_matmul_device(mat, ip, is_, op, os_, cell, S, torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    o = out.cpu().numpy()
    for s in range(S):
        want = O.matmul_shards(mat, list(data[s]))
        for j in range(7):
            assert np.array_equal(o[s, j], want[j])


@pytest.mark.parametrize("k,m", [(2, 1), (3, 2), (6, 3), (10, 4)])
@pytest.mark.parametrize("cell", [4096, 4096 + 16, 3 * 65536 + 48, (1 << 18) + 48, 5 * 65536 + 16])
@pytest.mark.parametrize("S", [3, 6, 7])
def test_pipelines_vs_oracle(dev, c_oracle, k, m, cell, S):
    """The default kernels by cell size: the LDS-DMA kernel (cells <= 256 KiB,
    k in {2, 3, 6}) and the register kernel (larger cells, and k = 10), full
    and partial tiles; S = 3, 6 and 7 stripes: tile-order groups of 3 and 2,
    and 7 = a group of 4 plus a stripe-major remainder of 3."""
    pipelines_body(dev, c_oracle, k, m, cell, S, coder(k, m))


def pipelines_body(dev, c_oracle, k, m, cell, S, cod):
    data = batch_data(S, k, cell, first=cell + k)
    want = oracle_batch_encode(c_oracle, k, m, data)
    d = torch.from_numpy(data).to(dev)
    p = torch.zeros((S, m, cell), dtype=torch.uint8, device=dev)
    H.encode_batch(cod, d, p)
    out = torch.zeros_like(d)
    H.decode_batch(cod, d, p, list(range(m)), out)
    torch.cuda.synchronize()
    assert np.array_equal(p.cpu().numpy(), want)
    assert torch.equal(out[:, :m], d[:, :m])


@pytest.mark.parametrize("S,chunk,cell", [(9, 4, 65536), (23, 2, 65536), (7, 7, 4096 + 16), (5, 1, 1000)])
def test_encode_host_batch_pinned(c_oracle, S, chunk, cell):
    # more chunks than device slots, partial last chunk, tails
    k, m = 6, 3
    data = batch_data(S, k, cell, first=40)
    want = oracle_batch_encode(c_oracle, k, m, data)
    h_in = torch.from_numpy(data).pin_memory()
    h_out = torch.zeros((S, m, cell), dtype=torch.uint8).pin_memory()
    for _ in range(2):  # second pass reuses the slots/events
        coder(k, m).encode_host_batch(h_in.data_ptr(), h_out.data_ptr(), cell, S, chunk)
        assert np.array_equal(h_out.numpy(), want)
        h_out.zero_()


# ---- full-size configs (BASELINE.json) via size-independent properties ---

def _device_random(shape, dev, seed):
    g = torch.Generator(device=dev)
    g.manual_seed(seed)
    return torch.randint(0, 256, shape, dtype=torch.uint8, device=dev, generator=g)


@pytest.mark.parametrize("k,m,cell,S", [(6, 3, 1 << 20, 64), (10, 4, 1 << 20, 32), (6, 3, 1 << 16, 2048),
                                        (3, 2, 1 << 20, 64)])
def test_full_size_roundtrip_and_oracle(dev, c_oracle, k, m, cell, S):
    d = _device_random((S, k, cell), dev, seed=k * 1000 + S)
    p = torch.empty((S, m, cell), dtype=torch.uint8, device=dev)
    H.encode_batch(coder(k, m), d, p)
    # worst case: the first m data shards missing
    miss = list(range(m))
    out = torch.zeros_like(d)
    H.decode_batch(coder(k, m), d, p, miss, out)
    torch.cuda.synchronize()
    assert torch.equal(out[:, :m], d[:, :m])
    # every stripe's parity and rebuilt cells against the C oracle
    # (stripe-parallel on the box's CPU share)
    present = ((1 << (k + m)) - 1) & ~sum(1 << i for i in miss)
    O.c_check_batch(c_oracle, k, m, d.cpu().numpy(), p.cpu().numpy(), present,
                    np.ascontiguousarray(out[:, :m].cpu().numpy()), threads=_cpu_share())


def test_work_queue_counters_reset_across_launches(dev, c_oracle):
    """The register kernel deals wave-tiles from per-stream launch counters
    (ec_kernels.hip queue_lease: two sets per stream, each launch zeroes the
    next launch's): launches of different tile counts back to back on one
    stream (fewer tiles than counters, fewer than CUs, many), then three
    streams at once -- a counter not zero at a launch's start would skip
    tiles of that launch."""
    k, m = 6, 3
    cod = coder(k, m)
    for S, cell in [(1, 1 << 20), (3, 1 << 20), (1, 4096), (200, 1 << 20), (5, 8192 + 16), (64, 1 << 20)]:
        d = _device_random((S, k, cell), dev, seed=S * 7 + cell)
        p = torch.empty((S, m, cell), dtype=torch.uint8, device=dev)
        H.encode_batch(cod, d, p)
        out = torch.zeros_like(d)
        H.decode_batch(cod, d, p, [0, 1, 2], out)
        torch.cuda.synchronize()
        assert torch.equal(out[:, :3], d[:, :3]), (S, cell)
        O.c_check_batch(c_oracle, k, m, d[:2].cpu().numpy(), p[:2].cpu().numpy(), threads=1)
    streams = [torch.cuda.Stream() for _ in range(3)]
    S, cell = 96, 1 << 20
    ds = [_device_random((S, k, cell), dev, seed=50 + i) for i in range(3)]
    ps = [torch.empty((S, m, cell), dtype=torch.uint8, device=dev) for _ in range(3)]
    want = [torch.empty_like(x) for x in ps]
    for i in range(3):
        H.encode_batch(cod, ds[i], want[i])
    torch.cuda.synchronize()
    for rep in range(3):
        for i, st in enumerate(streams):
            H.encode_batch(cod, ds[i], ps[i], st)
        torch.cuda.synchronize()
        for i in range(3):
            assert torch.equal(ps[i], want[i]), (rep, i)


def test_work_queue_per_thread_default_stream(dev):
    """hipStreamPerThread ((hipStream_t)2) is a different stream in every
    thread: the work-queue counter sets are keyed by hipStreamGetId, which
    resolves the handle to the thread's own stream, so threads encoding at
    once on that handle never share a counter set."""
    import threading
    k, m, S, cell = 6, 3, 48, 1 << 20
    ds = [_device_random((S, k, cell), dev, seed=70 + i) for i in range(4)]
    want = []
    for d in ds:
        p = torch.empty((S, m, cell), dtype=torch.uint8, device=dev)
        H.encode_batch(coder(k, m), d, p)
        want.append(p)
    torch.cuda.synchronize()
    errors = []

    def work(i):
        try:
            c = H.Coder(k, m, 0)
            dp, dst = H.stripe_layout_ptrs(ds[i], k)
            for _ in range(4):
                p = torch.zeros((S, m, cell), dtype=torch.uint8, device=dev)
                torch.cuda.synchronize()
                pp, pst = H.stripe_layout_ptrs(p, m)
                c.encode_device(dp, dst, pp, pst, cell, S, 2)  # hipStreamPerThread
                torch.cuda.synchronize()  # every stream of the device, this thread's included
                if not torch.equal(p, want[i]):
                    errors.append(i)
            c.close()
        except Exception as e:  # noqa: BLE001
            errors.append(repr(e))

    ts = [threading.Thread(target=work, args=(i,)) for i in range(4)]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    assert not errors, errors


SENTINEL = 0xA5


@pytest.mark.parametrize("k,m", [(2, 1), (3, 2), (6, 3), (10, 4)])
@pytest.mark.parametrize("cell", [8192 + 16, 3 * 65536 + 48])
def test_work_queue_kernels_back_to_back_sentinel(dev, c_oracle, k, m, cell):
    """Every work-queue kernel of the product, back to back on ONE stream,
    over batches of 3, 1 and 40 stripes whose cells end in partial wave-
    tiles (8208 B: RS(2,1) x 3 stripes is the r05u/r05v failure, DESIGN.md
    §3.1): the plain encode (gf_matmul_v16), the fused encode + CRC (the
    queue at k = 3 and 10), the plan-specialised decode + verify (the queue
    at every k) and the plain decode.  Every output starts as a sentinel
    byte, so a tile the queue never dealt shows up; parity, sums and the
    rebuilt shards are checked against the oracle."""
    bpc = 512
    cod = H.Coder(k, m, 0)
    lost = list(range(min(m, k)))
    assert cod.prepare_decode(lost, H.CHECKSUM_CRC32C), "hiprtc unavailable on the GPU box"
    st = torch.cuda.Stream()
    with torch.cuda.stream(st):
        for rep, S in enumerate([3, 1, 40, 3]):
            data = batch_data(S, k, cell, first=cell + 13 * S + rep)
            par = oracle_batch_encode(c_oracle, k, m, data)
            nch = (cell + bpc - 1) // bpc
            edge = [0, S - 1] if S > 1 else [0]  # the Python CRC oracle is slow: first and last stripe
            want_sums = _oracle_sums(np.concatenate([data[edge], par[edge]], axis=1), bpc)
            d = torch.from_numpy(data).to(dev)
            # plain encode
            p = torch.full((S, m, cell), SENTINEL, dtype=torch.uint8, device=dev)
            H.encode_batch(cod, d, p, st)
            # fused encode + CRC
            p2 = torch.full((S, m, cell), SENTINEL, dtype=torch.uint8, device=dev)
            sums = torch.full((S, k + m, nch, 4), SENTINEL, dtype=torch.uint8, device=dev)
            dp, ds = H.stripe_layout_ptrs(d, k)
            pp, ps = H.stripe_layout_ptrs(p2, m)
            cod.encode_crc_device(dp, ds, pp, ps, cell, S, bpc, sums.data_ptr(), st.cuda_stream)
            # decode + verify (specialised), data shards `lost` missing
            out = torch.full((S, k, cell), SENTINEL, dtype=torch.uint8, device=dev)
            bad = torch.full((S, k + m), 7, dtype=torch.uint8, device=dev)
            ptrs = [None if i in lost else dp[i] for i in range(k)] + pp
            op, os_ = H.stripe_layout_ptrs(out, k)
            before = H.jit_stats()["launches"]
            cod.decode_verify_device(H.CHECKSUM_CRC32C, ptrs, ds + ps, op, os_, cell, S, bpc,
                                     sums.data_ptr(), bad.data_ptr(), st.cuda_stream)
            # plain decode of the same shards
            out2 = torch.full((S, k, cell), SENTINEL, dtype=torch.uint8, device=dev)
            H.decode_batch(cod, d, p2, lost, out2, st)
            # every stripe's sums against the fixed-order CRC kernel (another kernel)
            ref = H.crc32c_batch(cod, torch.cat([d, torch.from_numpy(par).to(dev)], dim=1), bpc, st)
            st.synchronize()
            assert H.jit_stats()["launches"] > before
            assert np.array_equal(p.cpu().numpy(), par), (rep, S)
            assert np.array_equal(p2.cpu().numpy(), par), (rep, S)
            assert np.array_equal(sums.cpu().numpy()[edge], want_sums), (rep, S)
            assert torch.equal(sums, ref), (rep, S)
            assert not bad.cpu().numpy().any(), (rep, S)
            for o in (out, out2):
                on = o.cpu().numpy()
                assert np.array_equal(on[:, lost], data[:, lost]), (rep, S)
                assert (on[:, len(lost):] == SENTINEL).all(), (rep, S)  # present shards never written
    cod.close()


def _hip_runtime():
    """torch's libamdhip64 (the one HIP runtime of the process)."""
    import ctypes
    with open("/proc/self/maps") as f:
        for line in f:
            if "libamdhip64" in line:
                return ctypes.CDLL(line.split()[-1])
    raise RuntimeError("libamdhip64 not mapped")


def test_work_queue_stream_churn(dev, c_oracle):
    """Streams created and destroyed one after another (HIP hands the same
    handle out again): every encode / decode on the fresh streams is exact.
    With hipStreamGetId in the process each new stream gets sets of its own
    (the set count grows by one per stream); without it (the HIP a torch
    wheel bundles) a reused handle inherits its destroyed stream's sets,
    whose last launch hipStreamDestroy has waited for."""
    import ctypes
    hip = _hip_runtime()
    k, m, S, cell = 6, 3, 5, 8192 + 16
    cod = coder(k, m)
    data = batch_data(S, k, cell, first=4242)
    par = oracle_batch_encode(c_oracle, k, m, data)
    d = torch.from_numpy(data).to(dev)
    torch.cuda.synchronize()
    before = H.queue_stats(0)["streams"]
    handles = set()
    n = 40
    for i in range(n):
        s = ctypes.c_void_p()
        assert hip.hipStreamCreateWithFlags(ctypes.byref(s), 1) == 0  # hipStreamNonBlocking
        handles.add(s.value)
        p = torch.full((S, m, cell), SENTINEL, dtype=torch.uint8, device=dev)
        out = torch.full((S, k, cell), SENTINEL, dtype=torch.uint8, device=dev)
        torch.cuda.synchronize()
        dp, ds = H.stripe_layout_ptrs(d, k)
        pp, ps = H.stripe_layout_ptrs(p, m)
        cod.encode_device(dp, ds, pp, ps, cell, S, s.value)
        op, os_ = H.stripe_layout_ptrs(out, k)
        ptrs = [None, None, None] + dp[3:] + pp
        cod.decode_device(ptrs, ds + ps, op, os_, cell, S, s.value)
        assert hip.hipStreamSynchronize(s) == 0
        assert hip.hipStreamDestroy(s) == 0
        assert np.array_equal(p.cpu().numpy(), par), i
        assert np.array_equal(out[:, :3].cpu().numpy(), data[:, :3]), i
    grown = H.queue_stats(0)["streams"] - before
    if H.queue_stats(0)["keyed_by_id"]:
        assert grown == n, (grown, len(handles))
    else:  # handles the library saw before (destroyed coders' streams) may come back too
        assert grown <= len(handles), (grown, len(handles))


def test_work_queue_one_stream_two_threads(dev):
    """Two threads enqueue encodes on the SAME stream at once: the lease holds
    the stream's sets from choosing a set to enqueuing the kernel, so the
    launches alternate sets in their stream order and every output is exact."""
    import threading
    k, m, S, cell = 6, 3, 7, 3 * 65536 + 48
    cod = coder(k, m)
    ds = [_device_random((S, k, cell), dev, seed=90 + i) for i in range(2)]
    want = []
    for d in ds:
        p = torch.empty((S, m, cell), dtype=torch.uint8, device=dev)
        H.encode_batch(cod, d, p)
        want.append(p)
    torch.cuda.synchronize()
    st = torch.cuda.Stream()
    outs = [[torch.full((S, m, cell), SENTINEL, dtype=torch.uint8, device=dev) for _ in range(16)]
            for _ in range(2)]
    torch.cuda.synchronize()
    errors = []

    def work(i):
        try:
            c = H.Coder(k, m, 0)
            dp, dst = H.stripe_layout_ptrs(ds[i], k)
            for p in outs[i]:
                pp, pst = H.stripe_layout_ptrs(p, m)
                c.encode_device(dp, dst, pp, pst, cell, S, st.cuda_stream)
            st.synchronize()
            c.close()
        except Exception as e:  # noqa: BLE001
            errors.append(repr(e))

    ts = [threading.Thread(target=work, args=(i,)) for i in range(2)]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    assert not errors, errors
    for i in range(2):
        for j, p in enumerate(outs[i]):
            assert torch.equal(p, want[i]), (i, j)


def test_work_queue_graph_capture_replay(dev, c_oracle):
    """torch.cuda.graph (global capture mode) around an encode and a decode:
    the captured launches take graph counter sets of their own, zeroed by a
    memset node at every replay.  Replays on the capture stream between
    direct launches there, and on a second stream while the first runs
    direct launches, are all exact against the oracle."""
    k, m, S, cell = 6, 3, 6, 65536 + 48
    cod = H.Coder(k, m, 0)
    d_s = torch.zeros((S, k, cell), dtype=torch.uint8, device=dev)
    p_s = torch.zeros((S, m, cell), dtype=torch.uint8, device=dev)
    o_s = torch.zeros((S, k, cell), dtype=torch.uint8, device=dev)
    # warm-up outside the capture (first use of the capture stream's sets is
    # not needed: captured launches never touch them)
    torch.cuda.synchronize()
    g0 = H.queue_stats(0)["graph_sets"]
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        H.encode_batch(cod, d_s, p_s)
        H.decode_batch(cod, d_s, p_s, [0, 1, 2], o_s)
    assert H.queue_stats(0)["graph_sets"] - g0 == 2  # both launches took the work queue
    other = torch.cuda.Stream()
    d2 = _device_random((40, k, cell), dev, seed=11)
    p2 = torch.empty((40, m, cell), dtype=torch.uint8, device=dev)
    for rep in range(6):
        data = batch_data(S, k, cell, first=rep * 7 + 1)
        par = oracle_batch_encode(c_oracle, k, m, data)
        d_s.copy_(torch.from_numpy(data))
        p_s.fill_(SENTINEL)
        o_s.fill_(SENTINEL)
        torch.cuda.synchronize()
        if rep % 2 == 0:
            H.encode_batch(cod, d2, p2)     # direct launches on the current stream
            g.replay()                      # ... the graph between them
            H.encode_batch(cod, d2, p2)
        else:
            with torch.cuda.stream(other):
                g.replay()                  # the graph on another stream
            H.encode_batch(cod, d2, p2)     # while the current stream runs direct launches
            H.encode_batch(cod, d2, p2)
        torch.cuda.synchronize()
        assert np.array_equal(p_s.cpu().numpy(), par), rep
        assert torch.equal(o_s[:, :3], d_s[:, :3]), rep
    O.c_check_batch(c_oracle, k, m, d2[:3].cpu().numpy(), p2[:3].cpu().numpy(), threads=1)
    del g
    cod.close()


def test_linearity(dev):
    k, m, S, cell = 6, 3, 16, 1 << 18
    a = _device_random((S, k, cell), dev, 1)
    b = _device_random((S, k, cell), dev, 2)
    pa, pb, pab = (torch.empty((S, m, cell), dtype=torch.uint8, device=dev) for _ in range(3))
    H.encode_batch(coder(k, m), a, pa)
    H.encode_batch(coder(k, m), b, pb)
    H.encode_batch(coder(k, m), a ^ b, pab)
    torch.cuda.synchronize()
    assert torch.equal(pab, pa ^ pb)


def test_repeatable(dev):
    k, m, S, cell = 10, 4, 8, 1 << 20
    d = _device_random((S, k, cell), dev, 5)
    p1 = torch.empty((S, m, cell), dtype=torch.uint8, device=dev)
    p2 = torch.empty_like(p1)
    H.encode_batch(coder(k, m), d, p1)
    H.encode_batch(coder(k, m), d, p2)
    torch.cuda.synchronize()
    assert torch.equal(p1, p2)


# ---- heterogeneous per-stripe erasure patterns --------

def _random_masks(k, m, S, seed, allow_fail=False):
    rng = np.random.default_rng(seed)
    masks = []
    for s in range(S):
        n_missing = int(rng.integers(0, m + (2 if allow_fail else 1)))
        missing = rng.choice(k + m, size=n_missing, replace=False)
        mask = sum(1 << i for i in range(k + m) if i not in set(missing.tolist()))
        masks.append(mask)
    return masks


@pytest.mark.parametrize("k,m,cell", [(6, 3, 4096), (6, 3, 65536 + 64), (10, 4, 8192), (3, 2, 4096 + 16),
                                      (2, 1, 1024), (4, 2, 4096), (6, 3, 1000)])
def test_device_decode_mixed_patterns(dev, c_oracle, k, m, cell):
    """Random per-stripe patterns (rows past a stripe's erasure count skipped;
    the measurement build also runs them computed and dropped,
    tests/test_gpu_experimental.py)."""
    mixed_patterns_body(dev, c_oracle, k, m, cell, coder(k, m))


@pytest.mark.parametrize("k,m", [(6, 3), (10, 4)])
def test_device_decode_mixed_address_bit31(dev, c_oracle, k, m):
    """The mixed kernel moves each survivor's and output's base address from
    its LDS shard table into SGPRs (readfirstlane of both 32-bit halves).
    Data, parity and output live at addresses whose low word has bit 31 set
    (then clear), so a sign-extended low half cannot go unnoticed."""
    S, cell = 12, 4096
    data = batch_data(S, k, cell, first=4242 + k)
    par = oracle_batch_encode(c_oracle, k, m, data)
    masks = _random_masks(k, m, S, seed=77 + k)
    masks[0] = ((1 << (k + m)) - 1) & ~((1 << m) - 1)  # worst case: data 0..m-1
    need = S * (2 * k + m) * cell
    big = torch.empty((1 << 31) + need + (1 << 25), dtype=torch.uint8, device=dev)
    base = big.data_ptr()
    for bit31 in (1, 0):
        # first 4 KiB-aligned offset whose address has bit 31 == bit31
        off = 0
        while ((base + off) >> 31) & 1 != bit31:
            off += 1 << 24
        off += (-(base + off)) % 4096
        assert ((base + off) >> 31) & 1 == bit31 and ((base + off + need) >> 31) & 1 == bit31
        view = big[off:off + need]
        d = view[:S * k * cell].view(S, k, cell)
        p = view[S * k * cell:S * (k + m) * cell].view(S, m, cell)
        out = view[S * (k + m) * cell:].view(S, k, cell)
        d.copy_(torch.from_numpy(data))
        p.copy_(torch.from_numpy(par))
        out.fill_(0x5A)
        H.decode_batch_mixed(coder(k, m), d, p, masks, out)
        torch.cuda.synchronize()
        o = out.cpu().numpy()
        for s, mask in enumerate(masks):
            for i in range(k):
                if not (mask >> i) & 1:
                    assert np.array_equal(o[s, i], data[s, i]), (bit31, s, i)
    del big


def mixed_patterns_body(dev, c_oracle, k, m, cell, cod, knob_pairs=(), xlib=None):
    S = 40
    data = batch_data(S, k, cell, first=900 + k)
    par = oracle_batch_encode(c_oracle, k, m, data)
    masks = _random_masks(k, m, S, seed=k * 31 + cell)
    masks[0] = (1 << (k + m)) - 1          # nothing missing
    masks[1] = (1 << k) - 1                # only parity missing: no work
    masks[2] = ((1 << (k + m)) - 1) & ~((1 << m) - 1)  # worst case: data 0..m-1
    d = torch.from_numpy(data).to(dev)
    p = torch.from_numpy(par).to(dev)
    # scribble over the erased slots so a wrong survivor choice shows up
    for s, mask in enumerate(masks):
        for i in range(k + m):
            if not (mask >> i) & 1:
                (d[s, i] if i < k else p[s, i - k]).fill_(0xEE)
    out = torch.full_like(d, 0x5A)
    with knobs(knob_pairs, xlib):
        H.decode_batch_mixed(cod, d, p, masks, out)
        torch.cuda.synchronize()
    o = out.cpu().numpy()
    for s, mask in enumerate(masks):
        for i in range(k):
            if (mask >> i) & 1:
                assert (o[s, i] == 0x5A).all(), (s, i)  # untouched
            else:
                assert np.array_equal(o[s, i], data[s, i]), (s, i, bin(mask))


def test_device_decode_mixed_many_plans(dev):
    """RS(10,4), 512 stripes with random 1..4 erased shards: a few hundred
    distinct plans, more than the kernel keeps resident in LDS (the per-stripe
    restaging path)."""
    mixed_many_plans_body(dev, coder(10, 4))


def mixed_many_plans_body(dev, cod, knob_pairs=(), xlib=None, S=512):
    k, m, cell = 10, 4, 4096
    rng = np.random.default_rng(1234)
    data = rng.integers(0, 256, size=(S, k, cell), dtype=np.uint8)
    d = torch.from_numpy(data).to(dev)
    p = torch.empty((S, m, cell), dtype=torch.uint8, device=dev)
    H.encode_batch(cod, d, p)
    full = (1 << (k + m)) - 1
    masks = []
    for s in range(S):
        miss = rng.choice(k + m, size=int(rng.integers(1, m + 1)), replace=False)
        masks.append(full & ~sum(1 << int(i) for i in miss))
    dm = d.clone()
    pm = p.clone()
    for s, mask in enumerate(masks):
        for i in range(k + m):
            if not (mask >> i) & 1:
                (dm[s, i] if i < k else pm[s, i - k]).fill_(0xEE)
    out = torch.full_like(d, 0x5A)
    with knobs(knob_pairs, xlib):
        H.decode_batch_mixed(cod, dm, pm, masks, out)
        torch.cuda.synchronize()
    for s, mask in enumerate(masks):
        for i in range(k):
            if (mask >> i) & 1:
                assert bool((out[s, i] == 0x5A).all()), (s, i)
            else:
                assert torch.equal(out[s, i], d[s, i]), (s, i, bin(mask))


@pytest.mark.parametrize("S", [24, 160, 256])
def test_device_decode_mixed_plans_resident(dev, S):
    """RS(10,4) with random losses of any shards: a plan blob under 64 KiB of
    LDS (S = 24), and past 64 KiB but within the 156 KiB the launcher keeps
    resident with the dynamic-LDS attribute (S = 160, 256; 512 above restages
    per stripe)."""
    mixed_many_plans_body(dev, coder(10, 4), S=S)


def test_device_decode_mixed_resident_two_threads(dev):
    """Two threads share one RS(10,4) coder, each on its own stream, decoding
    mixed batches whose resident plan blobs need different dynamic-LDS sizes
    past 64 KiB (S = 160 and 256), three times over: the launcher sets the
    launch attribute to the resident ceiling, never to its own size, so one
    thread's setting cannot fail the other's launch."""
    import threading

    cod = coder(10, 4)
    errs = []

    def run(S):
        try:
            with torch.cuda.stream(torch.cuda.Stream(device=dev)):
                for _ in range(3):
                    mixed_many_plans_body(dev, cod, S=S)
        except Exception as e:  # noqa: BLE001 (re-raised below)
            errs.append(e)

    ts = [threading.Thread(target=run, args=(S,)) for S in (160, 256)]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    if errs:
        raise errs[0]


def test_device_decode_mixed_not_enough_shards_launches_nothing(dev):
    k, m, S, cell = 6, 3, 4, 4096
    d = torch.zeros((S, k, cell), dtype=torch.uint8, device=dev)
    p = torch.zeros((S, m, cell), dtype=torch.uint8, device=dev)
    full = (1 << 9) - 1
    masks = [full & ~1, full, full & ~0b1111, full]  # stripe 2 lost 4 shards
    out = torch.full_like(d, 7)
    with pytest.raises(H.ErasureCodingError):
        H.decode_batch_mixed(coder(k, m), d, p, masks, out)
    torch.cuda.synchronize()
    assert (out == 7).all()


def test_device_decode_mixed_matches_uniform_decode(dev, c_oracle):
    # same pattern on every stripe == hec_decode_device, at a full-size cell
    k, m, S, cell = 6, 3, 16, 1 << 20
    g = torch.Generator(device=dev)
    g.manual_seed(77)
    d = torch.randint(0, 256, (S, k, cell), dtype=torch.uint8, device=dev, generator=g)
    p = torch.empty((S, m, cell), dtype=torch.uint8, device=dev)
    H.encode_batch(coder(k, m), d, p)
    full = (1 << 9) - 1
    masks = [full & ~0b101 & ~(1 << 7)] * S  # data 0,2 and parity 7 missing
    o1 = torch.zeros_like(d)
    o2 = torch.zeros_like(d)
    H.decode_batch_mixed(coder(k, m), d, p, masks, o1)
    dp, ds = H.stripe_layout_ptrs(d, k)
    pp, ps = H.stripe_layout_ptrs(p, m)
    op, os_ = H.stripe_layout_ptrs(o2, k)
    ptrs = [None, dp[1], None, dp[3], dp[4], dp[5], pp[0], None, pp[2]]
    coder(k, m).decode_device(ptrs, ds + ps, op, os_, cell, S, torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    assert torch.equal(o1, o2)
    assert torch.equal(o1[:, 0], d[:, 0]) and torch.equal(o1[:, 2], d[:, 2])


@pytest.mark.parametrize("k,m,S", [(6, 3, 64), (10, 4, 32), (3, 2, 64)])
def test_device_decode_mixed_full_size_workspace_reuse(dev, c_oracle, k, m, S):
    """Full-size cells through the mixed decode's work queue (wave-tiles
    dealt by the launch counters the workspace upload zeroes): three calls in
    a row on ONE workspace with different patterns -- a counter left at its
    end value would skip every tile of the next call -- each checked against
    the original data, and the last call's stripe 0 against the oracle's
    decode."""
    cell = 1 << 20
    g = torch.Generator(device=dev)
    g.manual_seed(900 + k)
    d = torch.randint(0, 256, (S, k, cell), dtype=torch.uint8, device=dev, generator=g)
    p = torch.empty((S, m, cell), dtype=torch.uint8, device=dev)
    H.encode_batch(coder(k, m), d, p)
    ws = None
    full = (1 << (k + m)) - 1
    for call in range(3):
        masks = _random_masks(k, m, S, seed=31 * call + k)
        out = torch.full_like(d, 0x5A)
        ws = H.decode_batch_mixed(coder(k, m), d, p, masks, out, workspace=ws)
        torch.cuda.synchronize()
        lost = torch.tensor([[not (mk >> i) & 1 for i in range(k)] for mk in masks], device=dev)
        assert bool(((out == d) | ~lost[:, :, None]).all()), call
        assert bool(((out == 0x5A) | lost[:, :, None]).all()), call
    miss0 = [i for i in range(k + m) if not (masks[0] >> i) & 1]
    if any(i < k for i in miss0) and len(miss0) <= m:
        present = full & masks[0]
        d0 = d[:1].cpu().numpy()
        O.c_check_batch(c_oracle, k, m, d0, p[:1].cpu().numpy(), present,
                        np.ascontiguousarray(out[:1, [i for i in miss0 if i < k]].cpu().numpy()), threads=1)


# ---- rs-legacy codec (parity unpinned, see oracle) -----

@pytest.mark.parametrize("k,m", [(6, 3), (3, 2), (10, 4)])
def test_rs_legacy_codec_encode_decode(dev, k, m):
    cell, S = 8192 + 48, 6
    c = H.Coder(k, m, 0, codec="rs-legacy")
    data = batch_data(S, k, cell, first=7000 + k)
    d = torch.from_numpy(data).to(dev)
    p = torch.zeros((S, m, cell), dtype=torch.uint8, device=dev)
    H.encode_batch(c, d, p)
    torch.cuda.synchronize()
    got = p.cpu().numpy()
    for s in range(S):  # against Hadoop's long division (GaloisField.remainder)
        want = O.legacy_encode(k, m, list(data[s]))
        assert all(np.array_equal(got[s, j], want[j]) for j in range(m)), s
    # every data-erasure pattern of up to m shards (k = 10: a spread of them)
    pats = [lost for e in range(1, m + 1) for lost in itertools.combinations(range(k), e)]
    for lost in (pats if k <= 6 else pats[::7]):
        out = torch.zeros_like(d)
        H.decode_batch(c, d, p, list(lost), out)
        torch.cuda.synchronize()
        for i in lost:
            assert torch.equal(out[:, i], d[:, i]), lost
    # per-stripe patterns with parity shards missing too (other survivor sets)
    rng = np.random.default_rng(k)
    masks = []
    for s in range(S):
        lost = rng.choice(k + m, size=m, replace=False)
        masks.append(sum(1 << i for i in range(k + m) if i not in lost))
    out = torch.zeros_like(d)
    H.decode_batch_mixed(c, d, p, masks, out)
    torch.cuda.synchronize()
    for s, mask in enumerate(masks):
        for i in range(k):
            if not (mask >> i) & 1:
                assert torch.equal(out[s, i], d[s, i]), (s, i)
    # host API (Coder::decode shape)
    shards = [bytes(x) for x in data[0]] + [got[0, j].tobytes() for j in range(m)]
    shards[0] = None
    shards[k] = None
    c.decode(shards)
    assert shards[0] == data[0, 0].tobytes()


# ---- XOR-k-1 codec ------------------------------------

@pytest.mark.parametrize("k", [2, 3, 6])
def test_xor_codec_encode_decode(dev, k):
    cell, S = 4096 + 16, 5
    c = H.Coder(k, 1, 0, codec="xor")
    data = batch_data(S, k, cell, first=5000 + k)
    d = torch.from_numpy(data).to(dev)
    p = torch.zeros((S, 1, cell), dtype=torch.uint8, device=dev)
    H.encode_batch(c, d, p)
    torch.cuda.synchronize()
    want = np.bitwise_xor.reduce(data, axis=1)
    assert np.array_equal(p[:, 0].cpu().numpy(), want)
    for lost in range(k):
        out = torch.zeros_like(d)
        H.decode_batch(c, d, p, [lost], out)
        torch.cuda.synchronize()
        assert torch.equal(out[:, lost], d[:, lost])
    # host API too
    shards = [bytes(x) for x in data[0]] + [want[0].tobytes()]
    shards[1] = None
    c.decode(shards)
    assert shards[1] == data[0, 1].tobytes()
    c.close()


# ---- fused striping: vertical shard buffers -> file-order rows (§8f row 2) -

@pytest.mark.parametrize("k,m,lost", [(6, 3, (0, 1, 2)), (6, 3, (4, 7)), (3, 2, ()), (10, 4, (1, 5, 9, 12)),
                                      (3, 2, (2, 3))])
@pytest.mark.parametrize("rows,chunk,cell", [(7, 2, 65536), (5, 5, 4096 + 16), (9, 4, 1000)])
def test_decode_host_batch_file_order(c_oracle, k, m, lost, rows, chunk, cell):
    # file bytes striped into rows of k cells (CellBuffer::write), parity per
    # row, then the reader's vertical buffers: shard i = its cells in row order
    file = splitmix64_bytes(rows * 1000 + k, rows * k * cell)
    data = file.reshape(rows, k, cell)
    par = oracle_batch_encode(c_oracle, k, m, data)
    vertical = [np.ascontiguousarray(data[:, i, :]).ravel() for i in range(k)] + \
               [np.ascontiguousarray(par[:, j, :]).ravel() for j in range(m)]
    hv = [None if i in lost else torch.from_numpy(vertical[i]).pin_memory() for i in range(k + m)]
    out = torch.zeros(rows * k * cell, dtype=torch.uint8).pin_memory()
    coder(k, m).decode_host_batch([None if t is None else t.data_ptr() for t in hv], cell, rows, out.data_ptr(),
                                  chunk)
    assert np.array_equal(out.numpy(), file)


def test_decode_host_batch_too_many_losses():
    k, m, cell, rows = 6, 3, 4096, 2
    hv = [torch.zeros(rows * cell, dtype=torch.uint8).pin_memory() for _ in range(k + m)]
    ptrs = [t.data_ptr() for t in hv]
    for i in (0, 1, 2, 3):
        ptrs[i] = None
    out = torch.zeros(rows * k * cell, dtype=torch.uint8).pin_memory()
    with pytest.raises(H.ErasureCodingError):
        coder(k, m).decode_host_batch(ptrs, cell, rows, out.data_ptr(), 1)


@pytest.mark.parametrize("k,m", [(6, 3), (10, 4)])
def test_device_vertical_in_file_order_out(dev, c_oracle, k, m):
    # device API strides express the reader's layout directly: shard-major
    # vertical inputs, row-major (file order) outputs
    rows, cell = 6, 8192
    file = splitmix64_bytes(7 + k, rows * k * cell)
    data = file.reshape(rows, k, cell)
    par = oracle_batch_encode(c_oracle, k, m, data)
    vert_d = torch.from_numpy(np.ascontiguousarray(data.transpose(1, 0, 2))).to(dev)  # [k][rows][cell]
    vert_p = torch.from_numpy(np.ascontiguousarray(par.transpose(1, 0, 2))).to(dev)  # [m][rows][cell]
    out = torch.zeros(rows * k * cell, dtype=torch.uint8, device=dev)
    miss = set(range(m))
    shard_ptrs = [None if i in miss else vert_d[i].data_ptr() for i in range(k)] + \
                 [vert_p[j].data_ptr() for j in range(m)]
    strides = [cell] * (k + m)
    out_ptrs = [out.data_ptr() + i * cell for i in range(k)]
    coder(k, m).decode_device(shard_ptrs, strides, out_ptrs, [k * cell] * k, cell, rows,
                              torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    o = out.cpu().numpy().reshape(rows, k, cell)
    for i in range(m):
        assert np.array_equal(o[:, i], data[:, i])


# ---- CRC32C per checksum chunk ------------------------

def _oracle_sums(cells: np.ndarray, bpc: int) -> np.ndarray:
    S, n, cell = cells.shape
    nch = (cell + bpc - 1) // bpc
    out = np.zeros((S, n, nch, 4), dtype=np.uint8)
    for s in range(S):
        for i in range(n):
            out[s, i] = np.frombuffer(O.chunk_crc32c(cells[s, i].tobytes(), bpc), dtype=np.uint8).reshape(nch, 4)
    return out


CRC32C_CASES = [(512 * 64, 512, 3), (512 * 70 + 256, 512, 2), (1 << 16, 512, 9), (4096, 4096, 2), (1000, 512, 3),
                (3 * 512 + 16, 512, 1), (2048, 100, 2)]


@pytest.mark.parametrize("cell,bpc,n", CRC32C_CASES)
def test_crc32c_device_vs_oracle(dev, cell, bpc, n):
    """The default CRC32C kernel (each 128-B quarter folded by a sparse
    multiple of the polynomial, 11-bit slicing of the tail; partial last
    tasks and short last chunks) and the generic byte kernel (other chunk
    sizes, unaligned cells) against the oracle."""
    crc32c_body(dev, cell, bpc, n, coder(6, 3))


def crc32c_body(dev, cell, bpc, n, cod, knob_pairs=(), xlib=None):
    S = 3
    cells = batch_data(S, n, cell, first=cell + bpc)
    with knobs(knob_pairs, xlib):
        got = H.crc32c_batch(cod, torch.from_numpy(cells).to(dev), bpc)
        torch.cuda.synchronize()
    assert np.array_equal(got.cpu().numpy(), _oracle_sums(cells, bpc))


def test_crc32c_pipelined_full_size_vs_byte_kernel(dev):
    """The default CRC32C kernel at a size where its prefetch runs steady
    (9 x 1 MiB x 64 cells, ~36 tasks per wave); the same bytes one byte off
    the 16-B grid go through the generic byte kernel: two independent kernels
    must agree (size-independent), and stripe 0 against the oracle."""
    S, n, cell = 64, 9, 1 << 20
    c = coder(6, 3)
    g = torch.Generator(device=dev).manual_seed(11)
    x = torch.empty((S, n, cell), dtype=torch.uint8, device=dev)
    x.random_(0, 256, generator=g)
    got = H.crc32c_batch(c, x, 512)
    buf = torch.empty(S * n * cell + 16, dtype=torch.uint8, device=dev)
    buf[1:1 + S * n * cell].copy_(x.flatten())
    ref = torch.empty_like(got)
    c.crc32c_device([buf.data_ptr() + 1 + i * cell for i in range(n)], [n * cell] * n, cell, S, 512, ref.data_ptr(),
                    torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    assert torch.equal(got, ref)
    assert np.array_equal(got[:1].cpu().numpy(), _oracle_sums(x[:1].cpu().numpy(), 512))


def test_crc32c_verify_pipelined_full_size(dev):
    """Verify mode of the default CRC32C kernel at full size: exactly the
    corrupted cells are flagged -- first byte, last byte, a middle byte, two
    in one stripe."""
    S, n, cell = 64, 9, 1 << 20
    c = coder(6, 3)
    g = torch.Generator(device=dev).manual_seed(12)
    x = torch.empty((S, n, cell), dtype=torch.uint8, device=dev)
    x.random_(0, 256, generator=g)
    sums = H.crc32c_batch(c, x, 512)
    hits = {(0, 0): 0, (5, 8): cell - 1, (31, 4): cell // 2 + 3, (63, 2): 8191, (63, 6): 8192}
    for (s_, i), b in hits.items():
        x[s_, i, b] ^= 0x41
    bad = H.checksum_verify_batch(c, x, sums, H.CHECKSUM_CRC32C, 512)
    torch.cuda.synchronize()
    want = torch.zeros((S, n), dtype=torch.uint8)
    for s_, i in hits:
        want[s_, i] = 1
    assert torch.equal(bad.cpu(), want)


def test_crc32c_device_published_vector(dev):
    cells = np.frombuffer(b"123456789" + bytes(7), dtype=np.uint8).reshape(1, 1, 16).copy()
    got = H.crc32c_batch(coder(6, 3), torch.from_numpy(cells[:, :, :9].copy()).to(dev), 512)
    torch.cuda.synchronize()
    assert got.cpu().numpy().ravel().tobytes() == (0xE3069283).to_bytes(4, "big")


ENCODE_CRC_CASES = [
    ("rs", 6, 3, 1 << 16, 4), ("rs", 6, 3, 3 * 512 + 16, 5), ("rs", 6, 3, (1 << 16) + 48, 3),
    ("rs", 10, 4, 1 << 15, 3), ("rs", 10, 4, 70 * 512 + 256, 2), ("rs", 3, 2, 1 << 17, 3),
    ("rs", 2, 1, 8192 + 512, 4), ("rs", 12, 4, 1 << 14, 2), ("rs", 6, 3, 1000, 2), ("xor", 2, 1, 1 << 14, 3),
    ("rs", 3, 2, 8192 + 512, 4), ("rs", 6, 3, 1 << 14, 7), ("rs", 2, 1, 1 << 15, 2), ("rs", 10, 4, 1 << 14, 5)]


@pytest.mark.parametrize("codec,k,m,cell,S", ENCODE_CRC_CASES)
def test_encode_crc_device(dev, c_oracle, codec, k, m, cell, S):
    """Fused encode+CRC (k in {2,3,6,10}: 8 slabs per wave for k <= 6 and
    r <= 3, else 4 with the inputs two at a time) and the two-pass fallback
    (other k, unaligned cell_len) against oracle parity + oracle CRCs."""
    encode_crc_body(dev, c_oracle, codec, k, m, cell, S, None)


def encode_crc_body(dev, c_oracle, codec, k, m, cell, S, xlib, knob_pairs=()):
    bpc = 512
    data = batch_data(S, k, cell, first=31 + cell)
    if codec == "xor":
        par = np.bitwise_xor.reduce(data, axis=1, keepdims=True)
        cod = H.Coder(k, m, 0, "xor", lib=xlib)
    else:
        par = oracle_batch_encode(c_oracle, k, m, data)
        cod = coder(k, m, xlib)
    d = torch.from_numpy(data).to(dev)
    p = torch.zeros((S, m, cell), dtype=torch.uint8, device=dev)
    nch = (cell + bpc - 1) // bpc
    sums = torch.zeros((S, k + m, nch, 4), dtype=torch.uint8, device=dev)
    dp, ds = H.stripe_layout_ptrs(d, k)
    pp, ps = H.stripe_layout_ptrs(p, m)
    with knobs(knob_pairs, xlib):
        cod.encode_crc_device(dp, ds, pp, ps, cell, S, bpc, sums.data_ptr(), torch.cuda.current_stream().cuda_stream)
        torch.cuda.synchronize()
    assert np.array_equal(p.cpu().numpy(), par)
    want = _oracle_sums(np.concatenate([data, par], axis=1), bpc)
    assert np.array_equal(sums.cpu().numpy(), want)


@pytest.mark.parametrize("k,m,S", [(6, 3, 64), (10, 4, 24), (3, 2, 64)])
def test_encode_crc_full_size_properties(dev, k, m, S):
    """1 MiB cells fused (RS(6,3) block tiles; RS(10,4) and RS(3,2) through
    the work queue of wave-tiles, twice in a row on one stream): parity
    equals a plain encode and sums equal a standalone CRC pass over the same
    k+m cells (size-independent)."""
    cell = 1 << 20
    c = coder(k, m)
    d = torch.empty((S, k, cell), dtype=torch.uint8, device=dev)
    g = torch.Generator(device=dev).manual_seed(7)
    d.random_(0, 256, generator=g)
    p1 = torch.empty((S, m, cell), dtype=torch.uint8, device=dev)
    p2 = torch.empty_like(p1)
    H.encode_batch(c, d, p1)
    sums = torch.empty((S, k + m, cell // 512, 4), dtype=torch.uint8, device=dev)
    dp, ds = H.stripe_layout_ptrs(d, k)
    pp, ps = H.stripe_layout_ptrs(p2, m)
    for _ in range(2):
        p2.zero_()
        sums.zero_()
        c.encode_crc_device(dp, ds, pp, ps, cell, S, 512, sums.data_ptr(), torch.cuda.current_stream().cuda_stream)
        ref = H.crc32c_batch(c, torch.cat([d, p1], dim=1), 512)
        torch.cuda.synchronize()
        assert torch.equal(p1, p2)
        assert torch.equal(sums, ref)


# ---- Chunk checksums on the read path: CRC32 / CRC32C verify and the ----
# ---- verified striped read (connection.rs:477-504) ----

CKSUM_TYPES = [H.CHECKSUM_CRC32C, H.CHECKSUM_CRC32]


def _oracle_checksums(cells: np.ndarray, bpc: int, ctype: int) -> np.ndarray:
    S, n, cell = cells.shape
    nch = (cell + bpc - 1) // bpc
    out = np.zeros((S, n, nch, 4), dtype=np.uint8)
    for s in range(S):
        for i in range(n):
            out[s, i] = np.frombuffer(O.chunk_checksums(cells[s, i].tobytes(), bpc, ctype),
                                      dtype=np.uint8).reshape(nch, 4)
    return out


CHECKSUM_CASES = [(512 * 64, 512, 3), (512 * 70 + 256, 512, 2), (1000, 512, 3), (4096, 4096, 2), (2048, 100, 2)]


@pytest.mark.parametrize("ctype", CKSUM_TYPES)
@pytest.mark.parametrize("cell,bpc,n", CHECKSUM_CASES)
def test_checksum_device_vs_oracle(dev, ctype, cell, bpc, n):
    checksum_body(dev, ctype, cell, bpc, n, coder(6, 3))


def checksum_body(dev, ctype, cell, bpc, n, cod, knob_pairs=(), xlib=None):
    S = 3
    cells = batch_data(S, n, cell, first=cell + bpc + ctype)
    with knobs(knob_pairs, xlib):
        got = H.checksum_batch(cod, torch.from_numpy(cells).to(dev), ctype, bpc)
        torch.cuda.synchronize()
    assert np.array_equal(got.cpu().numpy(), _oracle_checksums(cells, bpc, ctype))


def test_checksum_device_catalog_checks(dev):
    cells = torch.from_numpy(np.frombuffer(b"123456789", dtype=np.uint8).reshape(1, 1, 9).copy()).to(dev)
    for ctype, want in ((H.CHECKSUM_CRC32C, 0xE3069283), (H.CHECKSUM_CRC32, 0x765E7680)):
        got = H.checksum_batch(coder(6, 3), cells, ctype, 512)
        torch.cuda.synchronize()
        assert got.cpu().numpy().ravel().tobytes() == want.to_bytes(4, "big")


@pytest.mark.parametrize("ctype", CKSUM_TYPES)
@pytest.mark.parametrize("cell,bpc", [(1 << 15, 512), (512 * 9 + 48, 512), (3000, 100)])
def test_checksum_verify_flags_exactly_the_corrupt_cells(dev, ctype, cell, bpc):
    S, n = 4, 5
    cells = batch_data(S, n, cell, first=77 + cell)
    sums = torch.from_numpy(_oracle_checksums(cells, bpc, ctype)).to(dev)
    bent = cells.copy()
    hits = {(0, 1): 0, (2, 4): cell - 1, (3, 0): cell // 2}  # first, last (short chunk), middle byte
    for (s, i), b in hits.items():
        bent[s, i, b] ^= 0x10
    bad = H.checksum_verify_batch(coder(6, 3), torch.from_numpy(bent).to(dev), sums, ctype, bpc)
    torch.cuda.synchronize()
    want = np.zeros((S, n), dtype=np.uint8)
    for s, i in hits:
        want[s, i] = 1
    assert np.array_equal(bad.cpu().numpy(), want)
    # CHECKSUM_NULL verifies nothing
    none = H.checksum_verify_batch(coder(6, 3), torch.from_numpy(bent).to(dev), sums, H.CHECKSUM_NULL, bpc)
    assert not none.any()


def _verified_read_expect(k, m, data, parity, missing, missing_parity, sums_np, bpc, ctype):
    """Per stripe: oracle verified_read_row -> (data [S,k,cell], bad [S,k+m],
    ok [S])."""
    S, _, cell = data.shape
    outs, bads, oks = np.zeros_like(data), np.zeros((S, k + m), dtype=np.uint8), []
    for s in range(S):
        cells = [None if i in missing else data[s, i].tobytes() for i in range(k)]
        cells += [None if j in missing_parity else parity[s, j].tobytes() for j in range(m)]
        sums = [sums_np[s, i].tobytes() for i in range(k + m)]
        try:
            got, bad = O.verified_read_row(k, m, cells, sums, bpc, ctype)
            outs[s] = np.stack([np.frombuffer(g, dtype=np.uint8) for g in got])
            oks.append(True)
        except O.NotEnoughShards:
            # flags the oracle saw before giving up: every available cell failed-or-read
            bad = [0] * (k + m)
            for i in range(k + m):
                if cells[i] is not None and not O.get_data_ok(cells[i], sums[i], bpc, ctype):
                    bad[i] = 1
            oks.append(False)
        bads[s] = bad
    return outs, bads, oks


VERIFY_CASES = [
    (6, 3, 1 << 15, 512, [0, 1, 2], []), (6, 3, 512 * 9 + 48, 512, [4], [1]), (6, 3, 1 << 14, 512, [], []),
    (10, 4, 1 << 14, 512, [0, 1, 2, 3], []), (10, 4, 1 << 13, 512, [7], [0]), (3, 2, 1 << 14, 512, [1], []),
    (2, 1, 8192, 512, [0], []), (12, 4, 1 << 13, 512, [2, 5], []), (6, 3, 3000, 100, [0, 5], []),
    (6, 3, 4096 + 16, 4096, [3], [])]


@pytest.mark.parametrize("ctype", CKSUM_TYPES)
@pytest.mark.parametrize("k,m,cell,bpc,missing,missing_parity", VERIFY_CASES)
def test_decode_verify_vs_oracle(dev, c_oracle, ctype, k, m, cell, bpc, missing, missing_parity):
    """Fused (k in {2,3,6,10}, 512-B chunks) and two-pass decode+verify: clean
    stripes, corrupt survivors (data and parity), a stripe that runs out of
    verified shards; rebuilt data, bad flags and the error all as the
    oracle's read_slice restatement."""
    decode_verify_body(dev, c_oracle, ctype, k, m, cell, bpc, missing, missing_parity, coder(k, m))


def decode_verify_body(dev, c_oracle, ctype, k, m, cell, bpc, missing, missing_parity, cod, knob_pairs=(),
                       xlib=None):
    S = 6
    data = batch_data(S, k, cell, first=5 + cell + k)
    parity = oracle_batch_encode(c_oracle, k, m, data)
    sums_np = _oracle_checksums(np.concatenate([data, parity], axis=1), bpc, ctype)
    avail = [i for i in range(k + m) if (i < k and i not in missing) or (i >= k and i - k not in missing_parity)]
    bd, bp = data.copy(), parity.copy()

    def bend(s, shard, byte):
        (bd[s, shard] if shard < k else bp[s, shard - k])[byte] ^= 0x5A

    spare = len(avail) - k
    bend(1, avail[0], 3)                       # first survivor
    bend(2, avail[k - 1], cell - 1)            # last survivor, last byte
    bend(3, avail[1], cell // 2)
    if spare >= 2:
        bend(3, avail[k], 0)                   # ... and its replacement too
    for t in range(spare + 1):                 # stripe 5: one failure too many
        bend(5, avail[t], 100 + t)
    want_data, want_bad, oks = _verified_read_expect(k, m, bd, bp, set(missing), set(missing_parity), sums_np,
                                                     bpc, ctype)
    assert not oks[5] and oks[0] and oks[4]
    d, p = torch.from_numpy(bd).to(dev), torch.from_numpy(bp).to(dev)
    out = torch.zeros_like(d)
    sums = torch.from_numpy(sums_np).to(dev)
    bad = torch.full((S, k + m), 7, dtype=torch.uint8, device=dev)
    dp, ds = H.stripe_layout_ptrs(d, k)
    pp, ps = H.stripe_layout_ptrs(p, m)
    op, os_ = H.stripe_layout_ptrs(out, k)
    ptrs = [None if i in missing else dp[i] for i in range(k)] + \
        [None if j in missing_parity else pp[j] for j in range(m)]
    with knobs(knob_pairs, xlib):
        with pytest.raises(H.ErasureCodingError):
            cod.decode_verify_device(ctype, ptrs, ds + ps, op, os_, cell, S, bpc, sums.data_ptr(), bad.data_ptr(),
                                     torch.cuda.current_stream().cuda_stream)
        torch.cuda.synchronize()
    o, b = out.cpu().numpy(), bad.cpu().numpy()
    for s in range(S):
        if not oks[s]:
            continue  # the reference returns no row; flags there are partial by design
        assert np.array_equal(b[s], want_bad[s]), s
        for i in range(k):
            if i in missing or want_bad[s, i]:
                assert np.array_equal(o[s, i], want_data[s, i]), (s, i)
            else:
                assert not o[s, i].any(), (s, i)  # present + verified: not copied


JIT_CASES = [c for c in VERIFY_CASES if c[0] in (2, 3, 6, 10) and c[3] == 512 and 1 <= len(c[4]) <= 4]


@pytest.mark.parametrize("ctype", CKSUM_TYPES)
@pytest.mark.parametrize("k,m,cell,bpc,missing,missing_parity", JIT_CASES)
def test_decode_verify_jit_specialised_vs_oracle(dev, c_oracle, ctype, k, m, cell, bpc, missing, missing_parity):
    """The plan-specialised fused decode + verify kernel (jit.cpp: the decode
    plan's bit-sliced XOR network compiled with hiprtc, prepared
    synchronously) over the same cases as the ahead-of-time kernel: rebuilt
    data, bad flags and the error as the oracle's read_slice restatement; the
    launch counter proves the specialised kernel ran."""
    cod = H.Coder(k, m, 0)
    lost = list(missing) + [k + j for j in missing_parity]
    assert cod.prepare_decode(lost, ctype), "hiprtc unavailable on the GPU box"
    before = H.jit_stats()["launches"]
    decode_verify_body(dev, c_oracle, ctype, k, m, cell, bpc, missing, missing_parity, cod)
    assert H.jit_stats()["launches"] > before
    cod.close()


def test_decode_verify_jit_full_size(dev):
    """RS(6,3) 1 MiB x 64 with data shards {0,1,2} lost through the
    specialised kernel: rebuilt cells == the originals, no flags; then with
    {0,1} lost (one spare survivor), one flipped byte in survivor 4 of stripe
    7 is flagged and routed around (parity 2 read instead, shard 4 rebuilt
    in place)."""
    k, m, cell, S = 6, 3, 1 << 20, 64
    c = H.Coder(k, m, 0)
    assert c.prepare_decode([0, 1, 2]) and c.prepare_decode([0, 1])
    d = torch.empty((S, k, cell), dtype=torch.uint8, device=dev)
    d.random_(0, 256, generator=torch.Generator(device=dev).manual_seed(17))
    p = torch.empty((S, m, cell), dtype=torch.uint8, device=dev)
    H.encode_batch(c, d, p)
    sums = H.checksum_batch(c, torch.cat([d, p], dim=1), H.CHECKSUM_CRC32C, 512)
    before = H.jit_stats()["launches"]
    out = torch.zeros_like(d)
    bad = H.decode_verify_batch(c, d, p, [0, 1, 2], sums, out)
    torch.cuda.synchronize()
    assert H.jit_stats()["launches"] == before + 1
    assert not bad.any()
    assert torch.equal(out[:, :3], d[:, :3])
    d[7, 4, 777] ^= 0x10
    out.zero_()
    before = H.jit_stats()["launches"]
    bad = H.decode_verify_batch(c, d, p, [0, 1], sums, out)
    torch.cuda.synchronize()
    assert H.jit_stats()["launches"] == before + 1
    assert bad.nonzero().tolist() == [[7, 4]]
    d[7, 4, 777] ^= 0x10
    assert torch.equal(out[:, :2], d[:, :2]) and torch.equal(out[7, 4], d[7, 4])
    c.close()


@pytest.mark.parametrize("ctype", CKSUM_TYPES)
def test_decode_verify_null_type_is_plain_decode(dev, c_oracle, ctype):
    k, m, cell, S = 6, 3, 1 << 14, 3
    data = batch_data(S, k, cell, first=99)
    parity = oracle_batch_encode(c_oracle, k, m, data)
    d, p = torch.from_numpy(data).to(dev), torch.from_numpy(parity).to(dev)
    out = torch.zeros_like(d)
    sums = torch.zeros((S, k + m, cell // 512, 4), dtype=torch.uint8, device=dev)  # wrong sums: ignored
    H.decode_verify_batch(coder(k, m), d, p, [0, 4], sums, out, H.CHECKSUM_NULL, 512)
    torch.cuda.synchronize()
    assert torch.equal(out[:, [0, 4]], d[:, [0, 4]])


def test_decode_verify_full_size_properties(dev):
    """RS(6,3) 1 MiB x 64: with shards {0,1,2} missing the fused verified
    read equals a plain decode with no flags; with {0,1} missing, one flipped
    byte in survivor 3 of stripe 5 is flagged and routed around (parity 2 is
    read instead) and that data cell is rebuilt too."""
    k, m, cell, S = 6, 3, 1 << 20, 64
    c = coder(k, m)
    d = torch.empty((S, k, cell), dtype=torch.uint8, device=dev)
    d.random_(0, 256, generator=torch.Generator(device=dev).manual_seed(11))
    p = torch.empty((S, m, cell), dtype=torch.uint8, device=dev)
    H.encode_batch(c, d, p)
    sums = H.checksum_batch(c, torch.cat([d, p], dim=1), H.CHECKSUM_CRC32C, 512)
    out = torch.zeros_like(d)
    bad = H.decode_verify_batch(c, d, p, [0, 1, 2], sums, out)
    torch.cuda.synchronize()
    assert not bad.any()
    assert torch.equal(out[:, :3], d[:, :3])
    d[5, 3, 12345] ^= 1
    out.zero_()
    bad = H.decode_verify_batch(c, d, p, [0, 1], sums, out)
    torch.cuda.synchronize()
    assert bad.nonzero().tolist() == [[5, 3]]
    d[5, 3, 12345] ^= 1
    assert torch.equal(out[:, :2], d[:, :2])
    assert torch.equal(out[5, 3], d[5, 3])
    assert not out[:5, 2:].any() and not out[6:, 2:].any()


def test_concurrent_threads_shared_and_private_coders(dev, c_oracle):
    # The reference Coder is Send + Sync and is called from many tokio workers
    # at once.  Eight threads (ctypes drops the GIL around every
    # call): half share one coder's host-buffer API (internal lock, shared
    # plan cache), half own a coder; every thread also runs the device API on
    # its own stream.  All results bit-exact against the oracle.
    import threading

    import ec_oracle as EO
    k, m = 6, 3
    shared = H.Coder(k, m, 0)
    errors = []

    def worker(t):
        try:
            rng = np.random.default_rng(0x7EAD + t)
            c = shared if t % 2 == 0 else H.Coder(k, m, 0)
            stream = torch.cuda.Stream(device=dev)
            for it in range(5):
                n = int(rng.integers(1, 70000))
                data = [rng.integers(0, 256, n, dtype=np.uint8) for _ in range(k)]
                par = [np.frombuffer(p, dtype=np.uint8) for p in c.encode(data)]
                want = EO.c_encode(c_oracle, k, m, data)
                assert all(np.array_equal(par[j], want[j]) for j in range(m)), f"t{t} encode"
                lost = rng.choice(k + m, size=int(rng.integers(1, m + 1)), replace=False)
                shards = [None if i in lost else (data[i] if i < k else par[i - k]).tobytes()
                          for i in range(k + m)]
                c.decode(shards)
                for i in range(k):
                    assert np.array_equal(np.frombuffer(shards[i], dtype=np.uint8), data[i]), f"t{t} decode"
                # device API on this thread's stream (allocation, copies and
                # kernels all ordered on it)
                S, cell = 3, 4096 * int(rng.integers(1, 9)) + 16 * int(rng.integers(0, 4))
                miss = sorted(int(i) for i in rng.choice(k, size=m, replace=False))
                with torch.cuda.stream(stream):
                    d = torch.from_numpy(batch_data(S, k, cell, first=1000 * t + it)).to(dev)
                    p = torch.zeros((S, m, cell), dtype=torch.uint8, device=dev)
                    out = torch.zeros_like(d)
                    H.encode_batch(c, d, p)
                    H.decode_batch(c, d, p, miss, out)
                stream.synchronize()
                wantb = oracle_batch_encode(c_oracle, k, m, d.cpu().numpy())
                assert np.array_equal(p.cpu().numpy(), wantb), f"t{t} encode_device"
                for i in miss:
                    assert torch.equal(out[:, i], d[:, i]), f"t{t} decode_device"
            if c is not shared:
                c.close()
        except Exception as e:  # surfaced below
            errors.append(repr(e))

    threads = [threading.Thread(target=worker, args=(t,)) for t in range(8)]
    for th in threads:
        th.start()
    for th in threads:
        th.join(timeout=100)
    assert not any(th.is_alive() for th in threads), "a worker hung"
    assert not errors, errors
    shared.close()


# ---- multi-GPU coder group (hec_group_*) ----------------------
# The box has one GPU: a group that lists device 0 several times runs several
# coders (own streams, own host threads) on it -- the same partitioning and
# threading as one slot per GPU.

@pytest.mark.parametrize("slots,S,chunk,cell", [(1, 5, 2, 65536), (3, 10, 2, 65536), (4, 3, 1, 4096 + 16),
                                                (8, 13, 3, 1000)])
def test_group_encode_host_batch(c_oracle, slots, S, chunk, cell):
    k, m = 6, 3
    g = H.CoderGroup(k, m, [0] * slots)
    data = batch_data(S, k, cell, first=70 + slots)
    want = oracle_batch_encode(c_oracle, k, m, data)
    h_in = torch.from_numpy(data).pin_memory()
    h_out = torch.zeros((S, m, cell), dtype=torch.uint8).pin_memory()
    g.encode_host_batch(h_in.data_ptr(), h_out.data_ptr(), cell, S, chunk)
    assert np.array_equal(h_out.numpy(), want)
    g.close()


@pytest.mark.parametrize("k,m,lost", [(6, 3, (0, 1, 2)), (10, 4, (1, 5, 9, 12)), (3, 2, ())])
@pytest.mark.parametrize("slots,rows", [(2, 7), (3, 2), (5, 9)])
def test_group_decode_host_batch_file_order(c_oracle, k, m, lost, slots, rows):
    cell = 4096 + 16
    file = splitmix64_bytes(rows * 77 + k + slots, rows * k * cell)
    data = file.reshape(rows, k, cell)
    par = oracle_batch_encode(c_oracle, k, m, data)
    vertical = [np.ascontiguousarray(data[:, i, :]).ravel() for i in range(k)] + \
               [np.ascontiguousarray(par[:, j, :]).ravel() for j in range(m)]
    hv = [None if i in lost else torch.from_numpy(vertical[i]).pin_memory() for i in range(k + m)]
    out = torch.zeros(rows * k * cell, dtype=torch.uint8).pin_memory()
    g = H.CoderGroup(k, m, [0] * slots)
    g.decode_host_batch([None if t is None else t.data_ptr() for t in hv], cell, rows, out.data_ptr(), 2)
    assert np.array_equal(out.numpy(), file)
    g.close()


def test_group_errors_and_slot_coders(dev, c_oracle):
    with pytest.raises(H.DeviceError):
        H.CoderGroup(6, 3, [0, 4096])  # no such device: the slots created so far are released
    with pytest.raises(H.UnsupportedErasureCodingPolicy):
        H.CoderGroup(6, 3, [0], codec="lrc")
    g = H.CoderGroup(6, 3, [0, 0, 0])
    assert len(g) == 3
    from hdfs_native_ec.dist import shard_range
    for total in (0, 1, 2, 10, 2048, 65537):
        assert [g.range(total, i) for i in range(3)] == [shard_range(total, 3, i) for i in range(3)]
    # every slot's coder serves the device-resident API on its GPU
    S, cell = 9, 8192
    data = batch_data(S, 6, cell, first=5)
    want = oracle_batch_encode(c_oracle, 6, 3, data)
    d = torch.from_numpy(data).to(dev)
    p = torch.zeros((S, 3, cell), dtype=torch.uint8, device=dev)
    for slot in range(3):
        first, count = g.range(S, slot)
        H.encode_batch(g.coder(slot), d[first:first + count], p[first:first + count])
    torch.cuda.synchronize()
    assert np.array_equal(p.cpu().numpy(), want)
    # too many losses: every slot reports it, the call returns the status
    cell, rows = 4096, 4
    hv = [torch.zeros(rows * cell, dtype=torch.uint8).pin_memory() for _ in range(9)]
    ptrs = [t.data_ptr() for t in hv]
    ptrs[0] = ptrs[1] = ptrs[2] = ptrs[3] = None
    out = torch.zeros(rows * 6 * cell, dtype=torch.uint8).pin_memory()
    with pytest.raises(H.ErasureCodingError):
        g.decode_host_batch(ptrs, cell, rows, out.data_ptr(), 1)
    g.close()


@pytest.mark.parametrize("k,m,slots", [(6, 3, 3), (10, 4, 2), (3, 2, 5)])
def test_group_device_resident_encode_decode(dev, c_oracle, k, m, slots):
    """hec_group_encode_device / hec_group_decode_device: every slot's stripes
    in its device's HBM (here all on device 0), each slot on its own stream,
    uneven per-slot stripe counts (one slot empty), enqueued from one thread;
    parity and rebuilt data bit-exact against the oracle."""
    cell = 8192 + 16
    g = H.CoderGroup(k, m, [0] * slots)
    counts = [(3 + 2 * i) if i != 1 else 0 for i in range(slots)]
    streams = [torch.cuda.Stream(dev) for _ in range(slots)]
    datas = [batch_data(max(c, 1), k, cell, first=300 + 17 * i)[:c] for i, c in enumerate(counts)]
    d = [torch.from_numpy(np.ascontiguousarray(x)).to(dev) for x in datas]
    p = [torch.zeros((c, m, cell), dtype=torch.uint8, device=dev) for c in counts]
    dp, ds, pp, ps = [], [], [], []
    for i in range(slots):
        a, b = H.stripe_layout_ptrs(d[i], k) if counts[i] else ([0] * k, [k * cell] * k)
        c_, e_ = H.stripe_layout_ptrs(p[i], m) if counts[i] else ([0] * m, [m * cell] * m)
        dp += a; ds += b; pp += c_; ps += e_
    torch.cuda.synchronize()
    g.encode_device(dp, ds, pp, ps, cell, counts, [s.cuda_stream for s in streams])
    torch.cuda.synchronize()
    for i in range(slots):
        if counts[i]:
            assert np.array_equal(p[i].cpu().numpy(), oracle_batch_encode(c_oracle, k, m, datas[i])), i
    # decode: data shards 0..m-1 lost in every slot, rebuilt into out
    out = [torch.zeros((c, k, cell), dtype=torch.uint8, device=dev) for c in counts]
    sp, ss, op, os_ = [], [], [], []
    for i in range(slots):
        a, b = (dp[i * k:(i + 1) * k], ds[i * k:(i + 1) * k])
        sp += [None if j < m else a[j] for j in range(k)] + pp[i * m:(i + 1) * m]
        ss += b + ps[i * m:(i + 1) * m]
        c_, e_ = H.stripe_layout_ptrs(out[i], k) if counts[i] else ([0] * k, [k * cell] * k)
        op += c_; os_ += e_
    g.decode_device(sp, ss, op, os_, cell, counts, [s.cuda_stream for s in streams])
    torch.cuda.synchronize()
    for i in range(slots):
        if counts[i]:
            assert torch.equal(out[i][:, :m], d[i][:, :m]), i
    # a slot with too many losses: its status comes back, the others still run
    bad = list(sp)
    for j in range(m + 1):
        bad[j] = None
    for i in range(slots):
        out[i].zero_()
    with pytest.raises(H.ErasureCodingError):
        g.decode_device(bad, ss, op, os_, cell, counts, [s.cuda_stream for s in streams])
    torch.cuda.synchronize()
    for i in range(1, slots):
        if counts[i]:
            assert torch.equal(out[i][:, :m], d[i][:, :m]), i
    g.close()


def test_numa_host_buffers_feed_the_host_batch(c_oracle):
    # hec_host_alloc (pinned, NUMA-placed) buffers through hec_encode_host_batch
    k, m, cell, S = 6, 3, 65536, 9
    node = H.device_numa_node(0)
    hin, hout = H.HostBuffer(S * k * cell, 0, -1), H.HostBuffer(S * m * cell, 0, -1)
    try:
        data = batch_data(S, k, cell, first=123)
        hin.array()[:] = data.ravel()
        coder(k, m).encode_host_batch(hin.ptr, hout.ptr, cell, S, 4)
        want = oracle_batch_encode(c_oracle, k, m, data)
        assert np.array_equal(hout.array().reshape(S, m, cell), want)
    finally:
        hin.close()
        hout.close()
    assert node >= -1
    import ctypes
    assert H.lib.hec_host_free(ctypes.c_void_p(12345)) == H.HEC_ERR_INVALID_ARG  # not ours: refused, not freed


# ---- full-batch oracle parity at the BASELINE sizes -------------------------
# Every byte of every stripe of the benchmark batches against the C
# restatement (oracle/ec_oracle.c), stripe-parallel on the box's CPU share:
# the engine's parity, and its decode of the worst-case erasure set against
# the oracle's decode of the same survivors (gf256.rs:61-137).

def _cpu_share():
    import os
    return max(1, min(16, int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or (os.cpu_count() or 8)))


@pytest.mark.parametrize("k,m,cell,S,lost", [(6, 3, 1 << 20, 1024, (0, 1, 2)), (6, 3, 1 << 16, 65536, (0, 1, 2)),
                                             (10, 4, 1 << 20, 256, (0, 1, 2, 3))])
def test_full_batch_vs_oracle(dev, c_oracle, k, m, cell, S, lost):
    cod = coder(k, m)
    d = _device_random((S, k, cell), dev, seed=0x5EED_EC00 + k * 7 + S)
    p = torch.empty((S, m, cell), dtype=torch.uint8, device=dev)
    H.encode_batch(cod, d, p)
    e = len(lost)
    rec = torch.empty((S, e, cell), dtype=torch.uint8, device=dev)
    dp, ds = H.stripe_layout_ptrs(d, k)
    pp, ps = H.stripe_layout_ptrs(p, m)
    shard_ptrs = [None if i in lost else dp[i] for i in range(k)] + pp
    out = [rec.data_ptr() + lost.index(i) * cell if i in lost else 0 for i in range(k)]
    cod.decode_device(shard_ptrs, ds + ps, out, [e * cell] * k, cell, S, torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    assert torch.equal(rec, d[:, list(lost)])  # the round trip, on the device
    present = ((1 << (k + m)) - 1) & ~sum(1 << i for i in lost)
    step = max(1, (1 << 31) // (k * cell))  # <= 2 GiB of data per slice on the host
    for a in range(0, S, step):
        b = min(S, a + step)
        O.c_check_batch(c_oracle, k, m, d[a:b].cpu().numpy(), p[a:b].cpu().numpy(), present,
                        rec[a:b].cpu().numpy(), threads=_cpu_share())


# ---- whole files: the last row short (CellBuffer / CellReader semantics) ----

def _file_sizes(k, cell):
    # rust/tests/test_ec.rs:77-87 sizes_to_test around this cell size, plus a
    # 1-byte file and one row +- 4
    return [1, 16, cell - 4, cell, cell + 4, k * cell - 4, k * cell, k * cell + 4, 5 * k * cell - 4, 5 * k * cell,
            5 * k * cell + 4]


def _want_parity(rows, k, m, cell):
    want = np.zeros((len(rows), m, cell), dtype=np.uint8)
    for r, row in enumerate(rows):
        for j in range(m):
            par = np.frombuffer(row[k + j], dtype=np.uint8)
            want[r, j, :len(par)] = par
    return want


@pytest.mark.parametrize("k,m", [(3, 2), (6, 3), (10, 4)])
def test_encode_rows_partial_last_row(dev, k, m):
    """hec_encode_rows_host / _device over whole files: full rows batched, the
    short last row padded as CellBuffer::encode (block_writer.rs:817-851),
    parity cells of len(cell 0) bytes, the slot past them zeroed."""
    cell = 1 << 16
    cod = coder(k, m)
    ws = torch.empty(cod.encode_rows_workspace_size(cell), dtype=torch.uint8, device=dev)
    for L in _file_sizes(k, cell):
        data = splitmix64_bytes(L * 3 + k, L)
        rows = O.striped_write(data.tobytes(), k, m, cell)
        want = _want_parity(rows, k, m, cell)
        hp = np.full((len(rows), m, cell), 0xA5, dtype=np.uint8)
        cod.encode_rows_host(data.ctypes.data, L, hp.ctypes.data, cell, 2)
        assert np.array_equal(hp, want), L
        dd = torch.from_numpy(data.copy()).to(dev)
        dpar = torch.full((len(rows), m, cell), 0xA5, dtype=torch.uint8, device=dev)
        cod.encode_rows_device(dd.data_ptr(), L, dpar.data_ptr(), cell, ws.data_ptr(), ws.numel(),
                               torch.cuda.current_stream().cuda_stream)
        torch.cuda.synchronize()
        assert np.array_equal(dpar.cpu().numpy(), want), L


def test_encode_rows_device_workspace_checked_first(dev):
    """A missing workspace is rejected before any row is queued (no parity
    half-written), and is not needed when no cell of the short row is short."""
    k, m, cell = 6, 3, 1 << 16
    cod = coder(k, m)
    s = torch.cuda.current_stream().cuda_stream
    L = 3 * k * cell + 2 * cell + 100  # cells 3.. of the last row are short
    data = torch.from_numpy(splitmix64_bytes(77, L)).to(dev)
    dpar = torch.full((4, m, cell), 0xA5, dtype=torch.uint8, device=dev)
    with pytest.raises(ValueError):
        cod.encode_rows_device(data.data_ptr(), L, dpar.data_ptr(), cell, 0, 0, s)
    torch.cuda.synchronize()
    assert bool((dpar == 0xA5).all()), "full rows were written before the argument check"
    # k == 1: the short row is one cell of n0 bytes, nothing to pad, so no
    # workspace is needed
    c1 = H.Coder(1, 2, 0)
    L1 = 3 * cell + 1000
    d1 = torch.from_numpy(splitmix64_bytes(78, L1)).to(dev)
    p1 = torch.full((4, 2, cell), 0xA5, dtype=torch.uint8, device=dev)
    c1.encode_rows_device(d1.data_ptr(), L1, p1.data_ptr(), cell, 0, 0, s)
    torch.cuda.synchronize()
    rows = O.striped_write(d1.cpu().numpy().tobytes(), 1, 2, cell)
    assert np.array_equal(p1.cpu().numpy(), _want_parity(rows, 1, 2, cell))
    c1.close()


@pytest.mark.parametrize("k,m", [(3, 2), (6, 3), (10, 4)])
def test_decode_rows_partial_last_row(c_oracle, k, m):
    """hec_decode_rows_host over the blocks a striped write leaves (shard i =
    max_offset(i) bytes, ec/mod.rs:40-60): short and absent cells read as
    zeros (CellReader::next_cell), the file trimmed to its length; every lost
    set the reader can meet, against the oracle's striped read."""
    cell = 1 << 16
    cod = coder(k, m)
    lost_sets = [(), (0,), (k - 1,), (0, k), tuple(range(m)), tuple(range(k - m, k))]
    for L in _file_sizes(k, cell):
        data = splitmix64_bytes(L * 5 + k, L).tobytes()
        vert = O.vertical_buffers(O.striped_write(data, k, m, cell), k, m)
        for i in range(k + m):
            assert len(vert[i]) == O.max_offset(k, cell, i, L)
        arrs = [np.frombuffer(v, dtype=np.uint8) for v in vert]
        for lost in lost_sets:
            want = O.striped_read([None if i in lost else vert[i] for i in range(k + m)], k, m, cell, L)
            assert want == data
            out = np.full(L + 64, 0x3C, dtype=np.uint8)  # 64 guard bytes past the file
            addrs = [0 if i in lost else arrs[i].ctypes.data for i in range(k + m)]
            lens = [0 if i in lost else len(vert[i]) for i in range(k + m)]
            cod.decode_rows_host(addrs, lens, cell, out.ctypes.data, L, 2)
            assert out[:L].tobytes() == data, (L, lost)
            assert (out[L:] == 0x3C).all(), (L, lost)


@pytest.mark.parametrize("k,m", [(3, 2), (6, 3)])
@pytest.mark.parametrize("route", ["default", "device", "host"])
def test_per_call_reference_sizes(c_oracle, k, m, route):
    """The per-call drop-in (hec_encode / hec_decode) on every row a striped
    write of the reference's sizes_to_test files (test_ec.rs:77-87, 1 MiB
    cells) produces, through the default size routing, the device forced
    (host limit 0) and the host routine forced; bit-exact vs the oracle."""
    cell = 1 << 20
    cod = H.Coder(k, m, 0)
    cod.host_limit = {"default": cod.host_limit, "device": 0, "host": 1 << 30}[route]
    for L in [16, cell - 4, cell, cell + 4, 5 * k * cell - 4, 5 * k * cell + 4]:
        data = splitmix64_bytes(L + 17 * k, L).tobytes()
        rows = O.cell_buffer_rows(data, k, cell)
        for r in (rows[0], rows[-1]):  # a full row (when there is one) and the last row
            n0 = len(r[0])
            padded = [c + b"\0" * (n0 - len(c)) for c in r]
            want = O.cell_buffer_encode(k, m, r)[k:]
            got = cod.encode(padded)
            assert got == want, (L, n0)
            shards = [None if i < m else (padded + got)[i] for i in range(k + m)]  # worst case
            cod.decode(shards)
            assert shards[:k] == padded, (L, n0)
    cod.close()


# ---- pooled coders (Coder::new per row) -------------------------------------

def test_coder_pool_reuses_and_isolates(dev, c_oracle):
    H.pool_trim()
    a = H.Coder(6, 3, 0, pooled=True)
    ha = a.handle.value
    a.close()
    b = H.Coder(6, 3, 0, pooled=True)
    assert b.handle.value == ha  # the idle coder comes back
    c = H.Coder(6, 3, 0, pooled=True)
    assert c.handle.value != ha  # b is still out: a second coder
    x = H.Coder(3, 2, -1, pooled=True)  # another key; any device
    assert x.device == 0 and x.handle.value not in (ha, c.handle.value)
    data = [splitmix64_bytes(40 + i, 4096) for i in range(6)]
    want = [w.tobytes() for w in O.c_encode(c_oracle, 6, 3, data)]
    assert b.encode(data) == want and c.encode(data) == want
    for cc in (b, c, x):
        cc.close()
    assert H.pool_trim() == 3


def test_coder_pool_threads(dev, c_oracle):
    # 8 threads x 300 acquire / encode / decode / release cycles of small rows
    import threading
    errors = []
    k, m = 6, 3

    def worker(t):
        rng = np.random.default_rng(t)
        try:
            for it in range(300):
                n = int(rng.integers(1, 5000))
                data = [rng.integers(0, 256, n, dtype=np.uint8) for _ in range(k)]
                c = H.Coder(k, m, 0, pooled=True)
                par = c.encode(data)
                shards = [None, None] + [d.tobytes() for d in data[2:]] + par
                c.decode(shards)
                c.close()
                if par != [w.tobytes() for w in O.c_encode(c_oracle, k, m, data)] or shards[0] != data[0].tobytes():
                    errors.append((t, it))
        except Exception as e:  # surfaced below
            errors.append(repr(e))

    ths = [threading.Thread(target=worker, args=(t,)) for t in range(8)]
    for th in ths:
        th.start()
    for th in ths:
        th.join(timeout=100)
    assert not errors, errors[:5]
    assert H.pool_trim() <= 8  # at most one idle coder per concurrent user


# ---- verified reads sharing one coder (the phase-2 scratch is serialised) ---

def test_decode_verify_two_threads_share_a_coder(dev, c_oracle):
    import threading
    k, m, cell, S = 6, 3, 1 << 14, 24
    cod = H.Coder(k, m, 0)
    data = batch_data(S, k, cell, first=4242)
    par = oracle_batch_encode(c_oracle, k, m, data)
    sums_np = np.concatenate([data, par], axis=1)
    sums = torch.from_numpy(np.stack([np.stack([np.frombuffer(O.chunk_crc32c(sums_np[s, i].tobytes(), 512),
                                                              dtype=np.uint8).reshape(-1, 4)
                                                for i in range(k + m)]) for s in range(S)])).to(dev)
    errors = []

    def worker(t):
        try:
            st = torch.cuda.Stream(dev)
            for it in range(15):
                bent = data.copy()
                bad_stripes = list(range(t, S, 2 + it % 3))  # different patterns per thread / round
                for s in bad_stripes:
                    bent[s, 1 + t, (it * 97 + s) % cell] ^= 0x41
                with torch.cuda.stream(st):
                    d = torch.from_numpy(bent).to(dev)
                    p = torch.from_numpy(par).to(dev)
                    out = torch.zeros_like(d)
                    bad = H.decode_verify_batch(cod, d, p, [0], sums, out, stream=st)
                st.synchronize()
                b = bad.cpu().numpy()
                want = np.zeros((S, k + m), dtype=np.uint8)
                want[bad_stripes, 1 + t] = 1
                o = out.cpu().numpy()
                if not np.array_equal(b, want) or not np.array_equal(o[:, 0], data[:, 0]):
                    errors.append((t, it, "flags/rebuilt"))
                if not all(np.array_equal(o[s, 1 + t], data[s, 1 + t]) for s in bad_stripes):
                    errors.append((t, it, "repair"))
        except Exception as e:  # surfaced below
            errors.append(repr(e))

    ths = [threading.Thread(target=worker, args=(t,)) for t in range(2)]
    for th in ths:
        th.start()
    for th in ths:
        th.join(timeout=100)
    cod.close()
    assert not errors, errors[:5]
