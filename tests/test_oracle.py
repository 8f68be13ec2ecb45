"""Pins the CPU oracle (oracle/) against the reference's own known-answer
tests and checks the C and Python restatements agree.  CPU only."""
import itertools

import numpy as np
import pytest

import ec_oracle as O
from hdfs_native_ec.synth import bench_counter_shards, splitmix64_bytes

# rust/src/ec/gf256.rs:144-192 -- "taken directly from the matrices created
# by Hadoop via RSUtil.genCauchyMatrix" (parity rows; identity rows above).
KAT_PARITY_ROWS = {
    (3, 2): [[244, 142, 1], [71, 167, 122]],
    (6, 3): [[122, 186, 71, 167, 142, 244], [186, 122, 167, 71, 244, 142],
             [173, 157, 221, 152, 61, 170]],
    (10, 4): [[221, 152, 173, 157, 93, 150, 61, 170, 142, 244],
              [152, 221, 157, 173, 150, 93, 170, 61, 244, 142],
              [61, 170, 93, 150, 173, 157, 221, 152, 71, 167],
              [170, 61, 150, 93, 157, 173, 152, 221, 167, 71]],
}


@pytest.mark.parametrize("k,m", list(KAT_PARITY_ROWS))
def test_gen_rs_matrix_kat_python(k, m):
    mat = O.gen_rs_matrix(k, m)
    assert mat[:k] == O.identity(k)
    assert mat[k:] == KAT_PARITY_ROWS[(k, m)]


@pytest.mark.parametrize("k,m", list(KAT_PARITY_ROWS))
def test_gen_rs_matrix_kat_c(c_oracle, k, m):
    buf = np.zeros((k + m) * k, dtype=np.uint8)
    assert c_oracle.orc_gen_rs_matrix(k, m, buf.ctypes.data) == 0
    mat = buf.reshape(k + m, k).tolist()
    assert mat[:k] == O.identity(k)
    assert mat[k:] == KAT_PARITY_ROWS[(k, m)]


def test_invert_kat_gf256_rs():
    # gf256.rs:194-202: rows {2,3,4} of RS(3,2); M^-1 * M == I
    mat = O.select_rows(O.gen_rs_matrix(3, 2), [2, 3, 4])
    assert O.matmul(O.invert(mat), mat) == O.identity(3)


def test_invert_kat_mod_rs():
    # ec/mod.rs:152-160
    mat = [[0, 0, 1], [244, 142, 1], [71, 167, 122]]
    assert O.matmul(O.invert(mat), mat) == O.identity(3)


def test_invert_bench_matrix():
    # benches/ec.rs:6-14 inverts rows 3..8 of RS(6,3)
    mat = O.select_rows(O.gen_rs_matrix(6, 3), range(3, 9))
    inv = O.invert(mat)
    assert O.matmul(inv, mat) == O.identity(6)
    # survey probe: missing {0,1,2} decode rows
    assert inv[:3] == [[130, 54, 212, 144, 144, 72], [213, 42, 96, 216, 214, 112], [153, 30, 142, 68, 72, 48]]


def test_c_invert_matches_python(c_oracle):
    for k, m in KAT_PARITY_ROWS:
        for rows in itertools.combinations(range(k + m), k):
            sub = O.select_rows(O.gen_rs_matrix(k, m), rows)
            buf = np.array(sub, dtype=np.uint8).ravel().copy()
            assert c_oracle.orc_invert(buf.ctypes.data, k) == 0
            assert buf.reshape(k, k).tolist() == O.invert(sub)
            if k == 10:
                break  # 1001 combos of 10x10 in pure python is slow; one is enough here


def test_select_rows_keeps_original_order():
    # matrix.rs:74-84 filters through a HashSet: order of the iterator is ignored
    mat = O.gen_rs_matrix(3, 2)
    assert O.select_rows(mat, [4, 0, 2]) == [mat[0], mat[2], mat[4]]


def test_singular_raises():
    with pytest.raises(ArithmeticError):
        O.invert([[1, 1], [1, 1]])


def test_gf_mul_tables_vs_bitserial(c_oracle):
    for a in range(256):
        for b in range(0, 256, 7):
            assert c_oracle.orc_gf_mul(a, b) == c_oracle.orc_gf_mul_slow(a, b) == O.gf_mul(a, b)


def test_field_axioms():
    for a in range(1, 256):
        assert O.gf_mul(a, O.gf_inv(a)) == 1
    # distributivity on a sample
    rng = np.random.default_rng(1)
    for a, b, c in rng.integers(0, 256, size=(500, 3)):
        assert O.gf_mul(int(a), int(b) ^ int(c)) == O.gf_mul(int(a), int(b)) ^ O.gf_mul(int(a), int(c))


@pytest.mark.parametrize("k,m", [(3, 2), (6, 3), (10, 4), (2, 1), (4, 4)])
def test_c_and_python_encode_agree(c_oracle, k, m):
    for n in (1, 15, 17, 257, 4093):
        data = splitmix64_bytes(77 + n, k * n).reshape(k, n)
        py = O.encode(k, m, list(data))
        c = O.c_encode(c_oracle, k, m, list(data))
        for a, b in zip(py, c):
            assert np.array_equal(a, b)


@pytest.mark.parametrize("k,m", [(3, 2), (6, 3), (10, 4)])
def test_decode_roundtrip_all_patterns(c_oracle, k, m):
    n = 61
    data = splitmix64_bytes(5 + k, k * n).reshape(k, n)
    par = O.encode(k, m, list(data))
    full = list(data) + par
    for e in range(0, m + 2):
        for miss in itertools.combinations(range(k + m), e):
            shards = [None if i in miss else full[i] for i in range(k + m)]
            n_present = k + m - e
            data_missing = any(i < k for i in miss)
            if data_missing and n_present < k:
                with pytest.raises(O.NotEnoughShards):
                    O.decode(k, m, shards)
                with pytest.raises(O.NotEnoughShards):
                    O.c_decode(c_oracle, k, m, shards)
                continue
            res = O.decode(k, m, shards)
            resc = O.c_decode(c_oracle, k, m, shards)
            for i in range(k):
                assert np.array_equal(res[i], data[i])
                assert np.array_equal(resc[i], data[i])
            # missing parity is never regenerated (gf256.rs:96-97)
            for i in range(k, k + m):
                if i in miss:
                    assert res[i] is None
            if k == 10 and e >= 3:
                break


def test_decode_uses_first_k_present():
    # gf256.rs:90-95: survivors are the first k present in index order
    surv, miss, dm = O.decode_plan(3, 2, [False, True, True, True, True])
    assert surv == [1, 2, 3] and miss == [0]


def test_golden_vectors_match_oracle(golden, c_oracle):
    manifest, arrays = golden
    for case in manifest["cases"]:
        key, k, m = case["key"], case["k"], case["m"]
        data = arrays[key + "_data"]
        par = arrays[key + "_parity"]
        got = O.c_encode(c_oracle, k, m, list(data))
        assert all(np.array_equal(a, b) for a, b in zip(got, par)), key
    for k, m in [(3, 2), (6, 3), (10, 4)]:
        for plan in manifest[f"rs{k}_{m}_decode_plans"][:50]:
            present = [i not in plan["missing"] for i in range(k + m)]
            surv, miss, dm = O.decode_plan(k, m, present)
            assert surv == plan["survivors"] and dm == plan["matrix"]


def test_bench_counter_fill():
    # rust/benches/ec.rs:19-27 big-endian i32 counter
    s = bench_counter_shards(2, 16)
    assert s[0].tolist() == [0, 0, 0, 0, 0, 0, 0, 1, 0, 0, 0, 2, 0, 0, 0, 3]
    assert s[1][:4].tolist() == [0, 0, 0, 16]


def test_cell_buffer_and_ec_decode_semantics():
    # block_writer.rs:817-851 pads to len(buffers[0]); mod.rs:62-89 splits cells
    k, m, cell = 3, 2, 8
    cells = [bytes(range(8)), bytes(range(10, 13)), b""]
    out = O.cell_buffer_encode(k, m, cells)
    assert [len(c) for c in out] == [8, 3, 0, 8, 8]
    vertical = [out[0], None, None, out[3], out[4]]
    # pad to cell size as CellReader::next_cell does (block_reader.rs:370-371)
    vertical = [None if v is None else v + b"\0" * (cell - len(v)) for v in vertical]
    cells_back = O.ec_decode(k, m, cell, "rs", vertical)
    assert cells_back[0] == bytes(range(8))
    assert cells_back[1][:3] == bytes(range(10, 13)) and cells_back[1][3:] == b"\0" * 5
    assert cells_back[2] == b"\0" * 8
    with pytest.raises(NotImplementedError):
        O.ec_decode(2, 1, cell, "xor", [None, b"\0" * 8, b"\0" * 8])


def test_xor_codec_oracle():
    # Hadoop XOR-2-1: parity = d0 ^ d1; any single loss is the XOR of the rest
    k = 2
    data = [np.array([1, 2, 250], dtype=np.uint8), np.array([7, 9, 5], dtype=np.uint8)]
    par = O.matmul_shards(O.gen_xor_matrix(k)[k:], data)[0]
    assert par.tolist() == [1 ^ 7, 2 ^ 9, 250 ^ 5]
    for lost in range(k):
        present = [i != lost for i in range(k + 1)]
        surv, miss, dm = O.decode_plan(k, 1, present, codec="xor")
        shards = data + [par]
        rec = O.matmul_shards(dm, [shards[i] for i in surv])[0]
        assert np.array_equal(rec, data[lost])


# CRC-32C/iSCSI published vectors: catalogue check value and RFC 3720 B.4
CRC32C_VECTORS = [
    (b"123456789", 0xE3069283),
    (bytes(32), 0x8A9136AA),
    (b"\xff" * 32, 0x62A8AB43),
    (bytes(range(32)), 0x46DD794E),
    (bytes(range(31, -1, -1)), 0x113FDB5C),
]


@pytest.mark.parametrize("data,want", CRC32C_VECTORS)
def test_crc32c_published_vectors(c_oracle, data, want):
    assert O.crc32c(data) == want
    buf = np.frombuffer(data, dtype=np.uint8).copy()
    assert c_oracle.orc_crc32c(buf.ctypes.data, len(data)) == want


def test_chunk_crc32c_c_vs_python(c_oracle):
    for n in (1, 511, 512, 513, 4096, 5000):
        data = splitmix64_bytes(n, n)
        for bpc in (512, 4096, 100):
            out = np.zeros(((n + bpc - 1) // bpc) * 4, dtype=np.uint8)
            c_oracle.orc_chunk_crc32c(data.ctypes.data, n, bpc, out.ctypes.data)
            assert out.tobytes() == O.chunk_crc32c(data.tobytes(), bpc)


# ---- CRC32 = CRC_32_CKSUM (connection.rs:37) and the verified read --------

def test_crc32_cksum_catalog_check(c_oracle):
    """crc-catalog 2.4.0 CRC_32_CKSUM check value."""
    assert O.crc32_cksum(b"123456789") == 0x765E7680
    buf = np.frombuffer(b"123456789", dtype=np.uint8).copy()
    assert c_oracle.orc_crc32_cksum(buf.ctypes.data, 9) == 0x765E7680


def test_crc32_cksum_vs_posix_cksum_fixtures():
    """POSIX cksum (coreutils, tests/golden/make_cksum.py) = CRC_32_CKSUM of
    the message followed by its length, little-endian, minimal bytes."""
    import json
    import os
    with open(os.path.join(os.path.dirname(__file__), "golden", "cksum_vectors.json")) as f:
        cases = json.load(f)["cases"]
    assert len(cases) >= 10
    for case in cases:
        data = bytes.fromhex(case["hex"])
        n, tail = len(data), b""
        while n:
            tail += bytes([n & 0xFF])
            n >>= 8
        assert O.crc32_cksum(data + tail) == case["posix_cksum"]


@pytest.mark.parametrize("ctype", [O.CHECKSUM_CRC32, O.CHECKSUM_CRC32C])
def test_chunk_checksum_c_vs_python(c_oracle, ctype):
    for n in (1, 511, 512, 513, 4096, 5000):
        data = splitmix64_bytes(n + 7, n)
        for bpc in (512, 4096, 100):
            out = np.zeros(((n + bpc - 1) // bpc) * 4, dtype=np.uint8)
            c_oracle.orc_chunk_checksum(ctype, data.ctypes.data, n, bpc, out.ctypes.data)
            assert out.tobytes() == O.chunk_checksums(data.tobytes(), bpc, ctype)


def test_verified_read_row_semantics():
    """block_reader.rs:480-525: a failing cell is skipped and the next shard
    read; all data rebuilt; too many failures -> Not enough valid shards."""
    k, m, n, bpc = 6, 3, 2048, 512
    data = [splitmix64_bytes(100 + i, n) for i in range(k)]
    cells = [d.tobytes() for d in data] + [p.tobytes() for p in O.encode(k, m, data)]
    sums = [O.chunk_checksums(c, bpc, O.CHECKSUM_CRC32C) for c in cells]
    # clean read: nothing bad
    out, bad = O.verified_read_row(k, m, list(cells), sums, bpc, O.CHECKSUM_CRC32C)
    assert out == cells[:k] and bad == [0] * (k + m)
    # data cell 2 corrupted, data 4 unavailable: parity 0 and 1 are read
    bent = list(cells)
    bent[2] = bent[2][:700] + bytes([bent[2][700] ^ 1]) + bent[2][701:]
    bent[4] = None
    out, bad = O.verified_read_row(k, m, bent, sums, bpc, O.CHECKSUM_CRC32C)
    assert out == cells[:k] and bad == [0, 0, 1, 0, 0, 0, 0, 0, 0]
    # parity never read when not needed: corrupt parity 2 is not flagged
    bent2 = list(bent)
    bent2[8] = bytes(n)
    _, bad = O.verified_read_row(k, m, bent2, sums, bpc, O.CHECKSUM_CRC32C)
    assert bad[8] == 0
    # m+1 cells lost or failed -> error
    bent2[6] = bytes(n)
    with pytest.raises(O.NotEnoughShards):
        O.verified_read_row(k, m, bent2, sums, bpc, O.CHECKSUM_CRC32C)
    # CHECKSUM_NULL verifies nothing: the corrupt cell is used as read
    out, bad = O.verified_read_row(k, m, bent, sums, bpc, O.CHECKSUM_NULL)
    assert bad == [0] * (k + m)
    assert out[2] == bent[2] and out[4] != cells[4]


def test_device_crc_tables_vs_oracle(tmp_path):
    """The compile-time tables the CRC kernels read (csrc/checksum_tables.hpp)
    recombined on the host with the kernels' own algebra (slicing-by-8,
    11-bit and folded quarters placed by zero-append tables, plus the
    byte-serial tail slot) give the oracle's per-512-B-chunk CRC32C and CRC32 bit for bit."""
    import os
    import shutil
    import subprocess
    gxx = shutil.which("g++")
    if gxx is None:
        pytest.skip("g++ not available")
    src = os.path.join(os.path.dirname(__file__), "cpp", "crc_tables_check.cpp")
    exe = str(tmp_path / "crc_tables_check")
    subprocess.run([gxx, "-std=c++17", "-O2", "-o", exe, src], check=True)
    chunks = 24
    res = subprocess.run([exe, "0x5eed", str(chunks)], check=True, capture_output=True)
    data = res.stderr
    assert len(data) == 512 * chunks
    lines = res.stdout.decode().split()
    assert len(lines) == 10 * chunks
    for i in range(chunks):
        c = data[512 * i:512 * (i + 1)]
        want32c = O.chunk_checksums(c, 512, O.CHECKSUM_CRC32C).hex()
        want32 = O.chunk_checksums(c, 512, O.CHECKSUM_CRC32).hex()
        row = lines[10 * i:10 * i + 10]
        # s8, w11, byte, fold 24 (scheme 12), fold 16 / 20 (measurement schemes 13 / 14),
        # fold 24 + slicing-by-32 tail (measurement scheme 15)
        assert row[0:3] + row[6:10] == [want32c] * 7, i
        assert row[3:6] == [want32] * 3, i


# ---- rs-legacy (Hadoop RSRawEncoderLegacy; parity unpinned, see oracle) ----

@pytest.mark.parametrize("k,m", [(6, 3), (3, 2), (10, 4), (2, 1), (20, 10)])
def test_legacy_codewords_vanish_at_generator_roots(k, m):
    # the defining property of the legacy code: the codeword polynomial
    # (parity j at degree j, data i at degree m+i) is a multiple of
    # g(x) = prod_{i<m} (x + 2^i), so it vanishes at 2^0 .. 2^(m-1)
    rng = np.random.default_rng(100 + k)
    data = [rng.integers(0, 256, 333, dtype=np.uint8) for _ in range(k)]
    par = O.legacy_encode(k, m, data)
    for i in range(m):
        assert not O.poly_eval_units(par + data, O.EXP[i]).any()
    # and the long division equals the matrix form the engine runs
    mat = O.gen_rs_legacy_matrix(k, m)
    want = O.matmul_shards(O.select_rows(mat, range(k, k + m)), data)
    assert all(np.array_equal(a, b) for a, b in zip(par, want))


def test_legacy_generator_small_cases():
    # g for m = 1 is x + 1 (parity = XOR of the data, as Hadoop's legacy
    # coder with one parity unit); m = 2: (x + 1)(x + 2) = x^2 + 3x + 2
    assert O.legacy_generator(1) == [1, 1]
    assert O.legacy_generator(2) == [2, 3, 1]
    assert O.gen_rs_legacy_matrix(4, 1)[4] == [1, 1, 1, 1]


def test_legacy_decode_plan_round_trip():
    k, m = 6, 3
    rng = np.random.default_rng(7)
    data = [rng.integers(0, 256, 64, dtype=np.uint8) for _ in range(k)]
    shards = data + O.legacy_encode(k, m, data)
    for lost in itertools.combinations(range(k + m), m):
        present = [i not in lost for i in range(k + m)]
        surv, miss, dm = O.decode_plan(k, m, present, codec="rs-legacy")
        if not miss:
            continue
        rec = O.matmul_shards(dm, [shards[i] for i in surv])
        for idx, arr in zip(miss, rec):
            assert np.array_equal(arr, data[idx])


def test_striped_write_matches_reference_block_lengths():
    # the oracle's striped writer (CellBuffer::write / encode restated) leaves
    # every shard exactly max_offset(i) bytes (ec/mod.rs:40-60, the
    # reference's own block-length rule), and its striped read (CellReader
    # zero-padding + ec_decode + trim) returns the file for every lost set
    # of up to m shards
    import itertools

    import ec_oracle as O
    for k, m, cell in [(3, 2, 4096), (6, 3, 1024), (10, 4, 512)]:
        for L in [1, 16, cell - 4, cell, cell + 4, k * cell - 4, k * cell, 5 * k * cell - 4, 5 * k * cell + 4]:
            data = bytes((i * 131 + L) & 0xFF for i in range(L))
            vert = O.vertical_buffers(O.striped_write(data, k, m, cell), k, m)
            assert [len(v) for v in vert] == [O.max_offset(k, cell, i, L) for i in range(k + m)]
            for e in range(m + 1):
                for lost in list(itertools.combinations(range(k + m), e))[:6]:
                    v = [None if i in lost else vert[i] for i in range(k + m)]
                    assert O.striped_read(v, k, m, cell, L) == data, (k, m, L, lost)
