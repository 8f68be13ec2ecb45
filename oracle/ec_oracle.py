"""Pure-Python / numpy twin of the C oracle (oracle/ec_oracle.c).

TEST INFRASTRUCTURE ONLY -- imported by tests/, __graft_entry__.smoke() and
bench.py's cpu_baseline leg as the checker; never by the shipped library.

Restates hdfs-native 0.14.1's EC path (read-only reference, Rust):
  rust/src/ec/gf256.rs:7        field GF(2^8), modulus 0x11D (g2p 1.2.2, not vendored)
  rust/src/ec/gf256.rs:40-57    Coder::gen_rs_matrix (Hadoop Cauchy matrix)
  rust/src/ec/gf256.rs:61-80    Coder::encode
  rust/src/ec/gf256.rs:84-137   Coder::decode (first-k-present survivors)
  rust/src/ec/matrix.rs:74-84   Matrix::select_rows (ascending original order)
  rust/src/ec/matrix.rs:101-162 Matrix::invert (Gauss-Jordan)
  rust/src/ec/matrix.rs:204-231 Mul<&[&[u8]]> (the hot loop)
  rust/src/ec/mod.rs:62-89      EcSchema::ec_decode
  rust/src/ec/mod.rs:93-144     resolve_ec_policy
  rust/src/hdfs/block_writer.rs:817-851  CellBuffer::encode padding semantics
  rust/src/hdfs/connection.rs:37-38, :477-504, :568-584  chunk checksums
      (crc 3.4.0 / crc-catalog 2.4.0, Cargo.lock:375-387, not vendored:
      CRC_32_ISCSI and CRC_32_CKSUM restated from their published parameters)
  rust/src/hdfs/block_reader.rs:480-525  read_slice: a cell whose packet
      fails its checksum drops that reader; the next parity reader is read

Pinning: tests/test_oracle.py checks this module and the C oracle against the
reference's own KATs (gf256.rs:144-202, mod.rs:152-160) and against each other.
"""
from __future__ import annotations

import ctypes
import os
from typing import List, Optional, Sequence

import numpy as np

POLY = 0x11D

EXP = [0] * 512
LOG = [0] * 256
_x = 1
for _i in range(255):
    EXP[_i] = _x
    LOG[_x] = _i
    _x <<= 1
    if _x & 0x100:
        _x ^= POLY
for _i in range(255, 512):
    EXP[_i] = EXP[_i - 255]


def gf_mul(a: int, b: int) -> int:
    if a == 0 or b == 0:
        return 0
    return EXP[LOG[a] + LOG[b]]


def gf_inv(a: int) -> int:
    if a == 0:
        raise ZeroDivisionError("GF(2^8) inverse of 0")
    return EXP[255 - LOG[a]]


def gf_div(a: int, b: int) -> int:
    return gf_mul(a, gf_inv(b))


# 256x256 product table for vectorised numpy multiply
MUL_TABLE = np.zeros((256, 256), dtype=np.uint8)
for _a in range(1, 256):
    for _b in range(1, 256):
        MUL_TABLE[_a, _b] = EXP[LOG[_a] + LOG[_b]]


def gen_rs_matrix(k: int, m: int) -> List[List[int]]:
    """gf256.rs:40-57: identity on top, row r>=k col c<k = 1/(r^c)."""
    mat = [[0] * k for _ in range(k + m)]
    for r in range(k):
        mat[r][r] = 1
    for r in range(k, k + m):
        for c in range(k):
            s = (r ^ c) & 0xFF
            mat[r][c] = 0 if s == 0 else gf_div(1, s)
    return mat


def gen_xor_matrix(k: int) -> List[List[int]]:
    """Hadoop XOR-k-1 (XORRawEncoder): parity = XOR of the data units."""
    return [[1 if i == j else 0 for j in range(k)] for i in range(k)] + [[1] * k]


# ---- rs-legacy (policy 3) -------------------------------
# The reference resolves RS-LEGACY-6-3-1024k (ec/mod.rs:118-124) but has no
# coder for it (mod.rs:69-78 decodes "rs" only), and Hadoop's Java coder is
# not under /root/reference.  Restated from Hadoop 3.x (published source):
#   RSUtil.getPrimitivePower  primitivePower[i] = GF.power(2, i)
#   RSRawEncoderLegacy.<init> gen = prod_{i<m} (primitivePower[i] + x)
#                             (GaloisField.multiply on coefficient arrays,
#                              index = degree)
#   RSRawEncoderLegacy.doEncode  all = [parity units (zeroed), data units];
#                             GaloisField.remainder(all, gen)
#   GaloisField.remainder     long division, highest degree first
# PARITY UNPINNED: no reference-held vector exists for this codec; tests pin
# it by the code's defining property (every codeword vanishes at 2^0..2^(m-1))
# and by this long division, which is independent of the matrix form.

def _poly_mul(p: Sequence[int], q: Sequence[int]) -> List[int]:
    """GaloisField.multiply(int[] p, int[] q): coefficient index = degree."""
    out = [0] * (len(p) + len(q) - 1)
    for i, a in enumerate(p):
        for j, b in enumerate(q):
            out[i + j] ^= gf_mul(a, b)
    return out


def legacy_generator(m: int) -> List[int]:
    """RSRawEncoderLegacy generating polynomial, lowest degree first, monic."""
    gen = [1]
    for i in range(m):
        gen = _poly_mul(gen, [EXP[i % 255], 1])
    return gen


def legacy_remainder(dividend: List[np.ndarray], divisor: Sequence[int]) -> None:
    """GaloisField.remainder(byte[][] dividend, int[] divisor), in place:
    for i from len(dividend)-len(divisor) down to 0, for every j, unit i+j
    ^= (unit[i+deg] / divisor[deg]) * divisor[j] (bytewise)."""
    deg = len(divisor) - 1
    inv_top = gf_inv(divisor[deg])
    for i in range(len(dividend) - len(divisor), -1, -1):
        ratio = MUL_TABLE[inv_top][dividend[i + deg]].copy()  # read before j = deg zeroes it
        for j in range(len(divisor)):
            if divisor[j]:
                dividend[i + j] ^= MUL_TABLE[divisor[j]][ratio]


def legacy_encode(k: int, m: int, data: Sequence[np.ndarray]) -> List[np.ndarray]:
    """RSRawEncoderLegacy.doEncode: parity unit j = coefficient j of
    (sum_i data_i x^(m+i)) mod gen."""
    assert len(data) == k
    n = len(data[0])
    allu = [np.zeros(n, dtype=np.uint8) for _ in range(m)] + [np.array(d, dtype=np.uint8) for d in data]
    legacy_remainder(allu, legacy_generator(m))
    return allu[:m]


def gen_rs_legacy_matrix(k: int, m: int) -> List[List[int]]:
    """(k+m) x k matrix of the legacy code: identity, then parity row j,
    column i = legacy_encode of the unit vector e_i (the code is linear)."""
    mat = [[1 if i == j else 0 for j in range(k)] for i in range(k)] + [[0] * k for _ in range(m)]
    for c in range(k):
        unit = [np.array([1 if i == c else 0], dtype=np.uint8) for i in range(k)]
        par = legacy_encode(k, m, unit)
        for j in range(m):
            mat[k + j][c] = int(par[j][0])
    return mat


def codec_matrix(codec: str, k: int, m: int) -> List[List[int]]:
    if codec == "xor":
        return gen_xor_matrix(k)
    if codec == "rs-legacy":
        return gen_rs_legacy_matrix(k, m)
    if codec == "rs":
        return gen_rs_matrix(k, m)
    raise NotImplementedError(f"codec: {codec}")


def poly_eval_units(units: Sequence[np.ndarray], x: int) -> np.ndarray:
    """Evaluates sum_d units[d] * x^d bytewise (Horner, highest degree first)."""
    acc = np.zeros(len(units[0]), dtype=np.uint8)
    for u in reversed(units):
        acc = MUL_TABLE[x][acc] ^ np.asarray(u, dtype=np.uint8)
    return acc


def select_rows(mat: List[List[int]], rows) -> List[List[int]]:
    """matrix.rs:74-84 -- HashSet filter: rows come out in ORIGINAL order."""
    keep = set(rows)
    return [row[:] for i, row in enumerate(mat) if i in keep]


def invert(mat: List[List[int]]) -> List[List[int]]:
    """matrix.rs:101-162, including the swap-with-every-later-nonzero-row loop."""
    n = len(mat)
    if any(len(r) != n for r in mat):
        raise ValueError("Cannot invert a non-square matrix")
    a = [row[:] + [1 if i == j else 0 for j in range(n)] for i, row in enumerate(mat)]
    w = 2 * n
    for r in range(n):
        if a[r][r] == 0:
            for rs in range(r + 1, n):
                if a[rs][r] != 0:
                    a[r], a[rs] = a[rs], a[r]
        if a[r][r] == 0:
            raise ArithmeticError("Matrix is singular")
        if a[r][r] != 1:
            scale = gf_div(1, a[r][r])
            a[r] = [gf_mul(v, scale) for v in a[r]]
        for rb in range(r + 1, n):
            scale = a[rb][r]
            if scale:
                a[rb] = [a[rb][c] ^ gf_mul(a[r][c], scale) for c in range(w)]
    for r in range(1, n):
        for ra in range(r):
            scale = a[ra][r]
            if scale:
                a[ra] = [a[ra][c] ^ gf_mul(a[r][c], scale) for c in range(w)]
    return [row[n:] for row in a]


def matmul(a: List[List[int]], b: List[List[int]]) -> List[List[int]]:
    """matrix.rs:181-199."""
    out = []
    for row in a:
        orow = []
        for j in range(len(b[0])):
            acc = 0
            for t in range(len(b)):
                acc ^= gf_mul(row[t], b[t][j])
            orow.append(acc)
        out.append(orow)
    return out


def identity(n: int) -> List[List[int]]:
    return [[1 if i == j else 0 for j in range(n)] for i in range(n)]


def matmul_shards(mat: List[List[int]], shards: Sequence[np.ndarray]) -> List[np.ndarray]:
    """matrix.rs:204-231 (i -> j -> byte order), vectorised over bytes."""
    n = len(shards[0])
    assert all(len(s) == n for s in shards)
    out = [np.zeros(n, dtype=np.uint8) for _ in mat]
    for i, src in enumerate(shards):
        src = np.asarray(src, dtype=np.uint8)
        for j, row in enumerate(mat):
            c = row[i]
            if c:
                out[j] ^= MUL_TABLE[c][src]
    return out


def encode(k: int, m: int, data: Sequence[np.ndarray]) -> List[np.ndarray]:
    """gf256.rs:61-80."""
    assert len(data) == k
    n = len(data[0])
    assert all(len(d) == n for d in data)
    mat = select_rows(gen_rs_matrix(k, m), range(k, k + m))
    return matmul_shards(mat, data)


class NotEnoughShards(Exception):
    """HdfsError::ErasureCodingError("Not enough valid shards") (gf256.rs:107-111)."""


def decode_plan(k: int, m: int, present: Sequence[bool], codec: str = "rs"):
    """Returns (survivors, missing_data, decode_matrix) per gf256.rs:84-126."""
    valid, invalid = [], []
    for i, p in enumerate(present):
        if p:
            valid.append(i)
        elif i < k:
            invalid.append(i)
    if not invalid:
        return [], [], []
    if len(valid) < k:
        raise NotEnoughShards("Not enough valid shards")
    surv = valid[:k]
    enc = codec_matrix(codec, k, m)
    dm = invert(select_rows(enc, surv))
    dm = select_rows(dm, invalid)
    return surv, invalid, dm


def decode(k: int, m: int, shards: List[Optional[np.ndarray]]) -> List[Optional[np.ndarray]]:
    """gf256.rs:84-137: fills missing DATA slots in a copy of `shards`."""
    assert len(shards) == k + m
    surv, miss, dm = decode_plan(k, m, [s is not None for s in shards])
    res = list(shards)
    if not miss:
        return res
    rec = matmul_shards(dm, [shards[i] for i in surv])
    for idx, arr in zip(miss, rec):
        res[idx] = arr
    return res


# ---- EcSchema-level helpers (mod.rs / block_writer.rs) --------------------

POLICIES = {  # mod.rs:93-144
    1: ("rs", 6, 3, 1024 * 1024),
    2: ("rs", 3, 2, 1024 * 1024),
    3: ("rs-legacy", 6, 3, 1024 * 1024),
    4: ("xor", 2, 1, 1024 * 1024),
    5: ("rs", 10, 4, 1024 * 1024),
}


def max_offset(k: int, cell: int, index: int, block_size: int) -> int:
    """mod.rs:40-60: bytes of block `index` (parity -> as block 0) in a block
    group holding block_size bytes of file data."""
    if index >= k:
        index = 0
    row = cell * k
    full_rows = block_size // row
    remaining = block_size - full_rows * row
    if remaining < index * cell:
        last = 0
    elif remaining > (index + 1) * cell:
        last = cell
    else:
        last = remaining - index * cell
    return full_rows * cell + last


def cell_buffer_encode(k: int, m: int, cells: Sequence[bytes]) -> List[bytes]:
    """block_writer.rs:817-851: pad every buffer to len(buffers[0]) with 0,
    encode, truncate data back, append parity."""
    size = len(cells[0])
    padded = [np.frombuffer(bytes(c) + b"\0" * (size - len(c)), dtype=np.uint8) for c in cells]
    parity = encode(k, m, padded)
    return [bytes(c) for c in cells] + [p.tobytes() for p in parity]


def cell_buffer_rows(data: bytes, k: int, cell: int) -> List[List[bytes]]:
    """block_writer.rs:791-805 + StripedBlockWriter's close: the file bytes
    split into rows of k cell buffers, buffer i of a row filled to `cell`
    before buffer i+1; the last row may be partial (short or empty buffers)."""
    rows, row = [], k * cell
    for start in range(0, len(data), row):
        chunk = data[start:start + row]
        rows.append([chunk[i * cell:(i + 1) * cell] for i in range(k)])
    return rows


def striped_write(data: bytes, k: int, m: int, cell: int) -> List[List[bytes]]:
    """What the striped writer emits per row: CellBuffer::encode's k data
    cells (unpadded) + m parity cells of len(buffers[0]) bytes."""
    return [cell_buffer_encode(k, m, r) for r in cell_buffer_rows(data, k, cell)]


def vertical_buffers(rows: List[List[bytes]], k: int, m: int) -> List[bytes]:
    """Per shard: its cells in row order, i.e. the block each of the k+m
    single-replica writers stores (its length is max_offset, mod.rs:40-60)."""
    return [b"".join(r[i] for r in rows) for i in range(k + m)]


def striped_read(vertical: List[Optional[bytes]], k: int, m: int, cell: int, file_len: int) -> bytes:
    """The read side over whole rows (block_reader.rs:480-554): every cell a
    CellReader returns is zero-padded to cell_size (:343-378; a missing tail
    is all zeros), ec_decode per row (mod.rs:62-89), cells concatenated in
    file order, trimmed to the file length."""
    rows = -(-file_len // (k * cell))
    out = []
    for r in range(rows):
        cells = []
        for i in range(k + m):
            v = vertical[i]
            if v is None:
                cells.append(None)
            else:
                c = v[r * cell:(r + 1) * cell]
                cells.append(c + b"\0" * (cell - len(c)))
        out.extend(ec_decode(k, m, cell, "rs", cells))
    return b"".join(out)[:file_len]


def ec_decode(k: int, m: int, cell_size: int, codec: str,
              vertical: List[Optional[bytes]]) -> List[bytes]:
    """mod.rs:62-89: decode when a data shard is missing, then split each data
    shard into cell_size cells in row order."""
    vs = list(vertical)
    if not all(v is not None or i >= k for i, v in enumerate(vs)):
        if codec != "rs":
            raise NotImplementedError(f"codec: {codec}")
        arrs = [None if v is None else np.frombuffer(v, dtype=np.uint8) for v in vs]
        arrs = decode(k, m, arrs)
        vs = [None if a is None else a.tobytes() for a in arrs]
    cells = []
    offs = [0] * k
    while vs[0] is not None and offs[0] < len(vs[0]):
        for i in range(k):
            if offs[i] + cell_size > len(vs[i]):  # Bytes::split_to panics (mod.rs:84)
                raise ValueError("split_to out of bounds")
            cells.append(vs[i][offs[i]:offs[i] + cell_size])
            offs[i] += cell_size
    return cells


# ---- CRC32C per checksum chunk (connection.rs:37-38, :568-584) ------------

def _crc32c_table():
    t = []
    for i in range(256):
        c = i
        for _ in range(8):
            c = (c >> 1) ^ (0x82F63B78 if c & 1 else 0)
        t.append(c)
    return t


CRC32C_TABLE = _crc32c_table()


def crc32c(data: bytes) -> int:
    """CRC-32C (iSCSI): reflected 0x82F63B78, init/xorout 0xFFFFFFFF."""
    crc = 0xFFFFFFFF
    for b in bytes(data):
        crc = CRC32C_TABLE[(crc ^ b) & 0xFF] ^ (crc >> 8)
    return crc ^ 0xFFFFFFFF


def chunk_crc32c(data: bytes, bytes_per_checksum: int) -> bytes:
    """WritePacket::calculate_checksum: one big-endian u32 per chunk."""
    out = bytearray()
    data = bytes(data)
    for start in range(0, len(data), bytes_per_checksum):
        out += crc32c(data[start:start + bytes_per_checksum]).to_bytes(4, "big")
    return bytes(out)


# CRC_32_CKSUM (crc-catalog: width 32, poly 0x04C11DB7, init 0, refin/refout
# false, xorout 0xFFFFFFFF, check 0x765E7680): the reference's "CRC32"
# (connection.rs:37), used for ChecksumTypeProto CHECKSUM_CRC32 on read.
def _cksum_table():
    t = []
    for i in range(256):
        c = i << 24
        for _ in range(8):
            c = ((c << 1) ^ 0x04C11DB7 if c & 0x80000000 else c << 1) & 0xFFFFFFFF
        t.append(c)
    return t


CKSUM_TABLE = _cksum_table()


def crc32_cksum(data: bytes) -> int:
    """CRC-32/CKSUM: MSB-first 0x04C11DB7, init 0, xorout 0xFFFFFFFF."""
    crc = 0
    for b in bytes(data):
        crc = CKSUM_TABLE[((crc >> 24) ^ b) & 0xFF] ^ ((crc << 8) & 0xFFFFFFFF)
    return crc ^ 0xFFFFFFFF


CHECKSUM_NULL, CHECKSUM_CRC32, CHECKSUM_CRC32C = 0, 1, 2  # ChecksumTypeProto (hadoop.hdfs.rs:1363)
_ALGO = {CHECKSUM_CRC32: crc32_cksum, CHECKSUM_CRC32C: crc32c}


def chunk_checksums(data: bytes, bytes_per_checksum: int, checksum_type: int = CHECKSUM_CRC32C) -> bytes:
    """One big-endian u32 per bytes_per_checksum chunk (last may be short)."""
    algo = _ALGO[checksum_type]
    data = bytes(data)
    return b"".join(algo(data[s:s + bytes_per_checksum]).to_bytes(4, "big")
                    for s in range(0, len(data), bytes_per_checksum))


def get_data_ok(data: bytes, sums: bytes, bytes_per_checksum: int, checksum_type: int) -> bool:
    """ReadPacket::get_data (connection.rs:477-504): False = ChecksumError."""
    if checksum_type == CHECKSUM_NULL:
        return True
    return chunk_checksums(data, bytes_per_checksum, checksum_type) == bytes(sums)


def verified_read_row(k: int, m: int, cells: List[Optional[bytes]], sums: List[bytes], bytes_per_checksum: int,
                      checksum_type: int):
    """One row of the striped read with verification (block_reader.rs:480-525
    then ec/mod.rs:62-89): cells are read in index order from the available
    shards (None = no reader); a cell that fails get_data drops its reader
    and the next shard is read, until k good cells are held.  Returns
    (data cells [k] as bytes, bad flags [k+m]); raises NotEnoughShards when
    fewer than k cells verify."""
    bad = [0] * (k + m)
    good: List[Optional[np.ndarray]] = [None] * (k + m)
    held = 0
    for i in range(k + m):
        if held == k:
            break
        if cells[i] is None:
            continue
        if get_data_ok(cells[i], sums[i], bytes_per_checksum, checksum_type):
            good[i] = np.frombuffer(bytes(cells[i]), dtype=np.uint8)
            held += 1
        else:
            bad[i] = 1
    if held < k:
        raise NotEnoughShards("Not enough valid shards")
    full = decode(k, m, good)
    return [full[i].tobytes() for i in range(k)], bad


# ---- ctypes access to the C oracle ----------------------------------------

_HERE = os.path.dirname(os.path.abspath(__file__))
C_LIB_PATH = os.path.join(_HERE, "build", "liboracle_ec.so")


def load_c_oracle() -> ctypes.CDLL:
    lib = ctypes.CDLL(C_LIB_PATH)
    P = ctypes.c_void_p
    S = ctypes.c_size_t
    lib.orc_gf_mul.argtypes = [ctypes.c_uint8, ctypes.c_uint8]
    lib.orc_gf_mul.restype = ctypes.c_uint8
    lib.orc_gf_mul_slow.argtypes = [ctypes.c_uint8, ctypes.c_uint8]
    lib.orc_gf_mul_slow.restype = ctypes.c_uint8
    lib.orc_gen_rs_matrix.argtypes = [S, S, P]
    lib.orc_invert.argtypes = [P, S]
    lib.orc_encode.argtypes = [S, S, P, S, P]
    lib.orc_decode.argtypes = [S, S, P, S, P]
    lib.orc_encode_batch.argtypes = [S, S, P, S, S, P]
    lib.orc_decode_batch.argtypes = [S, S, P, P, S, S, ctypes.c_uint64, P]
    lib.orc_matmul_shards.argtypes = [P, S, S, P, S, P]
    lib.orc_decode_matrix.argtypes = [S, S, P, P, P, P]
    lib.orc_crc32c.argtypes = [P, S]
    lib.orc_crc32c.restype = ctypes.c_uint32
    lib.orc_chunk_crc32c.argtypes = [P, S, S, P]
    lib.orc_crc32_cksum.argtypes = [P, S]
    lib.orc_crc32_cksum.restype = ctypes.c_uint32
    lib.orc_chunk_checksum.argtypes = [ctypes.c_int, P, S, S, P]
    return lib


def _ptrs(arrs):
    return (ctypes.c_void_p * len(arrs))(*[0 if a is None else a.ctypes.data for a in arrs])


def c_check_batch(lib, k: int, m: int, data: np.ndarray, parity: np.ndarray, present: int = None,
                  rebuilt: np.ndarray = None, threads: int = 16) -> None:
    """Full-batch checker (test infrastructure): every stripe of an engine
    batch against the C restatement, stripe-parallel on `threads` host
    threads (ctypes releases the GIL).  data [S,k,cell], parity [S,m,cell]
    (the engine's); with `present` (bit i = shard i available) and rebuilt
    [S,e,cell] (the engine's decode, ascending missing data index) the C
    decode of the same survivors is compared too.  Raises AssertionError
    naming the first mismatching stripe."""
    import threading
    S, _, n = data.shape
    data = np.ascontiguousarray(data)
    parity = np.ascontiguousarray(parity)
    threads = max(1, min(threads, S))
    errors = []

    def work(t):
        a, b = S * t // threads, S * (t + 1) // threads
        if a == b:
            return
        want = np.empty((b - a, m, n), dtype=np.uint8)
        rc = lib.orc_encode_batch(k, m, data[a:b].ctypes.data, n, b - a, want.ctypes.data)
        if rc != 0 or not np.array_equal(want, parity[a:b]):
            bad = [s for s in range(a, b) if not np.array_equal(want[s - a], parity[s])][:1]
            errors.append(f"parity != oracle at stripe {bad}")
            return
        if present is not None and rebuilt is not None:
            e = rebuilt.shape[1]
            got = np.empty((b - a, e, n), dtype=np.uint8)
            rc = lib.orc_decode_batch(k, m, data[a:b].ctypes.data, parity[a:b].ctypes.data, n, b - a,
                                      ctypes.c_uint64(present), got.ctypes.data)
            if rc != 0 or not np.array_equal(got, rebuilt[a:b]):
                bad = [s for s in range(a, b) if not np.array_equal(got[s - a], rebuilt[s])][:1]
                errors.append(f"rebuilt != oracle decode at stripe {bad}")

    ths = [threading.Thread(target=work, args=(t,)) for t in range(threads)]
    for th in ths:
        th.start()
    for th in ths:
        th.join()
    assert not errors, errors


def c_encode(lib, k: int, m: int, data: Sequence[np.ndarray]) -> List[np.ndarray]:
    n = len(data[0])
    data = [np.ascontiguousarray(d, dtype=np.uint8) for d in data]
    par = [np.empty(n, dtype=np.uint8) for _ in range(m)]
    rc = lib.orc_encode(k, m, _ptrs(data), n, _ptrs(par))
    if rc != 0:
        raise RuntimeError(f"orc_encode rc={rc}")
    return par


def c_decode(lib, k: int, m: int, shards: List[Optional[np.ndarray]]):
    n = len(next(s for s in shards if s is not None))
    shards = [None if s is None else np.ascontiguousarray(s, dtype=np.uint8) for s in shards]
    out = [np.empty(n, dtype=np.uint8) if (i < k and shards[i] is None) else None for i in range(k + m)]
    rc = lib.orc_decode(k, m, _ptrs(shards), n, _ptrs(out))
    if rc == -2:
        raise NotEnoughShards("Not enough valid shards")
    if rc != 0:
        raise RuntimeError(f"orc_decode rc={rc}")
    return [shards[i] if out[i] is None else out[i] for i in range(k + m)]
