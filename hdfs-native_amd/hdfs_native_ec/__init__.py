"""ctypes binding of the MI355X EC engine's C ABI (include/hdfs_ec_amd.h).

Mirrors the reference's Rust surface so parity tests read like the
reference's own tests:

  hdfs_native::ec::gf256::Coder::new(data_units, parity_units)   gf256.rs:32-38
  Coder::gen_rs_matrix(k, m)                                     gf256.rs:40-57
  Coder::encode(&[Bytes]) -> Vec<Bytes>                          gf256.rs:61-80
  Coder::decode(&mut [Option<Bytes>]) -> Result<()>              gf256.rs:84-137

plus the batched device-resident entry points used by bench.py.  There is no
CPU fallback anywhere: if lib/libhdfs_ec_amd.so is missing or fails to load,
import raises.
"""
from __future__ import annotations

import ctypes
import os
from typing import List, Optional, Sequence

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("HEC_LIB_PATH") or os.path.join(os.path.dirname(_HERE), "lib", "libhdfs_ec_amd.so")
# HEC_LIB_PATH: another in-tree build of the engine, for same-box A/B measurements

HEC_OK = 0
HEC_ERR_INVALID_ARG = -1
HEC_ERR_NOT_ENOUGH_SHARDS = -2
HEC_ERR_UNSUPPORTED_CODEC = -3
HEC_ERR_DEVICE = -4
HEC_ERR_NO_MEMORY = -5
HEC_ERR_SINGULAR = -6
HEC_ERR_CHECKSUM = -7
HEC_DEVICE_HOST = -2  # host-only coder: the engine's host routine, no GPU needed

# ChecksumTypeProto values (rust/src/proto/hadoop.hdfs.rs:1363)
CHECKSUM_NULL = 0
CHECKSUM_CRC32 = 1   # crc CRC_32_CKSUM (connection.rs:37)
CHECKSUM_CRC32C = 2  # crc CRC_32_ISCSI (connection.rs:38)

# Every symbol include/hdfs_ec_amd.h declares (checked by tests/test_capi.py).
EXPORTS = [
    "hec_strerror", "hec_abi_version", "hec_last_error", "hec_gen_rs_matrix", "hec_matrix_invert",
    "hec_gen_codec_matrix",
    "hec_decode_plan", "hec_coder_create", "hec_coder_destroy", "hec_coder_data_units",
    "hec_coder_parity_units", "hec_coder_device", "hec_encode", "hec_decode",
    "hec_encode_device", "hec_decode_device", "hec_gf_matmul_device",
    "hec_encode_host_batch", "hec_decode_mixed_workspace_size",
    "hec_decode_device_mixed", "hec_coder_create_codec", "hec_decode_host_batch",
    "hec_crc32c_device", "hec_encode_crc_device", "hec_checksum_device", "hec_checksum_verify_device",
    "hec_decode_verify_device", "hec_group_create", "hec_group_destroy", "hec_group_size", "hec_group_coder",
    "hec_group_range", "hec_group_encode_host_batch", "hec_group_decode_host_batch", "hec_group_encode_device",
    "hec_group_decode_device",
    "hec_device_alloc", "hec_device_free", "hec_device_copy", "hec_device_synchronize", "hec_device_numa_node",
    "hec_host_alloc", "hec_host_free",
    "hec_coder_acquire", "hec_coder_release", "hec_coder_pool_trim", "hec_coder_set_host_limit",
    "hec_coder_host_limit", "hec_gf_matmul_host", "hec_host_isa", "hec_encode_rows_host",
    "hec_coder_prepare_decode", "hec_jit_warm", "hec_jit_stats", "hec_queue_stats",
    "hec_encode_rows_workspace_size", "hec_encode_rows_device", "hec_decode_rows_host",
]


class HdfsError(Exception):
    """Base of the errors the reference reports (rust/src/error.rs)."""


class ErasureCodingError(HdfsError):
    """HdfsError::ErasureCodingError (error.rs:34-35)."""


class UnsupportedErasureCodingPolicy(HdfsError):
    """HdfsError::UnsupportedErasureCodingPolicy (error.rs:32-33)."""


class ChecksumError(HdfsError):
    """HdfsError::ChecksumError (error.rs; raised by ReadPacket::get_data,
    connection.rs:497-499)."""


class DeviceError(HdfsError):
    pass


def _share_torch_hip_runtime() -> None:
    """If PyTorch is installed, import it BEFORE loading the engine.

    torch's wheel bundles its own libamdhip64 and links it by the unversioned
    name; our .so links libamdhip64.so.7.  Loaded lib-first, the process ends
    up with two HIP runtimes and whichever initialises first owns the GPU
    (the other reports "no ROCm-capable device").  Loaded torch-first, our
    DT_NEEDED libamdhip64.so.7 matches the SONAME of torch's copy and one
    runtime serves both.  Set HEC_NO_TORCH_PRELOAD=1 to skip."""
    import importlib.util
    if os.environ.get("HEC_NO_TORCH_PRELOAD") == "1":
        return
    if importlib.util.find_spec("torch") is not None:
        import torch  # noqa: F401


EXP_LIB_PATH = os.path.join(os.path.dirname(_HERE), "lib", "libhdfs_ec_amd_exp.so")


def _load(path: str = LIB_PATH) -> ctypes.CDLL:
    _share_torch_hip_runtime()
    if not os.path.exists(path):
        raise ImportError(
            f"{path} not built: run `make -C hdfs-native_amd` (or __graft_entry__.build()). "
            "There is no CPU fallback.")
    lib = ctypes.CDLL(path)
    P, S, I = ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int
    PP = ctypes.POINTER(ctypes.c_void_p)
    SP = ctypes.POINTER(ctypes.c_size_t)
    sig = {
        "hec_strerror": ([I], ctypes.c_char_p),
        "hec_abi_version": ([], I),
        "hec_last_error": ([], ctypes.c_char_p),
        "hec_gen_rs_matrix": ([S, S, P], I),
        "hec_gen_codec_matrix": ([ctypes.c_char_p, S, S, P], I),
        "hec_matrix_invert": ([P, S], I),
        "hec_decode_plan": ([S, S, P, SP, SP, SP, P], I),
        "hec_coder_create": ([S, S, I, ctypes.POINTER(P)], I),
        "hec_coder_create_codec": ([ctypes.c_char_p, S, S, I, ctypes.POINTER(P)], I),
        "hec_coder_destroy": ([P], None),
        "hec_coder_data_units": ([P], S),
        "hec_coder_parity_units": ([P], S),
        "hec_coder_device": ([P], I),
        "hec_encode": ([P, PP, S, PP], I),
        "hec_decode": ([P, PP, S, PP], I),
        "hec_encode_device": ([P, PP, SP, PP, SP, S, S, P], I),
        "hec_decode_device": ([P, PP, SP, PP, SP, S, S, P], I),
        "hec_gf_matmul_device": ([P, P, S, S, PP, SP, PP, SP, S, S, P], I),
        "hec_encode_host_batch": ([P, P, P, S, S, S], I),
        "hec_decode_host_batch": ([P, PP, S, S, P, S], I),
        "hec_crc32c_device": ([P, PP, SP, S, S, S, S, P, P], I),
        "hec_encode_crc_device": ([P, PP, SP, PP, SP, S, S, S, P, P], I),
        "hec_checksum_device": ([P, I, PP, SP, S, S, S, S, P, P], I),
        "hec_checksum_verify_device": ([P, I, PP, SP, S, S, S, S, P, P, P], I),
        "hec_decode_verify_device": ([P, I, PP, SP, PP, SP, S, S, S, P, P, P], I),
        "hec_decode_mixed_workspace_size": ([P, S], S),
        "hec_decode_device_mixed": ([P, PP, SP, PP, SP, ctypes.POINTER(ctypes.c_uint64), S, S, P, S, P], I),
        "hec_group_create": ([ctypes.c_char_p, S, S, ctypes.POINTER(I), S, ctypes.POINTER(P)], I),
        "hec_group_destroy": ([P], None),
        "hec_group_size": ([P], S),
        "hec_group_coder": ([P, S], P),
        "hec_group_range": ([P, S, S, SP, SP], I),
        "hec_group_encode_host_batch": ([P, P, P, S, S, S], I),
        "hec_group_decode_host_batch": ([P, PP, S, S, P, S], I),
        "hec_group_encode_device": ([P, PP, SP, PP, SP, S, SP, PP], I),
        "hec_group_decode_device": ([P, PP, SP, PP, SP, S, SP, PP], I),
        "hec_device_alloc": ([I, S, ctypes.c_uint, ctypes.POINTER(P)], I),
        "hec_device_free": ([I, P], I),
        "hec_device_numa_node": ([I], I),
        "hec_device_copy": ([I, P, P, S], I),
        "hec_device_synchronize": ([I, P], I),
        "hec_host_alloc": ([I, S, I, ctypes.POINTER(P)], I),
        "hec_host_free": ([P], I),
        "hec_coder_acquire": ([ctypes.c_char_p, S, S, I, ctypes.POINTER(P)], I),
        "hec_coder_release": ([P], None),
        "hec_coder_pool_trim": ([], S),
        "hec_coder_set_host_limit": ([P, S], I),
        "hec_coder_host_limit": ([P], S),
        "hec_coder_prepare_decode": ([P, P, I, P], I),
        "hec_jit_warm": ([S, S, P, I], I),
        "hec_jit_stats": ([P, P, P, P], None),
        "hec_queue_stats": ([I, P, P, P], None),
        "hec_gf_matmul_host": ([P, S, S, PP, PP, S], I),
        "hec_host_isa": ([], ctypes.c_char_p),
        "hec_encode_rows_host": ([P, P, S, P, S, S], I),
        "hec_encode_rows_workspace_size": ([P, S], S),
        "hec_encode_rows_device": ([P, P, S, P, S, P, S, P], I),
        "hec_decode_rows_host": ([P, PP, SP, S, P, S, S], I),
    }
    if hasattr(lib, "hec_tune_set"):  # the measurement build only (include/hdfs_ec_amd_exp.h)
        sig["hec_tune_set"] = ([I, I], I)
    for name, (args, res) in sig.items():
        if os.environ.get("HEC_LIB_PATH") and not hasattr(lib, name):
            continue  # an older build loaded for a same-box A/B: entry points it predates stay unbound
        fn = getattr(lib, name)
        fn.argtypes = args
        fn.restype = res
    return lib


lib = _load()
_exp_lib = None


def experimental_available() -> bool:
    return os.path.exists(EXP_LIB_PATH)


def experimental_lib() -> ctypes.CDLL:
    """The HEC_EXPERIMENTAL measurement build (lib/libhdfs_ec_amd_exp.so,
    `make -C hdfs-native_amd exp`: the default kernels plus every shape a knob
    can select and the measured-and-rejected variants).  Pass it as
    Coder(..., lib=experimental_lib()); its knobs (include/hdfs_ec_amd_exp.h)
    are its own.  The product library has no knobs."""
    global _exp_lib
    if _exp_lib is None:
        if not experimental_available():
            raise ImportError(f"{EXP_LIB_PATH} not built: run `make -C hdfs-native_amd exp` (measurement build)")
        _exp_lib = _load(EXP_LIB_PATH)
    return _exp_lib


def strerror(rc: int) -> str:
    return lib.hec_strerror(rc).decode()


def _check(rc: int) -> None:
    if rc == HEC_OK:
        return
    msg = strerror(rc)
    if rc == HEC_ERR_NOT_ENOUGH_SHARDS:
        raise ErasureCodingError("Not enough valid shards")
    if rc == HEC_ERR_UNSUPPORTED_CODEC:
        raise UnsupportedErasureCodingPolicy(msg)
    if rc == HEC_ERR_CHECKSUM:
        raise ChecksumError(msg)
    if rc in (HEC_ERR_INVALID_ARG, HEC_ERR_SINGULAR):
        raise ValueError(msg)
    if rc == HEC_ERR_NO_MEMORY:
        raise MemoryError(msg)
    raise DeviceError(f"{msg} (status {rc}): {lib.hec_last_error().decode()}")


def _pp(addrs: Sequence[int]):
    return (ctypes.c_void_p * len(addrs))(*addrs)


def _sp(vals: Sequence[int]):
    return (ctypes.c_size_t * len(vals))(*vals)


def gen_rs_matrix(data_units: int, parity_units: int) -> List[List[int]]:
    buf = (ctypes.c_uint8 * ((data_units + parity_units) * data_units))()
    _check(lib.hec_gen_rs_matrix(data_units, parity_units, buf))
    k = data_units
    return [list(buf[r * k:(r + 1) * k]) for r in range(data_units + parity_units)]


def gen_codec_matrix(codec: str, data_units: int, parity_units: int) -> List[List[int]]:
    """The (k+m) x k matrix a coder of `codec` ("rs", "xor", "rs-legacy") uses."""
    buf = (ctypes.c_uint8 * ((data_units + parity_units) * data_units))()
    _check(lib.hec_gen_codec_matrix(codec.encode(), data_units, parity_units, buf))
    k = data_units
    return [list(buf[r * k:(r + 1) * k]) for r in range(data_units + parity_units)]


def matrix_invert(mat: List[List[int]]) -> List[List[int]]:
    n = len(mat)
    buf = (ctypes.c_uint8 * (n * n))(*[v for row in mat for v in row])
    _check(lib.hec_matrix_invert(buf, n))
    return [list(buf[r * n:(r + 1) * n]) for r in range(n)]


def host_isa() -> str:
    """The host routine's ISA (hec_host_isa): avx512bw+gfni, avx2 or scalar."""
    return lib.hec_host_isa().decode()


def gf_matmul_host(matrix: List[List[int]], shards: Sequence) -> List[bytes]:
    """hec_gf_matmul_host: the hot loop Mul<&[&[u8]]> (matrix.rs:204-231) on
    the host -- out[j] = sum_i matrix[j][i] * shards[i] over GF(2^8)."""
    import numpy as np
    rows, cols = len(matrix), len(matrix[0])
    ins = [np.ascontiguousarray(np.frombuffer(bytes(x) if not isinstance(x, np.ndarray) else x, dtype=np.uint8))
           for x in shards]
    n = len(ins[0])
    outs = [np.empty(n, dtype=np.uint8) for _ in range(rows)]
    mat = (ctypes.c_uint8 * (rows * cols))(*[v for r in matrix for v in r])
    _check(lib.hec_gf_matmul_host(mat, rows, cols, _pp([a.ctypes.data for a in ins]),
                                  _pp([a.ctypes.data for a in outs]), n))
    return [o.tobytes() for o in outs]


def pool_trim() -> int:
    """hec_coder_pool_trim: destroys the idle pooled coders."""
    return lib.hec_coder_pool_trim()


def decode_plan(data_units: int, parity_units: int, present: Sequence[bool]):
    k, m = data_units, parity_units
    pres = (ctypes.c_uint8 * (k + m))(*[1 if p else 0 for p in present])
    e = ctypes.c_size_t(0)
    surv = (ctypes.c_size_t * k)()
    miss = (ctypes.c_size_t * k)()
    mat = (ctypes.c_uint8 * (k * k))()
    _check(lib.hec_decode_plan(k, m, pres, ctypes.byref(e), surv, miss, mat))
    e = e.value
    return list(surv) if e else [], list(miss[:e]), [list(mat[r * k:(r + 1) * k]) for r in range(e)]


ALLOC_DEFAULT = 0
ALLOC_CONTIGUOUS = 1


class DeviceBuffer:
    """HBM from hec_device_alloc (optionally physically contiguous), exposed
    to torch through __cuda_array_interface__: `torch.as_tensor(buf,
    device=...)` views it without a copy.  Freed by close()."""

    def __init__(self, nbytes: int, device: int = 0, flags: int = ALLOC_DEFAULT):
        p = ctypes.c_void_p()
        _check(lib.hec_device_alloc(device, nbytes, flags, ctypes.byref(p)))
        self.ptr, self.nbytes, self.device = p.value, nbytes, device

    @property
    def __cuda_array_interface__(self):
        return {"shape": (self.nbytes,), "typestr": "|u1", "data": (self.ptr, False), "version": 2}

    def close(self) -> None:
        if self.ptr:
            _check(lib.hec_device_free(self.device, ctypes.c_void_p(self.ptr)))
            self.ptr = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class HostBuffer:
    """Page-locked host memory on a NUMA node (hec_host_alloc; numa_node -1
    = the node of `device`).  .array() views it as a numpy uint8 array."""

    def __init__(self, nbytes: int, device: int = 0, numa_node: int = -1):
        p = ctypes.c_void_p()
        _check(lib.hec_host_alloc(device, nbytes, numa_node, ctypes.byref(p)))
        self.ptr, self.nbytes = p.value, nbytes

    def array(self):
        import numpy as np
        return np.ctypeslib.as_array((ctypes.c_uint8 * self.nbytes).from_address(self.ptr))

    def close(self) -> None:
        if self.ptr:
            _check(lib.hec_host_free(ctypes.c_void_p(self.ptr)))
            self.ptr = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def device_numa_node(device: int = 0) -> int:
    return lib.hec_device_numa_node(device)


def tune_set(key: int, value: int, lib_=None) -> None:
    """hec_tune_set on the measurement build (default: experimental_lib())."""
    _check((lib_ or experimental_lib()).hec_tune_set(key, value))


def _addr(buf) -> int:
    """Address of a writable/readable contiguous host buffer (numpy array,
    bytearray, ctypes array, or bytes via a copy-free view when possible)."""
    import numpy as np
    if isinstance(buf, np.ndarray):
        assert buf.flags["C_CONTIGUOUS"]
        return buf.ctypes.data
    arr = np.frombuffer(buf, dtype=np.uint8)
    return arr.ctypes.data


class Coder:
    """Drop-in for hdfs_native::ec::gf256::Coder on one MI355X.  pooled=True
    takes the coder from the process-wide pool (hec_coder_acquire; device -1
    = any) and close() returns it (hec_coder_release)."""

    def __init__(self, data_units: int, parity_units: int, device: int = 0, codec: str = "rs", lib=None,
                 pooled: bool = False):
        self._lib = lib or globals()["lib"]
        h = ctypes.c_void_p()
        if pooled:
            _check(self._lib.hec_coder_acquire(codec.encode(), data_units, parity_units, device, ctypes.byref(h)))
            device = self._lib.hec_coder_device(h)
        else:
            _check(self._lib.hec_coder_create_codec(codec.encode(), data_units, parity_units, device,
                                                    ctypes.byref(h)))
        self.pooled = pooled
        self.codec = codec
        self._h = h
        self.data_units = data_units
        self.parity_units = parity_units
        self.device = device

    def close(self) -> None:
        if getattr(self, "_h", None):
            (self._lib.hec_coder_release if self.pooled else self._lib.hec_coder_destroy)(self._h)
            self._h = None

    @property
    def host_limit(self) -> int:
        """Rows of at most this many bytes per shard are coded on the host
        (hec_coder_host_limit); 0 = always the device."""
        return self._lib.hec_coder_host_limit(self._h)

    @host_limit.setter
    def host_limit(self, max_shard_len: int) -> None:
        _check(self._lib.hec_coder_set_host_limit(self._h, max_shard_len))

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    @property
    def handle(self):
        return self._h

    gen_rs_matrix = staticmethod(gen_rs_matrix)

    # -- host-buffer API: Coder::encode / Coder::decode --------------------
    def encode(self, data: Sequence[bytes]) -> List[bytes]:
        """gf256.rs:61-80: returns m parity shards as bytes."""
        import numpy as np
        assert len(data) == self.data_units, "data.len() == data_units (gf256.rs:62)"
        n = len(data[0])
        assert all(len(d) == n for d in data), "equal shard lengths (gf256.rs:65)"
        ins = [np.ascontiguousarray(np.frombuffer(bytes(d) if not isinstance(d, np.ndarray) else d,
                                                  dtype=np.uint8)) for d in data]
        outs = [np.empty(n, dtype=np.uint8) for _ in range(self.parity_units)]
        _check(self._lib.hec_encode(self._h, _pp([a.ctypes.data for a in ins]), n,
                              _pp([a.ctypes.data for a in outs])))
        return [o.tobytes() for o in outs]

    def decode(self, data: List[Optional[bytes]]) -> None:
        """gf256.rs:84-137: fills missing data slots of `data` in place."""
        import numpy as np
        k, m = self.data_units, self.parity_units
        assert len(data) == k + m
        present = [d for d in data if d is not None]
        if not present:
            _check(HEC_ERR_NOT_ENOUGH_SHARDS if any(d is None for d in data[:k]) else HEC_OK)
            return
        n = len(present[0])
        ins = [None if d is None else np.ascontiguousarray(np.frombuffer(bytes(d), dtype=np.uint8))
               for d in data]
        outs = [np.empty(n, dtype=np.uint8) if (i < k and data[i] is None) else None for i in range(k + m)]
        _check(self._lib.hec_decode(self._h, _pp([0 if a is None else a.ctypes.data for a in ins]), n,
                              _pp([0 if a is None else a.ctypes.data for a in outs])))
        for i in range(k):
            if data[i] is None:
                data[i] = outs[i].tobytes()

    def prepare_decode(self, missing: Sequence[int], checksum_type: int = 2) -> bool:
        """hec_coder_prepare_decode: compile the plan-specialised fused decode
        + verify kernel for shards `missing` unavailable, now; True when it
        is ready (see include/hdfs_ec_amd.h)."""
        n = self.data_units + self.parity_units
        present = (ctypes.c_uint8 * n)(*[0 if i in set(missing) else 1 for i in range(n)])
        flag = ctypes.c_int(0)
        _check(self._lib.hec_coder_prepare_decode(self._h, present, checksum_type, ctypes.byref(flag)))
        return bool(flag.value)

    # -- device-resident batched API ----------------------------------------
    def encode_device(self, data_ptrs, data_strides, parity_ptrs, parity_strides, cell_len, stripes,
                      stream: int = 0) -> None:
        _check(self._lib.hec_encode_device(self._h, _pp(data_ptrs), _sp(data_strides), _pp(parity_ptrs),
                                     _sp(parity_strides), cell_len, stripes, ctypes.c_void_p(stream)))

    def decode_device(self, shard_ptrs, shard_strides, out_ptrs, out_strides, cell_len, stripes,
                      stream: int = 0) -> None:
        _check(self._lib.hec_decode_device(self._h, _pp([p or 0 for p in shard_ptrs]), _sp(shard_strides),
                                     _pp([p or 0 for p in out_ptrs]), _sp(out_strides), cell_len, stripes,
                                     ctypes.c_void_p(stream)))

    def crc32c_device(self, ptrs, strides, cell_len, stripes, bytes_per_checksum, out_ptr, stream: int = 0):
        _check(self._lib.hec_crc32c_device(self._h, _pp(ptrs), _sp(strides), len(ptrs), cell_len, stripes,
                                     bytes_per_checksum, ctypes.c_void_p(out_ptr), ctypes.c_void_p(stream)))

    def checksum_device(self, checksum_type: int, ptrs, strides, cell_len, stripes, bytes_per_checksum, out_ptr,
                        stream: int = 0):
        _check(self._lib.hec_checksum_device(self._h, checksum_type, _pp(ptrs), _sp(strides), len(ptrs), cell_len, stripes,
                                       bytes_per_checksum, ctypes.c_void_p(out_ptr), ctypes.c_void_p(stream)))

    def checksum_verify_device(self, checksum_type: int, ptrs, strides, cell_len, stripes, bytes_per_checksum,
                               expected_ptr, bad_ptr, stream: int = 0):
        _check(self._lib.hec_checksum_verify_device(self._h, checksum_type, _pp(ptrs), _sp(strides), len(ptrs), cell_len,
                                              stripes, bytes_per_checksum, ctypes.c_void_p(expected_ptr),
                                              ctypes.c_void_p(bad_ptr), ctypes.c_void_p(stream)))

    def decode_verify_device(self, checksum_type: int, shard_ptrs, shard_strides, out_ptrs, out_strides, cell_len,
                             stripes, bytes_per_checksum, sums_ptr, bad_ptr, stream: int = 0) -> None:
        """Verified striped read (hec_decode_verify_device): raises
        ErasureCodingError when a stripe has fewer than k cells that verify
        (the bad flags are written either way)."""
        _check(self._lib.hec_decode_verify_device(self._h, checksum_type, _pp(shard_ptrs), _sp(shard_strides),
                                            _pp(out_ptrs), _sp(out_strides), cell_len, stripes, bytes_per_checksum,
                                            ctypes.c_void_p(sums_ptr), ctypes.c_void_p(bad_ptr),
                                            ctypes.c_void_p(stream)))

    def encode_crc_device(self, data_ptrs, data_strides, parity_ptrs, parity_strides, cell_len, stripes,
                          bytes_per_checksum, sums_ptr, stream: int = 0):
        _check(self._lib.hec_encode_crc_device(self._h, _pp(data_ptrs), _sp(data_strides), _pp(parity_ptrs),
                                         _sp(parity_strides), cell_len, stripes, bytes_per_checksum,
                                         ctypes.c_void_p(sums_ptr), ctypes.c_void_p(stream)))

    def decode_mixed_workspace_size(self, stripes: int) -> int:
        return self._lib.hec_decode_mixed_workspace_size(self._h, stripes)

    def decode_device_mixed(self, shard_ptrs, shard_strides, out_ptrs, out_strides, present_masks, cell_len,
                            stripes, workspace_ptr, workspace_bytes, stream: int = 0) -> None:
        masks = (ctypes.c_uint64 * stripes)(*present_masks)
        _check(self._lib.hec_decode_device_mixed(self._h, _pp(shard_ptrs), _sp(shard_strides), _pp(out_ptrs),
                                           _sp(out_strides), masks, cell_len, stripes,
                                           ctypes.c_void_p(workspace_ptr), workspace_bytes,
                                           ctypes.c_void_p(stream)))

    def gf_matmul_device(self, matrix: List[List[int]], in_ptrs, in_strides, out_ptrs, out_strides, cell_len,
                         stripes, stream: int = 0) -> None:
        rows, cols = len(matrix), len(matrix[0])
        mat = (ctypes.c_uint8 * (rows * cols))(*[v for r in matrix for v in r])
        _check(self._lib.hec_gf_matmul_device(self._h, mat, rows, cols, _pp(in_ptrs), _sp(in_strides), _pp(out_ptrs),
                                        _sp(out_strides), cell_len, stripes, ctypes.c_void_p(stream)))

    def decode_host_batch(self, vertical_addrs, cell_len: int, rows: int, h_file_addr: int, chunk_rows: int) -> None:
        """vertical_addrs[k+m]: host addresses of the per-shard vertical
        buffers (0/None = missing) -> file-order bytes at h_file_addr."""
        _check(self._lib.hec_decode_host_batch(self._h, _pp([a or 0 for a in vertical_addrs]), cell_len, rows,
                                         ctypes.c_void_p(h_file_addr), chunk_rows))

    def encode_host_batch(self, h_data_addr: int, h_parity_addr: int, cell_len: int, stripes: int,
                          chunk_stripes: int) -> None:
        _check(self._lib.hec_encode_host_batch(self._h, ctypes.c_void_p(h_data_addr), ctypes.c_void_p(h_parity_addr),
                                         cell_len, stripes, chunk_stripes))

    # -- whole files: the last row may be short (CellBuffer semantics) --------
    def encode_rows_host(self, h_data_addr: int, data_len: int, h_parity_addr: int, cell_len: int,
                         chunk_stripes: int = 16) -> None:
        _check(self._lib.hec_encode_rows_host(self._h, ctypes.c_void_p(h_data_addr), data_len,
                                              ctypes.c_void_p(h_parity_addr), cell_len, chunk_stripes))

    def encode_rows_workspace_size(self, cell_len: int) -> int:
        return self._lib.hec_encode_rows_workspace_size(self._h, cell_len)

    def encode_rows_device(self, d_data: int, data_len: int, d_parity: int, cell_len: int, workspace: int,
                           workspace_bytes: int, stream: int = 0) -> None:
        _check(self._lib.hec_encode_rows_device(self._h, ctypes.c_void_p(d_data), data_len, ctypes.c_void_p(d_parity),
                                                cell_len, ctypes.c_void_p(workspace), workspace_bytes,
                                                ctypes.c_void_p(stream)))

    def decode_rows_host(self, vertical_addrs, vertical_lens, cell_len: int, h_file_addr: int, file_len: int,
                         chunk_rows: int = 16) -> None:
        _check(self._lib.hec_decode_rows_host(self._h, _pp([a or 0 for a in vertical_addrs]), _sp(vertical_lens),
                                              cell_len, ctypes.c_void_p(h_file_addr), file_len, chunk_rows))


# ---- torch helpers (device memory comes from torch; plumbing only) --------

def jit_warm(k: int, m: int, missing: Sequence[int], checksum_type: int = 2) -> None:
    """hec_jit_warm: the specialised decode + verify kernel for this plan into
    the code-object caches (no device needed)."""
    present = (ctypes.c_uint8 * (k + m))(*[0 if i in set(missing) else 1 for i in range(k + m)])
    _check(lib.hec_jit_warm(k, m, present, checksum_type))


def jit_stats() -> dict:
    """hec_jit_stats: process totals of the plan-time JIT."""
    v = [ctypes.c_uint64(0) for _ in range(4)]
    lib.hec_jit_stats(*[ctypes.byref(x) for x in v])
    return dict(zip(("compiled", "from_disk", "failed", "launches"), (x.value for x in v)))


def queue_stats(device: int = 0) -> dict:
    """hec_queue_stats: the work-queue counter sets of `device` (streams that
    launched a queue kernel, graph sets handed out to captured launches, and
    whether streams are told apart by hipStreamGetId or by handle)."""
    v = [ctypes.c_uint64(0) for _ in range(2)]
    by_id = ctypes.c_int(0)
    lib.hec_queue_stats(device, *[ctypes.byref(x) for x in v], ctypes.byref(by_id))
    return {"streams": v[0].value, "graph_sets": v[1].value, "keyed_by_id": bool(by_id.value)}


def stripe_layout_ptrs(t, units: int):
    """For a uint8 tensor [stripes, units, cell] return (ptrs, strides)."""
    assert t.dim() == 3 and t.shape[1] == units and t.is_contiguous()
    cell = t.shape[2]
    base = t.data_ptr()
    return [base + i * cell for i in range(units)], [units * cell] * units


def encode_batch(coder: Coder, data, parity, stream=None) -> None:
    """data: uint8 cuda tensor [S, k, cell]; parity: [S, m, cell]."""
    import torch
    s = stream if stream is not None else torch.cuda.current_stream(data.device)
    dp, ds = stripe_layout_ptrs(data, coder.data_units)
    pp, ps = stripe_layout_ptrs(parity, coder.parity_units)
    coder.encode_device(dp, ds, pp, ps, data.shape[2], data.shape[0], s.cuda_stream)


def crc32c_batch(coder: Coder, cells, bytes_per_checksum: int = 512, stream=None):
    """cells: uint8 cuda tensor [S, n, cell] -> uint8 tensor [S, n, nchunks, 4]
    of big-endian CRC32C per chunk (WritePacket::calculate_checksum)."""
    import torch
    S, n, cell = cells.shape
    s = stream if stream is not None else torch.cuda.current_stream(cells.device)
    nchunks = (cell + bytes_per_checksum - 1) // bytes_per_checksum
    out = torch.empty((S, n, nchunks, 4), dtype=torch.uint8, device=cells.device)
    ptrs, strides = stripe_layout_ptrs(cells, n)
    coder.crc32c_device(ptrs, strides, cell, S, bytes_per_checksum, out.data_ptr(), s.cuda_stream)
    return out


def checksum_batch(coder: Coder, cells, checksum_type: int = CHECKSUM_CRC32C, bytes_per_checksum: int = 512,
                   stream=None):
    """cells: uint8 cuda tensor [S, n, cell] -> uint8 tensor [S, n, nchunks, 4]
    of big-endian chunk checksums (CRC32C or CRC32 = CRC_32_CKSUM)."""
    import torch
    S, n, cell = cells.shape
    s = stream if stream is not None else torch.cuda.current_stream(cells.device)
    nchunks = (cell + bytes_per_checksum - 1) // bytes_per_checksum
    out = torch.empty((S, n, nchunks, 4), dtype=torch.uint8, device=cells.device)
    ptrs, strides = stripe_layout_ptrs(cells, n)
    coder.checksum_device(checksum_type, ptrs, strides, cell, S, bytes_per_checksum, out.data_ptr(), s.cuda_stream)
    return out


def checksum_verify_batch(coder: Coder, cells, expected, checksum_type: int = CHECKSUM_CRC32C,
                          bytes_per_checksum: int = 512, stream=None):
    """ReadPacket::get_data's check: -> uint8 tensor [S, n], 1 where a cell
    has a chunk whose checksum differs from `expected` [S, n, nchunks, 4]."""
    import torch
    S, n, cell = cells.shape
    s = stream if stream is not None else torch.cuda.current_stream(cells.device)
    bad = torch.zeros((S, n), dtype=torch.uint8, device=cells.device)
    ptrs, strides = stripe_layout_ptrs(cells, n)
    coder.checksum_verify_device(checksum_type, ptrs, strides, cell, S, bytes_per_checksum,
                                 expected.data_ptr(), bad.data_ptr(), s.cuda_stream)
    return bad


def decode_verify_batch(coder: Coder, data, parity, missing: Sequence[int], sums, out,
                        checksum_type: int = CHECKSUM_CRC32C, bytes_per_checksum: int = 512, stream=None,
                        missing_parity: Sequence[int] = ()):
    """Verified striped read over data [S,k,cell] / parity [S,m,cell] with
    data shards `missing` (and parity shards `missing_parity`) unavailable
    for the batch; sums [S, k+m, nchunks, 4] are the packets' checksums.
    Rebuilt data lands in out [S,k,cell]; returns the bad-cell flags
    [S, k+m] (uint8 cuda tensor)."""
    import torch
    k, m = coder.data_units, coder.parity_units
    S = data.shape[0]
    s = stream if stream is not None else torch.cuda.current_stream(data.device)
    dp, ds = stripe_layout_ptrs(data, k)
    pp, ps = stripe_layout_ptrs(parity, m)
    op, os_ = stripe_layout_ptrs(out, k)
    miss, pmiss = set(missing), set(missing_parity)
    ptrs = [None if i in miss else dp[i] for i in range(k)] + [None if j in pmiss else pp[j] for j in range(m)]
    bad = torch.empty((S, k + m), dtype=torch.uint8, device=data.device)
    coder.decode_verify_device(checksum_type, ptrs, ds + ps, op, os_, data.shape[2], S, bytes_per_checksum,
                               sums.data_ptr(), bad.data_ptr(), s.cuda_stream)
    return bad


def decode_batch_mixed(coder: Coder, data, parity, present_masks: Sequence[int], out, stream=None,
                       workspace=None) -> None:
    """Per-stripe erasure patterns: present_masks[s] bit i = shard i present.
    Rebuilt data shards land in out [S,k,cell] where missing."""
    import torch
    k, m = coder.data_units, coder.parity_units
    S = data.shape[0]
    s = stream if stream is not None else torch.cuda.current_stream(data.device)
    dp, ds = stripe_layout_ptrs(data, k)
    pp, ps = stripe_layout_ptrs(parity, m)
    op, os_ = stripe_layout_ptrs(out, k)
    nbytes = coder.decode_mixed_workspace_size(S)
    if workspace is None:
        workspace = torch.empty(max(nbytes, 1), dtype=torch.uint8, device=data.device)
    coder.decode_device_mixed(dp + pp, ds + ps, op, os_, list(present_masks), data.shape[2], S,
                              workspace.data_ptr(), workspace.numel(), s.cuda_stream)
    return workspace


def decode_batch(coder: Coder, data, parity, missing: Sequence[int], out, stream=None) -> None:
    """Reconstruct data shards `missing` of every stripe (one erasure pattern
    for the batch) from data [S,k,cell] / parity [S,m,cell] into out
    [S,k,cell] (only the missing slots are written)."""
    import torch
    k, m = coder.data_units, coder.parity_units
    s = stream if stream is not None else torch.cuda.current_stream(data.device)
    dp, ds = stripe_layout_ptrs(data, k)
    pp, ps = stripe_layout_ptrs(parity, m)
    op, os_ = stripe_layout_ptrs(out, k)
    miss = set(missing)
    ptrs = [None if i in miss else dp[i] for i in range(k)] + pp
    coder.decode_device(ptrs, ds + ps, op, os_, data.shape[2], data.shape[0], s.cuda_stream)


class _Borrowed(Coder):
    """A group slot's coder: the group owns (and destroys) the handle."""

    def __init__(self, handle, k, m, device, codec):  # noqa: D107 (no super().__init__: no new coder)
        self._lib = lib
        self._h = handle
        self.codec, self.data_units, self.parity_units, self.device = codec, k, m, device

    def close(self) -> None:
        self._h = None


class CoderGroup:
    """Multi-GPU coder group (hec_group_*): a batch split into
    contiguous stripe ranges, one per device, each on its own host thread."""

    def __init__(self, data_units: int, parity_units: int, devices: Sequence[int], codec: str = "rs"):
        h = ctypes.c_void_p()
        devs = (ctypes.c_int * len(devices))(*devices)
        _check(lib.hec_group_create(codec.encode(), data_units, parity_units, devs, len(devices), ctypes.byref(h)))
        self._h = h
        self.data_units, self.parity_units, self.devices, self.codec = data_units, parity_units, list(devices), codec

    def close(self) -> None:
        if getattr(self, "_h", None):
            lib.hec_group_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __len__(self) -> int:
        return lib.hec_group_size(self._h)

    def coder(self, slot: int) -> Coder:
        h = lib.hec_group_coder(self._h, slot)
        if not h:
            raise IndexError(slot)
        return _Borrowed(ctypes.c_void_p(h), self.data_units, self.parity_units, self.devices[slot], self.codec)

    def range(self, total: int, slot: int):
        first, count = ctypes.c_size_t(), ctypes.c_size_t()
        _check(lib.hec_group_range(self._h, total, slot, ctypes.byref(first), ctypes.byref(count)))
        return first.value, count.value

    def encode_host_batch(self, h_data_addr: int, h_parity_addr: int, cell_len: int, stripes: int,
                          chunk_stripes: int) -> None:
        _check(lib.hec_group_encode_host_batch(self._h, ctypes.c_void_p(h_data_addr), ctypes.c_void_p(h_parity_addr),
                                               cell_len, stripes, chunk_stripes))

    def decode_host_batch(self, vertical_addrs, cell_len: int, rows: int, h_file_addr: int, chunk_rows: int) -> None:
        _check(lib.hec_group_decode_host_batch(self._h, _pp([a or 0 for a in vertical_addrs]), cell_len, rows,
                                               ctypes.c_void_p(h_file_addr), chunk_rows))

    def encode_device(self, data_ptrs, data_strides, parity_ptrs, parity_strides, cell_len: int, stripes,
                      streams=None) -> None:
        """hec_group_encode_device: per-slot lists (slot-major), each slot's
        stripes on its own device; asynchronous on `streams` (raw handles)."""
        _check(lib.hec_group_encode_device(self._h, _pp(data_ptrs), _sp(data_strides), _pp(parity_ptrs),
                                           _sp(parity_strides), cell_len, _sp(stripes),
                                           _pp(streams) if streams is not None else None))

    def decode_device(self, shard_ptrs, shard_strides, out_ptrs, out_strides, cell_len: int, stripes,
                      streams=None) -> None:
        """hec_group_decode_device: shard_ptrs slot-major k+m per slot (None =
        missing), out_ptrs k per slot."""
        _check(lib.hec_group_decode_device(self._h, _pp([a or 0 for a in shard_ptrs]), _sp(shard_strides),
                                           _pp([a or 0 for a in out_ptrs]), _sp(out_strides), cell_len,
                                           _sp(stripes), _pp(streams) if streams is not None else None))
