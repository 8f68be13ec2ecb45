"""C-ABI checks that need no GPU: the library loads, exports every symbol the
header declares, and its host-side helpers (coding matrix, inversion, decode
plan) match the oracle.  No compute is launched here."""
import ctypes
import itertools
import os
import re

import pytest

import ec_oracle as O
import hdfs_native_ec as H
from conftest import ROOT, gpu_available

HEADER = os.path.join(ROOT, "include", "hdfs_ec_amd.h")


def header_functions():
    text = open(HEADER).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(hec_[a-z_0-9]+)\s*\(", text)))


def test_header_declares_what_binding_binds():
    assert header_functions() == sorted(H.EXPORTS)


def test_library_exports_every_declared_symbol():
    lib = ctypes.CDLL(H.LIB_PATH)
    for name in header_functions():
        assert hasattr(lib, name), name


def test_abi_version_and_strerror():
    assert H.lib.hec_abi_version() == 5
    assert "Not enough valid shards" in H.strerror(H.HEC_ERR_NOT_ENOUGH_SHARDS)
    assert H.strerror(H.HEC_ERR_CHECKSUM) == "checksum error"
    assert H.strerror(12345) == "unknown status"


@pytest.mark.parametrize("k,m", [(3, 2), (6, 3), (10, 4), (1, 1), (32, 16), (2, 1)])
def test_gen_rs_matrix_matches_oracle(k, m):
    assert H.gen_rs_matrix(k, m) == O.gen_rs_matrix(k, m)


def test_gen_rs_matrix_rejects_bad_args():
    buf = (ctypes.c_uint8 * 16)()
    assert H.lib.hec_gen_rs_matrix(0, 2, buf) == H.HEC_ERR_INVALID_ARG
    assert H.lib.hec_gen_rs_matrix(200, 100, buf) == H.HEC_ERR_INVALID_ARG
    assert H.lib.hec_gen_rs_matrix(3, 2, None) == H.HEC_ERR_INVALID_ARG


def test_invert_matches_oracle_every_rs63_submatrix():
    for rows in itertools.combinations(range(9), 6):
        sub = O.select_rows(O.gen_rs_matrix(6, 3), rows)
        assert H.matrix_invert(sub) == O.invert(sub)


def test_invert_singular_is_status_not_abort():
    with pytest.raises(ValueError):
        H.matrix_invert([[1, 1], [1, 1]])


@pytest.mark.parametrize("k,m", [(3, 2), (6, 3), (10, 4)])
def test_decode_plan_matches_oracle_all_patterns(k, m):
    for e in range(0, m + 2):
        for miss in itertools.combinations(range(k + m), e):
            present = [i not in miss for i in range(k + m)]
            try:
                want = O.decode_plan(k, m, present)
            except O.NotEnoughShards:
                with pytest.raises(H.ErasureCodingError):
                    H.decode_plan(k, m, present)
                continue
            assert H.decode_plan(k, m, present) == (list(want[0]), list(want[1]), want[2])


def test_coder_create_validates_args():
    h = ctypes.c_void_p()
    assert H.lib.hec_coder_create(0, 3, 0, ctypes.byref(h)) == H.HEC_ERR_INVALID_ARG
    assert H.lib.hec_coder_create(33, 3, 0, ctypes.byref(h)) == H.HEC_ERR_INVALID_ARG
    assert H.lib.hec_coder_create(6, 17, 0, ctypes.byref(h)) == H.HEC_ERR_INVALID_ARG
    assert H.lib.hec_coder_create(6, 3, 0, None) == H.HEC_ERR_INVALID_ARG


def test_null_coder_calls_return_status():
    assert H.lib.hec_encode(None, None, 16, None) == H.HEC_ERR_INVALID_ARG
    assert H.lib.hec_decode(None, None, 16, None) == H.HEC_ERR_INVALID_ARG
    assert H.lib.hec_coder_data_units(None) == 0
    assert H.lib.hec_checksum_device(None, 2, None, None, 1, 16, 1, 512, None, None) == H.HEC_ERR_INVALID_ARG
    assert H.lib.hec_checksum_verify_device(None, 2, None, None, 1, 16, 1, 512, None, None,
                                            None) == H.HEC_ERR_INVALID_ARG
    assert H.lib.hec_checksum_verify_device(None, 0, None, None, 1, 16, 1, 512, None, None,
                                            None) == H.HEC_ERR_INVALID_ARG
    assert H.lib.hec_decode_verify_device(None, 2, None, None, None, None, 16, 1, 512, None, None,
                                          None) == H.HEC_ERR_INVALID_ARG
    H.lib.hec_coder_destroy(None)


@pytest.mark.skipif(gpu_available(), reason="checks the no-device error path")
def test_coder_create_without_device_is_clean_error():
    h = ctypes.c_void_p()
    assert H.lib.hec_coder_create(6, 3, 0, ctypes.byref(h)) == H.HEC_ERR_DEVICE
    assert not h.value


@pytest.mark.parametrize("codec,k,m", [("rs", 6, 3), ("rs", 32, 16), ("xor", 2, 1), ("xor", 7, 1),
                                       ("rs-legacy", 6, 3), ("rs-legacy", 3, 2), ("rs-legacy", 10, 4),
                                       ("rs-legacy", 1, 1), ("rs-legacy", 32, 16)])
def test_gen_codec_matrix_matches_oracle(codec, k, m):
    # rs-legacy: the oracle's matrix comes from Hadoop's long division
    # (GaloisField.remainder) on unit vectors; the library's from g(x) directly
    assert H.gen_codec_matrix(codec, k, m) == O.codec_matrix(codec, k, m)


def test_gen_codec_matrix_errors():
    buf = (ctypes.c_uint8 * 64)()
    assert H.lib.hec_gen_codec_matrix(b"lrc", 3, 2, buf) == H.HEC_ERR_UNSUPPORTED_CODEC
    assert H.lib.hec_gen_codec_matrix(b"xor", 3, 2, buf) == H.HEC_ERR_INVALID_ARG
    assert H.lib.hec_gen_codec_matrix(b"rs-legacy", 0, 2, buf) == H.HEC_ERR_INVALID_ARG
    assert H.lib.hec_gen_codec_matrix(b"rs-legacy", 3, 2, None) == H.HEC_ERR_INVALID_ARG


@pytest.mark.parametrize("k,m", [(3, 2), (6, 3), (10, 4)])
def test_rs_legacy_is_mds(k, m):
    # every k of the k+m rows invertible: any k survivors decode (the unique
    # codeword Hadoop's RSRawDecoderLegacy also finds)
    mat = H.gen_codec_matrix("rs-legacy", k, m)
    for rows in itertools.combinations(range(k + m), k):
        sub = (ctypes.c_uint8 * (k * k))(*[v for r in rows for v in mat[r]])
        assert H.lib.hec_matrix_invert(sub, k) == H.HEC_OK, rows


def test_codec_names_validated():
    h = ctypes.c_void_p()
    assert H.lib.hec_coder_create_codec(b"lrc", 6, 3, 0, ctypes.byref(h)) == H.HEC_ERR_UNSUPPORTED_CODEC
    assert H.lib.hec_coder_create_codec(b"xor", 2, 2, 0, ctypes.byref(h)) == H.HEC_ERR_INVALID_ARG
    assert not h.value


def test_group_argument_checks_need_no_device():
    # hec_group_* (SURVEY §8e): bad arguments are statuses, never a crash
    out = ctypes.c_void_p()
    devs = (ctypes.c_int * 2)(0, 0)
    assert H.lib.hec_group_create(b"rs", 6, 3, devs, 0, ctypes.byref(out)) == H.HEC_ERR_INVALID_ARG
    assert H.lib.hec_group_create(b"rs", 6, 3, None, 2, ctypes.byref(out)) == H.HEC_ERR_INVALID_ARG
    assert H.lib.hec_group_create(b"rs", 6, 3, devs, 65, ctypes.byref(out)) == H.HEC_ERR_INVALID_ARG
    assert H.lib.hec_group_create(b"rs", 6, 3, devs, 2, None) == H.HEC_ERR_INVALID_ARG
    assert H.lib.hec_group_size(None) == 0
    assert not H.lib.hec_group_coder(None, 0)
    first, count = ctypes.c_size_t(), ctypes.c_size_t()
    assert H.lib.hec_group_range(None, 10, 0, ctypes.byref(first), ctypes.byref(count)) == H.HEC_ERR_INVALID_ARG
    assert H.lib.hec_group_encode_host_batch(None, None, None, 16, 1, 1) == H.HEC_ERR_INVALID_ARG
    assert H.lib.hec_group_decode_host_batch(None, None, 16, 1, None, 1) == H.HEC_ERR_INVALID_ARG
    assert H.lib.hec_group_encode_device(None, None, None, None, None, 16, None, None) == H.HEC_ERR_INVALID_ARG
    assert H.lib.hec_group_decode_device(None, None, None, None, None, 16, None, None) == H.HEC_ERR_INVALID_ARG
    H.lib.hec_group_destroy(None)
    if not gpu_available():
        assert H.lib.hec_group_create(b"rs", 6, 3, devs, 2, ctypes.byref(out)) == H.HEC_ERR_DEVICE
        assert not out.value



@pytest.mark.skipif(gpu_available(), reason="CPU container only (the run expects no device)")
def test_host_paths_under_address_sanitizer(tmp_path):
    # ASan + LSan over the host-side C ABI (matrices, inversion, every RS(10,4)
    # decode plan, creation failure paths): scripts/asan_host.sh
    import shutil
    import subprocess
    objs = [os.path.join(ROOT, "hdfs-native_amd", "build", f"{n}.o") for n in ("ec_kernels", "ec_fused", "checksum")]
    if not shutil.which("/opt/rocm/bin/hipcc") or not all(os.path.exists(o) for o in objs):
        pytest.skip("needs hipcc and the built kernel objects")
    r = subprocess.run(["bash", os.path.join(ROOT, "scripts", "asan_host.sh"), str(tmp_path)], capture_output=True,
                       text=True, timeout=600)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    assert "bad=0" in r.stdout


def test_product_library_has_no_knobs():
    # measurement knobs live only in the HEC_EXPERIMENTAL build
    # (include/hdfs_ec_amd_exp.h); the product library neither declares nor
    # exports them
    lib = ctypes.CDLL(H.LIB_PATH)
    assert not hasattr(lib, "hec_tune_set")
    assert "hec_tune_set" not in header_functions()


@pytest.mark.skipif(not H.experimental_available(), reason="measurement build not built")
def test_tune_set_validates_without_device():
    # knobs are host-side atomics of the measurement build: no device needed
    xlib = H.experimental_lib()
    assert xlib.hec_tune_set(3, 2) == H.HEC_OK
    assert xlib.hec_tune_set(3, 0) == H.HEC_OK
    for key, value in [(6, 3), (11, 13), (16, 1), (3, 99), (18, 2), (17, 6), (19, 3), (20, 3), (21, 2), (5, 3), (13, 1), (15, 2), (22, 2), (23, 2), (24, 6), (25, 4097), (26, 5), (27, 4), (28, 3), (29, 3), (30, 2), (31, 3), (32, 2), (33, 512), (34, 0), (0, 0)]:
        assert xlib.hec_tune_set(key, value) == H.HEC_ERR_INVALID_ARG, (key, value)


# ---- the host small-row path (hec_gf_matmul_host) on the CPU ---------------
# rust/tests/test_ec.rs:77-87 sizes_to_test: 16 B, cell +- 4, 5 rows +- 4 (a
# 64 KiB cell keeps it quick; the GPU suite runs the 1 MiB cells)

def _sizes_to_test(k, cell):
    return [16, cell - 4, cell, cell + 4, 5 * k * cell - 4, 5 * k * cell, 5 * k * cell + 4]


@pytest.mark.parametrize("k,m", [(3, 2), (6, 3), (10, 4)])
def test_gf_matmul_host_vs_oracle_reference_sizes(k, m):
    import numpy as np
    from hdfs_native_ec.synth import splitmix64_bytes
    enc = O.gen_rs_matrix(k, m)
    for total in _sizes_to_test(k, 65536):
        # the writer's row split of a file of `total` bytes: the last row's
        # cells zero-padded to buffers[0].len() (block_writer.rs:817-851)
        n = min(65536, total)
        data = [splitmix64_bytes(total * 10 + i, n) for i in range(k)]
        got = H.gf_matmul_host(enc[k:], data)
        want = O.c_encode(O.load_c_oracle(), k, m, data)
        assert all(g == w.tobytes() for g, w in zip(got, want)), (k, m, total)
        # decode matrix of the worst case (data 0..m-1 lost)
        surv, miss, dm = O.decode_plan(k, m, [i >= m for i in range(k + m)])
        shards = data + [np.frombuffer(g, dtype=np.uint8) for g in got]
        rec = H.gf_matmul_host(dm, [shards[i] for i in surv])
        for r, i in enumerate(miss):
            assert rec[r] == data[i].tobytes()


def test_gf_matmul_host_args():
    buf = (ctypes.c_uint8 * 4)()
    ptrs = (ctypes.c_void_p * 2)()
    assert H.lib.hec_gf_matmul_host(None, 1, 1, ptrs, ptrs, 16) == H.HEC_ERR_INVALID_ARG
    assert H.lib.hec_gf_matmul_host(buf, 1, 33, ptrs, ptrs, 16) == H.HEC_ERR_INVALID_ARG
    assert H.lib.hec_gf_matmul_host(buf, 1, 1, ptrs, ptrs, 0) == H.HEC_ERR_INVALID_ARG
    assert H.lib.hec_gf_matmul_host(buf, 1, 1, ptrs, ptrs, 16) == H.HEC_ERR_INVALID_ARG  # null shard pointers
    assert H.host_isa() in ("avx512bw+gfni", "avx2", "scalar")


def test_coder_pool_args_need_no_device():
    h = ctypes.c_void_p()
    assert H.lib.hec_coder_acquire(b"rs", 6, 3, 0, None) == H.HEC_ERR_INVALID_ARG
    assert H.lib.hec_coder_acquire(b"rs", 6, 3, -3, ctypes.byref(h)) == H.HEC_ERR_INVALID_ARG
    assert H.lib.hec_coder_acquire(b"lrc", 6, 3, 0, ctypes.byref(h)) in (H.HEC_ERR_UNSUPPORTED_CODEC,
                                                                         H.HEC_ERR_DEVICE)
    assert not h.value
    H.lib.hec_coder_release(None)
    assert H.lib.hec_coder_set_host_limit(None, 5) == H.HEC_ERR_INVALID_ARG
    assert H.lib.hec_coder_host_limit(None) == 0
    if not gpu_available():
        # no GPU: "any device" is a host-only coder (Coder::new stays infallible)
        assert H.lib.hec_coder_acquire(b"rs", 6, 3, -1, ctypes.byref(h)) == H.HEC_OK
        assert H.lib.hec_coder_device(h) == H.HEC_DEVICE_HOST
        H.lib.hec_coder_release(h)
        assert H.pool_trim() == 1


# ---- host-only coders (HEC_DEVICE_HOST): run here, no GPU ------------------

def test_host_only_coder_encode_decode_vs_oracle(c_oracle):
    """Coder::new without a GPU (gf256.rs:32-38 is infallible): a host-only
    coder codes every row on the engine's host routine, bit-exact with the
    oracle, at sizes far above the device host limit."""
    import numpy as np
    for k, m in [(3, 2), (6, 3), (10, 4)]:
        c = H.Coder(k, m, H.HEC_DEVICE_HOST)
        assert H.lib.hec_coder_device(c.handle) == H.HEC_DEVICE_HOST
        c.host_limit = 0  # ignored: a host-only coder never routes to a device
        for n in (1, 17, 4096, (1 << 20) + 3):
            data = [np.frombuffer(os.urandom(n), dtype=np.uint8) for _ in range(k)]
            got = c.encode([d.tobytes() for d in data])
            want = O.c_encode(c_oracle, k, m, data)
            assert all(g == w.tobytes() for g, w in zip(got, want)), (k, m, n)
            full = [d.tobytes() for d in data] + got
            for miss in [(0,), tuple(range(m)), tuple(range(k - 1, k - 1 + m))]:
                shards = [None if i in miss else full[i] for i in range(k + m)]
                c.decode(shards)
                assert shards[:k] == full[:k], (k, m, n, miss)
        c.close()


def test_host_only_coder_batches_and_device_calls():
    """Host-batch calls run on the host routine; device-resident calls are
    HEC_ERR_DEVICE (never a HIP call)."""
    import numpy as np
    k, m, cell, S = 6, 3, 4096, 5
    c = H.Coder(k, m, H.HEC_DEVICE_HOST)
    data = np.frombuffer(os.urandom(S * k * cell), dtype=np.uint8).reshape(S, k, cell).copy()
    par = np.zeros((S, m, cell), dtype=np.uint8)
    c.encode_host_batch(data.ctypes.data, par.ctypes.data, cell, S, 2)
    for s in range(S):
        want = O.encode(k, m, list(data[s]))
        assert [bytes(x) for x in par[s]] == [bytes(w) for w in want]
    # decode straight into file order with data shards 0 and 4 lost
    vert = [np.ascontiguousarray(data[:, i]) for i in range(k)] + [np.ascontiguousarray(par[:, j]) for j in range(m)]
    addrs = [0 if i in (0, 4) else v.ctypes.data for i, v in enumerate(vert)]
    out = np.zeros(S * k * cell, dtype=np.uint8)
    c.decode_host_batch(addrs, cell, S, out.ctypes.data, 2)
    assert np.array_equal(out, data.reshape(-1))
    with pytest.raises(H.DeviceError):
        c.encode_device([0] * k, [0] * k, [0] * m, [0] * m, cell, 1)
    with pytest.raises(H.DeviceError):
        c.decode_device([1] * (k + m), [0] * (k + m), [1] * k, [0] * k, cell, 1)
    c.close()


def test_pool_acquire_without_gpu_is_host_only():
    """hec_coder_acquire(device -1) with no visible GPU hands out a host-only
    coder; release resets the host limit and ignores a double release."""
    if gpu_available():
        pytest.skip("a GPU is visible: acquire(-1) picks it")
    c = H.Coder(6, 3, -1, pooled=True)
    assert c.device == H.HEC_DEVICE_HOST
    raw = c.handle
    H.lib.hec_coder_release(raw)
    H.lib.hec_coder_release(raw)  # second release of an idle coder: ignored
    c._h = None
    a, b = H.Coder(6, 3, -1, pooled=True), H.Coder(6, 3, -1, pooled=True)
    assert a.handle.value != b.handle.value, "a double release handed one coder out twice"
    a.close()
    b.close()
    assert H.lib.hec_coder_pool_trim() >= 2


# ---- plan-time JIT (hiprtc runs on the CPU: no GPU needed to compile) -------

def test_jit_warm_compiles_and_caches(tmp_path):
    """hec_jit_warm compiles the plan-specialised decode + verify kernel with
    hiprtc into the disk cache; a second process finds it there.  Shapes:
    RS(6,3) with data 0..2 lost (8 slabs) and RS(10,4) with 4 lost (4 slabs,
    inputs in pairs), CRC32C; a plan without a fused kernel is refused."""
    import json
    import subprocess
    import sys
    code = ("import json, sys; sys.path.insert(0, %r); import hdfs_native_ec as H; "
            "H.jit_warm(6, 3, [0, 1, 2]); H.jit_warm(10, 4, [0, 1, 2, 3], 2); "
            "print(json.dumps(H.jit_stats()))") % os.path.join(ROOT, "hdfs-native_amd")
    env = dict(os.environ, HEC_JIT_CACHE=str(tmp_path))
    first = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=300)
    assert first.returncode == 0, first.stderr[-3000:]
    s1 = json.loads(first.stdout.strip().splitlines()[-1])
    assert s1["compiled"] == 2 and s1["failed"] == 0, s1
    assert len(list(tmp_path.glob("dv-*.co"))) == 2
    second = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=300)
    assert second.returncode == 0, second.stderr[-3000:]
    s2 = json.loads(second.stdout.strip().splitlines()[-1])
    assert s2["from_disk"] == 2 and s2["compiled"] == 0, s2
    # a truncated cache file (a write cut short by a full disk) fails its size
    # and checksum check and is recompiled, never loaded
    victim = sorted(tmp_path.glob("dv-*.co"))[0]
    victim.write_bytes(victim.read_bytes()[:-100])
    third = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=300)
    assert third.returncode == 0, third.stderr[-3000:]
    s3 = json.loads(third.stdout.strip().splitlines()[-1])
    assert s3["from_disk"] == 1 and s3["compiled"] == 1 and s3["failed"] == 0, s3
    with pytest.raises(ValueError):
        H.jit_warm(5, 3, [0])  # k = 5: no fused decode + verify kernel
    with pytest.raises(ValueError):
        H.jit_warm(6, 3, [6])  # only parity lost: nothing to rebuild


def test_prepare_decode_args_without_device():
    """hec_coder_prepare_decode: argument checks, and a host-only coder (no
    device kernels to specialise) is HEC_ERR_DEVICE, never a HIP call."""
    c = H.Coder(6, 3, H.HEC_DEVICE_HOST)
    present = (ctypes.c_uint8 * 9)(0, 0, 0, 1, 1, 1, 1, 1, 1)
    flag = ctypes.c_int(7)
    assert H.lib.hec_coder_prepare_decode(None, present, 2, ctypes.byref(flag)) == H.HEC_ERR_INVALID_ARG
    assert flag.value == 0
    assert H.lib.hec_coder_prepare_decode(c.handle, None, 2, None) == H.HEC_ERR_INVALID_ARG
    assert H.lib.hec_coder_prepare_decode(c.handle, present, 0, None) == H.HEC_ERR_INVALID_ARG  # NULL type
    assert H.lib.hec_coder_prepare_decode(c.handle, present, 2, ctypes.byref(flag)) == H.HEC_ERR_DEVICE
    assert flag.value == 0
    c.close()
    st = H.jit_stats()
    assert set(st) == {"compiled", "from_disk", "failed", "launches"}


def test_queue_stats_of_a_missing_device():
    """hec_queue_stats reports zeros for a device that does not exist (and,
    in this container, for every device: no GPU) without creating state."""
    for d in (-1, 4096):
        assert H.queue_stats(d) == {"streams": 0, "graph_sets": 0, "keyed_by_id": False}
