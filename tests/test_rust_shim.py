"""The Rust side of the drop-in (no cargo in this image, so it is checked
as text): the forwarding patch applies to the reference's EC sources, and
the shim's FFI declarations name only functions the C ABI header declares,
at the header's ABI version."""
import os
import re
import shutil
import subprocess

import pytest

from conftest import ROOT

REF_EC = "/root/reference/rust/src/ec"
REF_HDFS = "/root/reference/rust/src/hdfs"
REF_BENCH = "/root/reference/rust/benches/ec.rs"
PATCH = os.path.join(ROOT, "rust", "patches", "ec_mi355x.patch")
SHIM = os.path.join(ROOT, "rust", "src", "ec", "mi355x.rs")
HEADER = os.path.join(ROOT, "include", "hdfs_ec_amd.h")


@pytest.mark.skipif(not os.path.isdir(REF_EC), reason="reference checkout not present")
def test_forwarding_patch_applies_to_reference(tmp_path):
    ec = tmp_path / "rust" / "src" / "ec"
    hd = tmp_path / "rust" / "src" / "hdfs"
    ec.mkdir(parents=True)
    hd.mkdir(parents=True)
    for name in ("gf256.rs", "mod.rs", "matrix.rs"):
        shutil.copy(os.path.join(REF_EC, name), ec / name)
    for name in ("mod.rs", "block_writer.rs", "block_reader.rs"):
        shutil.copy(os.path.join(REF_HDFS, name), hd / name)
    (tmp_path / "rust" / "benches").mkdir()
    shutil.copy(REF_BENCH, tmp_path / "rust" / "benches" / "ec.rs")
    r = subprocess.run(["patch", "-p1", "--dry-run", "-i", PATCH], cwd=tmp_path, capture_output=True, text=True)
    assert r.returncode == 0, r.stdout + r.stderr
    r = subprocess.run(["patch", "-p1", "-i", PATCH], cwd=tmp_path, capture_output=True, text=True)
    assert r.returncode == 0
    text = (ec / "gf256.rs").read_text()
    # Coder::new acquires a pooled engine coder (None -> the reference CPU
    # path, kept unchanged); encode / decode forward to it when present
    assert "gpu: Option<super::mi355x::PooledCoder>" in text
    assert "super::mi355x::PooledCoder::acquire(\"rs\"" in text and ".ok()," in text
    assert text.count("if let Some(gpu) = self.gpu.as_ref()") == 2
    assert '#[cfg(not(feature = "mi355x"))]' not in text  # the CPU bodies stay in both builds
    assert "pub mod mi355x;" in (ec / "mod.rs").read_text()
    # the striped writer and reader are the reference's, unchanged: they code
    # one row per Coder call (block_writer.rs:838, ec/mod.rs:71-72) and the
    # engine routes those pageable rows to its host routine -- the 4-row
    # batching of round 4 is gone (measured, the device route
    # lost at both call shapes, and 4 rows bought the host routine +8 % on
    # encode for 4x the writer's buffer)
    for name in ("mod.rs", "block_writer.rs", "block_reader.rs"):
        assert (hd / name).read_text() == open(os.path.join(REF_HDFS, name)).read(), name
    patched = {ln[6:].strip() for ln in open(PATCH) if ln.startswith("+++ b/")}
    assert patched == {"rust/src/ec/gf256.rs", "rust/src/ec/mod.rs", "rust/benches/ec.rs"}, patched
    # the reference's Criterion bench gains a device-resident group (features
    # benchmark + mi355x) beside its own, which stays as it was: the same
    # 6 x 16 MiB slices, encode and decode 1 / 2 / 3 missing through GpuCoder
    bench = (tmp_path / "rust" / "benches" / "ec.rs").read_text()
    ref = open(REF_BENCH).read()
    assert bench.startswith(ref[:ref.index("criterion_group!")])
    assert "fn bench_mi355x(c: &mut Criterion)" in bench
    assert 'benchmark_group("rs-encode-mi355x")' in bench and 'benchmark_group("rs-decode-mi355x")' in bench
    assert "coder.encode_device(" in bench and "coder.decode_device(" in bench
    assert "criterion_group!(benches, bench, bench_mi355x);" in bench
    assert '#[cfg(not(feature = "mi355x"))]\ncriterion_group!(benches, bench);' in bench
    assert not os.path.exists(os.path.join(ROOT, "rust", "src", "hdfs", "ec_rows.rs"))


def test_shim_ffi_matches_header():
    header = re.sub(r"/\*.*?\*/", "", open(HEADER).read(), flags=re.S)
    declared = set(re.findall(r"\b(hec_[a-z_0-9]+)\s*\(", header))
    shim = open(SHIM).read()
    ffi = shim[shim.index('unsafe extern "C" {'):]
    ffi = ffi[:ffi.index("\n}\n")]
    used = set(re.findall(r"fn (hec_[a-z_0-9]+)\(", ffi))
    assert used and used <= declared, used - declared
    abi = int(re.search(r"#define HEC_ABI_VERSION (\d+)", header).group(1))
    assert f"const ABI_VERSION: c_int = {abi};" in shim
