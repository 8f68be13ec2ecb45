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
    # the striped writer: the reference CellBuffer only without the feature,
    # the row-batched one (rust/src/hdfs/ec_rows.rs) with it
    w = (hd / "block_writer.rs").read_text()
    assert "use super::ec_rows::CellBuffer;" in w
    assert w.count('#[cfg(not(feature = "mi355x"))]') == 3
    assert "pub(crate) mod ec_rows;" in (hd / "mod.rs").read_text()
    # the striped reader: read_slice batches rows into vertical stripes
    rd = (hd / "block_reader.rs").read_text()
    assert rd.count("async fn read_slice") == 2 and "async fn read_row" in rd
    assert "super::ec_rows::ROWS_PER_CALL" in rd and "pending_row: None" in rd
    # ONE copy of the reference's row loop and of its skip / trim, shared by
    # both cfg variants of read_slice ...
    assert rd.count("trying next replica") == 1
    assert rd.count("async fn read_row") == 1 and rd.count("fn skip_and_trim") == 1
    assert rd.count("Skip any bytes at the beginning") == 1
    assert rd.count("self.read_row().await?") == 2 and rd.count("self.skip_and_trim(decoded)") == 2
    # ... and current_block_start advances once per row read, inside
    # read_row, so a reader opened for a later row of a batch starts at that
    # row (replayed by tests/cpp/shim_replay.c)
    row_fn = rd[rd.index("async fn read_row"):rd.index("fn skip_and_trim")]
    assert "self.current_block_start += self.ec_schema.cell_size;" in row_fn
    assert rd.count("self.current_block_start +=") == 1
    # the module the writer hunk imports exists and uses only the
    # reference's own Coder / EcSchema API
    rows = open(os.path.join(ROOT, "rust", "src", "hdfs", "ec_rows.rs")).read()
    assert "pub(crate) const ROWS_PER_CALL" in rows and "pub(crate) struct CellBuffer" in rows
    assert "self.coder.encode(&part)" in rows


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
