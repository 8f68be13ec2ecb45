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
PATCH = os.path.join(ROOT, "rust", "patches", "ec_mi355x.patch")
SHIM = os.path.join(ROOT, "rust", "src", "ec", "mi355x.rs")
HEADER = os.path.join(ROOT, "include", "hdfs_ec_amd.h")


@pytest.mark.skipif(not os.path.isdir(REF_EC), reason="reference checkout not present")
def test_forwarding_patch_applies_to_reference(tmp_path):
    dst = tmp_path / "rust" / "src" / "ec"
    dst.mkdir(parents=True)
    for name in ("gf256.rs", "mod.rs", "matrix.rs"):
        shutil.copy(os.path.join(REF_EC, name), dst / name)
    r = subprocess.run(["patch", "-p1", "--dry-run", "-i", PATCH], cwd=tmp_path, capture_output=True, text=True)
    assert r.returncode == 0, r.stdout + r.stderr
    r = subprocess.run(["patch", "-p1", "-i", PATCH], cwd=tmp_path, capture_output=True, text=True)
    assert r.returncode == 0
    text = (dst / "gf256.rs").read_text()
    # Coder::new acquires a pooled engine coder; encode / decode forward to it
    assert "super::mi355x::PooledCoder::acquire(\"rs\"" in text
    assert text.count('#[cfg(feature = "mi355x")]') >= 4 and text.count('#[cfg(not(feature = "mi355x"))]') == 2
    assert "pub mod mi355x;" in (dst / "mod.rs").read_text()


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
