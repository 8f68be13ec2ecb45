import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG_DIR = os.path.join(ROOT, "hdfs-native_amd")
ORACLE_DIR = os.path.join(ROOT, "oracle")
for p in (PKG_DIR, ORACLE_DIR, ROOT):
    if p not in sys.path:
        sys.path.insert(0, p)


def _ensure_built() -> None:
    """Build the oracle (C) and the HIP library in-tree if a fresh checkout
    lacks them (hipcc cross-compiles without a GPU)."""
    if not os.path.exists(os.path.join(ORACLE_DIR, "build", "liboracle_ec.so")):
        subprocess.check_call(["make", "-s", "-C", ORACLE_DIR])
    if not os.path.exists(os.path.join(PKG_DIR, "lib", "libhdfs_ec_amd.so")):
        subprocess.check_call(["make", "-s", "-j4", "-C", PKG_DIR])


_ensure_built()


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs on the GPU box)")


def gpu_available() -> bool:
    try:
        import torch
        return torch.cuda.is_available()
    except Exception:
        return False


@pytest.fixture(scope="session")
def golden():
    import json

    import numpy as np
    d = os.path.join(ROOT, "tests", "golden")
    with open(os.path.join(d, "ec_vectors.json")) as f:
        manifest = json.load(f)
    arrays = np.load(os.path.join(d, "ec_vectors.npz"), allow_pickle=False)
    return manifest, arrays


@pytest.fixture(scope="session")
def c_oracle():
    import ec_oracle
    return ec_oracle.load_c_oracle()
