"""The engine's host-side GF(2^8) multiply (hdfs-native_amd/csrc/host_gf.cpp:
AVX-512BW+GFNI, AVX2, scalar), the per-call drop-in's small-row path, against
the oracle on the CPU: tests/cpp/host_gf_check.cpp runs every ISA this CPU
supports over RS encode/decode matrices and random matrices at every tail
length, and checks the affine bit matrix of every coefficient."""
import os
import subprocess

from conftest import PKG_DIR

BIN = os.path.join(PKG_DIR, "build", "host_gf_check")


def test_host_gf_every_isa_vs_oracle():
    if not os.path.exists(BIN):
        subprocess.check_call(["make", "-s", "-C", PKG_DIR, "build/host_gf_check"])
    out = subprocess.run([BIN], capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stderr[-4000:]
    assert "host gf ok" in out.stdout


BSL_BIN = os.path.join(PKG_DIR, "build", "bitslice_check")


def test_bitslice_networks_vs_oracle():
    """The fused encode kernel's bit-sliced parity (8x8 bit transpose +
    generated XOR networks) equals the oracle's RS parity, per byte."""
    subprocess.check_call(["make", "-s", "-C", PKG_DIR, "build/bitslice_check"])
    out = subprocess.run([BSL_BIN], capture_output=True, text=True, timeout=120)
    assert out.returncode == 0, out.stderr[-4000:]
    assert "ok" in out.stdout


NET_BIN = os.path.join(PKG_DIR, "build", "xor_net_check")


def test_plan_time_xor_networks_every_decode_plan():
    """The networks the JIT-specialised decode + verify kernel runs
    (csrc/xor_net.hpp): every decode plan of RS(3,2), RS(6,3) and RS(10,4)
    and random 1..4-row matrices, evaluated on bit-sliced cells on the host,
    equal the oracle's decode / multiply."""
    subprocess.check_call(["make", "-s", "-C", PKG_DIR, "build/xor_net_check"])
    out = subprocess.run([NET_BIN], capture_output=True, text=True, timeout=120)
    assert out.returncode == 0, out.stdout[-4000:] + out.stderr[-4000:]
    assert "xor net ok" in out.stdout
