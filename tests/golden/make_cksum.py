"""Generates tests/golden/cksum_vectors.json -- known answers for CRC_32_CKSUM,
the reference's CHECKSUM_CRC32 algorithm (rust/src/hdfs/connection.rs:37,
crc 3.4.0 / crc-catalog 2.4.0, not vendored).

The outputs come from the system's POSIX `cksum` utility (coreutils), an
independent published implementation: `cksum` is CRC_32_CKSUM over the
message followed by its length as little-endian bytes (no trailing zero
bytes).  tests/test_oracle.py checks the oracle's crc32_cksum against these
vectors by appending the same length bytes.  Re-run:
  python tests/golden/make_cksum.py
"""
import json
import os
import subprocess
import sys

OUT = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(OUT))
sys.path.insert(0, os.path.join(ROOT, "hdfs-native_amd"))

from hdfs_native_ec.synth import splitmix64_bytes  # noqa: E402

LENGTHS = [0, 1, 9, 15, 16, 127, 128, 511, 512, 513, 1000, 4096]


def main() -> None:
    cases = []
    for n in LENGTHS:
        data = b"123456789" if n == 9 else splitmix64_bytes(0xC45C + n, n).tobytes()
        out = subprocess.run(["cksum"], input=data, capture_output=True, check=True).stdout.split()
        assert int(out[1]) == n
        cases.append({"hex": data.hex(), "posix_cksum": int(out[0])})
    with open(os.path.join(OUT, "cksum_vectors.json"), "w") as f:
        json.dump({"generator": "tests/golden/make_cksum.py (coreutils cksum)", "cases": cases}, f, indent=0)


if __name__ == "__main__":
    main()
