"""The round kernel's lane-fold image, checked on the host (CPU suite): tests/native/fold_image.cpp
restates one 4 KiB round of the kernel's arithmetic (64-byte lane segments, chained slice-by-4 steps
from 0, lane-specific nibble fold entries, xor over a chunk's lanes) and compares every chunk with the
byte-at-a-time SWCrc32c loop (src/common/SWCrc32c.cpp:97-104), for G = 8 / 16 / 32 / 64, both
polynomials (CRC32C and the CRC-32 of CHECKSUM_CRC32), and both image forms: round 5's, whose
entries carry each chain's last table step (build_fold_nibbles_pre), and round 4's (lab 157)."""
import os
import subprocess

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_fold_image_matches_sw_crc(tmp_path):
    exe = tmp_path / "fold_image"
    subprocess.run(["g++", "-std=c++17", "-O2", "-I", os.path.join(REPO, "libhdfs3_amd", "csrc"),
                    os.path.join(REPO, "tests", "native", "fold_image.cpp"), "-o", str(exe)], check=True)
    out = subprocess.run([str(exe)], capture_output=True, text=True, timeout=120)
    assert out.returncode == 0, out.stdout[-2000:] + out.stderr[-2000:]
    assert "fold image ok" in out.stdout
