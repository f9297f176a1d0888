"""Generate tests/golden/ fixtures from the REFERENCE's own HWCrc32c engine.

Run in the build container only (needs oracle/_ref/libref_hwcrc32c.so, compiled by
`make -C oracle ref` straight from /root/reference/src/common/HWCrc32c.cpp):

    python tests/golden/make_golden.py

Inputs are regenerated at test time from tests/util.splitmix_bytes (seeds below),
so only expected outputs are stored. checksum1.in / checksum2.in are the
reference's own test data files (test/data/), copied verbatim.
"""
from __future__ import annotations

import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
from util import fill_buffer, ptr, ref_lib, splitmix_bytes  # noqa: E402

SEED_LEN = 0x5EED
SEED_PKT = 0x5EED0001
SEED_BPC = 0x5EED0002


def ref_crc(lib, a: np.ndarray) -> int:
    return int(lib.ref_hw_crc32c(ptr(a) if a.nbytes else None, a.nbytes))


def ref_chunks(lib, data: np.ndarray, bpc: int) -> np.ndarray:
    n = (data.nbytes + bpc - 1) // bpc
    out = np.zeros(n, dtype=">u4")
    for i in range(n):
        out[i] = ref_crc(lib, data[i * bpc:(i + 1) * bpc])
    return out.view(np.uint8)


def main() -> None:
    lib = ref_lib()
    if lib is None:
        raise SystemExit("oracle/_ref/libref_hwcrc32c.so missing: run `make -C oracle ref` here first")

    # (1) every length 0..4096 at alignments 0..7 (TestChecksum.cpp:92-99 alignment sweep)
    buf = splitmix_bytes(4096 + 8, SEED_LEN)
    lens = np.zeros((8, 4097), dtype=np.uint32)
    for a in range(8):
        for n in range(4097):
            lens[a, n] = ref_crc(lib, buf[a:a + n])

    # (2) one 64 KiB packet (config 1: 128 x 512 B), clean / bit-flipped / short tail
    pkt = splitmix_bytes(65536, SEED_PKT)
    pkt_crc = ref_chunks(lib, pkt, 512)
    bad = pkt.copy()
    bad[77 * 512 + 100] ^= 0x08
    tail_len = 65536 - 100
    tail_crc = ref_chunks(lib, pkt[:tail_len], 512)
    tail_crc_corrupt = tail_crc.copy()
    tail_crc_corrupt[4 * 127] ^= 0xFF
    verify = {
        "clean_remote": int(lib.ref_hw_verify(ptr(pkt), 65536, 512, ptr(pkt_crc), 0)),
        "flip77_remote": int(lib.ref_hw_verify(ptr(bad), 65536, 512, ptr(pkt_crc), 0)),
        "flip77_local": int(lib.ref_hw_verify(ptr(bad), 65536, 512, ptr(pkt_crc), 1)),
        "tail_clean_local": int(lib.ref_hw_verify(ptr(pkt), tail_len, 512, ptr(tail_crc), 1)),
        "tail_corrupt_remote": int(lib.ref_hw_verify(ptr(pkt), tail_len, 512, ptr(tail_crc_corrupt), 0)),
        "tail_corrupt_local": int(lib.ref_hw_verify(ptr(pkt), tail_len, 512, ptr(tail_crc_corrupt), 1)),
    }

    # (3) per-bpc CRC arrays over a 1 MiB buffer (configs 2/3 bpc sweep, small)
    big = splitmix_bytes(1 << 20, SEED_BPC)
    bpcs = {f"bpc{b}": ref_chunks(lib, big, b) for b in (512, 2048, 4096)}

    # (4) FillBuffer pattern (mock/TestUtil.h:44-53) KATs, named in SURVEY.md §8c
    fb = {
        "off0_len512": ref_crc(lib, fill_buffer(512, 0)),
        "off512_len512": ref_crc(lib, fill_buffer(512, 512)),
        "off0_len2048": ref_crc(lib, fill_buffer(2048, 0)),
        "off0_len4096": ref_crc(lib, fill_buffer(4096, 0)),
        "str_123456789": ref_crc(lib, np.frombuffer(b"123456789", dtype=np.uint8)),
        "zeros512": ref_crc(lib, np.zeros(512, np.uint8)),
        "zeros2048": ref_crc(lib, np.zeros(2048, np.uint8)),
        "zeros4096": ref_crc(lib, np.zeros(4096, np.uint8)),
        "ff512": ref_crc(lib, np.full(512, 0xFF, np.uint8)),
    }

    np.savez_compressed(os.path.join(HERE, "ref_hwcrc32c.npz"), lengths=lens, pkt_crc=pkt_crc,
                        tail_crc=tail_crc, **bpcs)
    with open(os.path.join(HERE, "ref_hwcrc32c.json"), "w") as f:
        json.dump({"generator": "tests/golden/make_golden.py",
                   "engine": "reference src/common/HWCrc32c.cpp (compiled by oracle/Makefile ref)",
                   "seeds": {"lengths": SEED_LEN, "packet": SEED_PKT, "bpc": SEED_BPC},
                   "packet": {"flip_byte": 77 * 512 + 100, "flip_mask": 8, "tail_len": tail_len},
                   "verify": verify, "kat": fb}, f, indent=1, sort_keys=True)
    print("wrote", os.listdir(HERE))


if __name__ == "__main__":
    main()
